// Attention-side memory-bound kernels for CDNA4:
//  * rotary_split: fused QKV layout transform + rotary embedding + query pre-scaling
//    (GPT-NeoX layout [B,S,heads,3*hd] -> q,k,v each [B,heads,S,hd]); and its backward.
//    Reference analogues: bias_add_transform_0213 / transform4d_0213
//    (csrc/transformer/transform_kernels.cu:161-560), extended with NeoX partial rotary.
//  * scaled masked softmax fwd/bwd over score rows (reference attn_softmax /
//    softmax_backward_kernel, csrc/transformer/softmax_kernels.cu:9-580) with causal,
//    additive-mask and key-padding variants; rows held in registers, one 256-thread
//    block per row, wave64 reductions (the reference is warp32 and capped at S<8192).
#include "../include/dsa_common.h"
#include "../include/launchers.h"

namespace dsa {

// --------------------------------------------------------------------------------------
// rotary_split forward. One thread per 8-element vector of the [B,S,heads,3*hd] input.
// cs: [S, rot/2] float2 table (cos, sin) for positions 0..S-1 (+ pos_offset).
// --------------------------------------------------------------------------------------
template <typename T>
__global__ void __launch_bounds__(256) rotary_split_fwd_kernel(const T* __restrict__ qkv, T* __restrict__ q,
                                                               T* __restrict__ k, T* __restrict__ v,
                                                               const float2* __restrict__ cs, int B, int S,
                                                               int NH, int HD, int ROT, float qscale) {
  const int vec_per_item = 3 * HD / 8;
  const int64_t total = (int64_t)B * S * NH * vec_per_item;
  const int half = ROT / 2;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int vi = (int)(t % vec_per_item);
    const int64_t item = t / vec_per_item;  // (b, s, h)
    const int h = (int)(item % NH);
    const int s = (int)((item / NH) % S);
    const int b = (int)(item / ((int64_t)NH * S));
    const int e0 = vi * 8;                // element within 3*hd
    const int which = e0 / HD;            // 0=q 1=k 2=v
    const int d0 = e0 - which * HD;       // element within hd (vector never straddles: HD % 8 == 0)
    const T* src = qkv + item * 3 * HD;
    float x[8];
    Vec16<T>::load(src + e0, x);
    if (which < 2 && d0 < ROT) {
      float o[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int d = d0 + j;
        if (d < ROT) {
          const int i = d < half ? d : d - half;
          const float2 c = cs[(int64_t)s * half + i];
          const int pd = d < half ? d + half : d - half;
          const float partner = Conv<T>::load(src, which * HD + pd);
          o[j] = d < half ? x[j] * c.x - partner * c.y : x[j] * c.x + partner * c.y;
        } else {
          o[j] = x[j];
        }
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) x[j] = o[j];
    }
    if (which == 0) {
#pragma unroll
      for (int j = 0; j < 8; ++j) x[j] *= qscale;
    }
    T* dst = which == 0 ? q : (which == 1 ? k : v);
    const int64_t off = (((int64_t)b * NH + h) * S + s) * HD + d0;
    Vec16<T>::store(dst + off, x);
  }
}

// backward: dq,dk,dv [B,heads,S,hd] -> dqkv [B,S,heads,3*hd] (inverse rotation, q scale)
template <typename T>
__global__ void __launch_bounds__(256) rotary_split_bwd_kernel(const T* __restrict__ dq, const T* __restrict__ dk,
                                                               const T* __restrict__ dv, T* __restrict__ dqkv,
                                                               const float2* __restrict__ cs, int B, int S,
                                                               int NH, int HD, int ROT, float qscale) {
  const int vec_per_item = 3 * HD / 8;
  const int64_t total = (int64_t)B * S * NH * vec_per_item;
  const int half = ROT / 2;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int vi = (int)(t % vec_per_item);
    const int64_t item = t / vec_per_item;
    const int h = (int)(item % NH);
    const int s = (int)((item / NH) % S);
    const int b = (int)(item / ((int64_t)NH * S));
    const int e0 = vi * 8;
    const int which = e0 / HD;
    const int d0 = e0 - which * HD;
    const T* src = which == 0 ? dq : (which == 1 ? dk : dv);
    const int64_t off = (((int64_t)b * NH + h) * S + s) * HD;
    float g[8];
    Vec16<T>::load(src + off + d0, g);
    const float sc = which == 0 ? qscale : 1.f;
    if (which < 2 && d0 < ROT) {
      float o[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int d = d0 + j;
        if (d < ROT) {
          const int i = d < half ? d : d - half;
          const float2 c = cs[(int64_t)s * half + i];
          const int pd = d < half ? d + half : d - half;
          const float gp = Conv<T>::load(src + off, pd);
          // y1 = x1 c - x2 s ; y2 = x2 c + x1 s  =>  dx1 = dy1 c + dy2 s ; dx2 = dy2 c - dy1 s
          o[j] = d < half ? g[j] * c.x + gp * c.y : g[j] * c.x - gp * c.y;
        } else {
          o[j] = g[j];
        }
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) g[j] = o[j];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) g[j] *= sc;
    Vec16<T>::store(dqkv + item * 3 * HD + e0, g);
  }
}

// Row form of rotary_split for the common (head_dim, rotary_dim) pairs: one thread per
// (b, s, head, q|k|v) row of HD elements, the row held in registers so the rotate-half
// partner is a compile-time register (no partner reloads, no 64-bit index math per element).
// Consecutive threads read consecutive HD-element pieces of the qkv row (fully used 16-B
// loads); each thread writes one contiguous HD-element row of q, k or v.
template <typename T, int HD, int ROT>
__global__ void __launch_bounds__(256) rotary_split_fwd_row_kernel(const T* __restrict__ qkv, T* __restrict__ q,
                                                                   T* __restrict__ k, T* __restrict__ v,
                                                                   const float2* __restrict__ cs, int rows, int S,
                                                                   int NH, float qscale) {
  constexpr int NVEC = HD / 8;
  constexpr int HALF = ROT / 2;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= rows * 3) return;
  const int which = t % 3;
  const int item = t / 3;  // (b, s, h)
  const int h = item % NH;
  const int bs = item / NH;
  const int s = bs % S;
  const int b = bs / S;
  const T* src = qkv + (int64_t)t * HD;
  float x[NVEC][8];
#pragma unroll
  for (int i = 0; i < NVEC; ++i) Vec16<T>::load(src + 8 * i, x[i]);
  if (ROT > 0 && which < 2) {
    const float2* c = cs + (int64_t)s * HALF;
#pragma unroll
    for (int i = 0; i < HALF; ++i) {
      const float2 cc = c[i];
      const float a = x[i / 8][i % 8], p = x[(i + HALF) / 8][(i + HALF) % 8];
      x[i / 8][i % 8] = a * cc.x - p * cc.y;
      x[(i + HALF) / 8][(i + HALF) % 8] = p * cc.x + a * cc.y;
    }
  }
  if (which == 0) {
#pragma unroll
    for (int i = 0; i < NVEC; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) x[i][j] *= qscale;
  }
  T* dst = (which == 0 ? q : (which == 1 ? k : v)) + (((int64_t)b * NH + h) * S + s) * HD;
#pragma unroll
  for (int i = 0; i < NVEC; ++i) Vec16<T>::store(dst + 8 * i, x[i]);
}

template <typename T, int HD, int ROT>
__global__ void __launch_bounds__(256) rotary_split_bwd_row_kernel(const T* __restrict__ dq, const T* __restrict__ dk,
                                                                   const T* __restrict__ dv, T* __restrict__ dqkv,
                                                                   const float2* __restrict__ cs, int rows, int S,
                                                                   int NH, float qscale) {
  constexpr int NVEC = HD / 8;
  constexpr int HALF = ROT / 2;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= rows * 3) return;
  const int which = t % 3;
  const int item = t / 3;
  const int h = item % NH;
  const int bs = item / NH;
  const int s = bs % S;
  const int b = bs / S;
  const T* src = (which == 0 ? dq : (which == 1 ? dk : dv)) + (((int64_t)b * NH + h) * S + s) * HD;
  float g[NVEC][8];
#pragma unroll
  for (int i = 0; i < NVEC; ++i) Vec16<T>::load(src + 8 * i, g[i]);
  if (ROT > 0 && which < 2) {
    const float2* c = cs + (int64_t)s * HALF;
    // y1 = x1 c - x2 s ; y2 = x2 c + x1 s  =>  dx1 = dy1 c + dy2 s ; dx2 = dy2 c - dy1 s
#pragma unroll
    for (int i = 0; i < HALF; ++i) {
      const float2 cc = c[i];
      const float a = g[i / 8][i % 8], p = g[(i + HALF) / 8][(i + HALF) % 8];
      g[i / 8][i % 8] = a * cc.x + p * cc.y;
      g[(i + HALF) / 8][(i + HALF) % 8] = p * cc.x - a * cc.y;
    }
  }
  if (which == 0) {
#pragma unroll
    for (int i = 0; i < NVEC; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) g[i][j] *= qscale;
  }
  T* dst = dqkv + (int64_t)t * HD;
#pragma unroll
  for (int i = 0; i < NVEC; ++i) Vec16<T>::store(dst + 8 * i, g[i]);
}

// LDS-tiled rotary split: one workgroup per (b, 16 positions, 4 heads).  The QKV projection
// output is read as its [s][h][which] runs (2.3 KB contiguous at HD 96) and q/k/v are written
// as [which][h][s] runs (3 KB contiguous), both with one 16-byte chunk per lane per instruction;
// the row-per-thread kernels above make every lane walk its own 192-byte row, which spreads each
// load/store instruction over 64 separate cache lines (3.2 TB/s on the 20B shapes).  BWD runs the
// same tile the other way round (dq/dk/dv -> dqkv with the inverse rotation).
constexpr int ROT_SB = 16, ROT_HB = 4;
constexpr int which_chunks(int hd, int rot) { return hd / 8 > (rot + 7) / 8 ? hd / 8 : (rot + 7) / 8; }

template <typename T, int HD, int ROT, bool BWD, bool PAD = true>
__global__ void __launch_bounds__(256) rotary_split_tiled_kernel(const T* __restrict__ qkv_in, T* __restrict__ qkv_out,
                                                                 const T* __restrict__ q_in, const T* __restrict__ k_in,
                                                                 const T* __restrict__ v_in, T* __restrict__ q_out,
                                                                 T* __restrict__ k_out, T* __restrict__ v_out,
                                                                 const float2* __restrict__ cs, int S, int NH,
                                                                 float qscale) {
  constexpr int CPR = HD / 8, HALF = ROT / 2;
  constexpr int ROWS = 3 * ROT_HB * ROT_SB, CHUNKS = ROWS * CPR;
  // rows padded by 16 bytes: in the per-row rotation phase every lane walks its own row, and an
  // unpadded 256-byte row (HD 128) puts all 64 lanes' accesses on the same banks
  constexpr int HDP = PAD ? HD + 8 : HD;
  __shared__ __attribute__((aligned(16))) uint16_t tile[ROWS * HDP];  // [which][h][s][HD (+8)]
  const int tid = threadIdx.x;
  const int nsb = S / ROT_SB, nhb = NH / ROT_HB;
  const int hb = blockIdx.x % nhb, sb = (blockIdx.x / nhb) % nsb, b = blockIdx.x / (nhb * nsb);
  const int s0 = sb * ROT_SB, h0 = hb * ROT_HB;
  auto lds_off = [](int which, int hl, int sl) { return ((which * ROT_HB + hl) * ROT_SB + sl) * HDP; };
  // packed side ([B,S,NH,3,HD], GPT-NeoX's per-head interleave) chunk order: s, h, which, chunk
  auto packed_chunk = [&](int c, int& which, int& hl, int& sl, int& ch) {
    ch = c % CPR; int r = c / CPR;
    which = r % 3; r /= 3;
    hl = r % ROT_HB; sl = r / ROT_HB;
  };
  // split side ([B,NH,S,HD] x 3) chunk order: which, h, s, chunk
  auto split_chunk = [&](int c, int& which, int& hl, int& sl, int& ch) {
    ch = c % CPR; int r = c / CPR;
    sl = r % ROT_SB; r /= ROT_SB;
    hl = r % ROT_HB; which = r / ROT_HB;
  };
  // one load and its LDS store per chunk: issuing all of a thread's loads before the first store
  // (PER uint4 registers live at once) ran 28 % slower -- 188 vs 136 us on the 20B shape,
  // profiles/r6l_rotary_load_loop_ab.log -- the loop lets more workgroups' loads overlap instead
  for (int c = tid; c < CHUNKS; c += 256) {
    int which, hl, sl, ch;
    uint4 v;
    if constexpr (!BWD) {
      packed_chunk(c, which, hl, sl, ch);
      v = *reinterpret_cast<const uint4*>(qkv_in + ((((int64_t)b * S + s0 + sl) * NH + h0 + hl) * 3 + which) * HD + ch * 8);
    } else {
      split_chunk(c, which, hl, sl, ch);
      const T* src = which == 0 ? q_in : (which == 1 ? k_in : v_in);
      v = *reinterpret_cast<const uint4*>(src + (((int64_t)b * NH + h0 + hl) * S + s0 + sl) * HD + ch * 8);
    }
    *reinterpret_cast<uint4*>(tile + lds_off(which, hl, sl) + ch * 8) = v;
  }
  __syncthreads();
  if (tid < ROWS) {
    const int which = tid / (ROT_HB * ROT_SB), hl = (tid / ROT_SB) % ROT_HB, sl = tid % ROT_SB;
    if (which < 2) {
      uint16_t* row = tile + lds_off(which, hl, sl);
      constexpr int NV = which_chunks(HD, ROT);
      float x[NV][8];
      const int nv = which == 0 ? CPR : (ROT + 7) / 8;
#pragma unroll
      for (int i = 0; i < NV; ++i)
        if (i < nv) Vec16<T>::load(reinterpret_cast<const T*>(row) + 8 * i, x[i]);
      if constexpr (ROT > 0) {
        const float2* c = cs + (int64_t)(s0 + sl) * HALF;
#pragma unroll
        for (int i = 0; i < HALF; ++i) {
          const float2 cc = c[i];
          const float a = x[i / 8][i % 8], p = x[(i + HALF) / 8][(i + HALF) % 8];
          // forward: y1 = x1 c - x2 s, y2 = x2 c + x1 s; backward: the transposed rotation
          x[i / 8][i % 8] = BWD ? a * cc.x + p * cc.y : a * cc.x - p * cc.y;
          x[(i + HALF) / 8][(i + HALF) % 8] = BWD ? p * cc.x - a * cc.y : p * cc.x + a * cc.y;
        }
      }
      if (which == 0) {
#pragma unroll
        for (int i = 0; i < NV; ++i)
#pragma unroll
          for (int j = 0; j < 8; ++j) x[i][j] *= qscale;
      }
#pragma unroll
      for (int i = 0; i < NV; ++i)
        if (i < nv) Vec16<T>::store(reinterpret_cast<T*>(row) + 8 * i, x[i]);
    }
  }
  __syncthreads();
  for (int c = tid; c < CHUNKS; c += 256) {
    int which, hl, sl, ch;
    if constexpr (!BWD) split_chunk(c, which, hl, sl, ch);
    else packed_chunk(c, which, hl, sl, ch);
    const uint4 v = *reinterpret_cast<const uint4*>(tile + lds_off(which, hl, sl) + ch * 8);
    if constexpr (!BWD) {
      T* dst = which == 0 ? q_out : (which == 1 ? k_out : v_out);
      *reinterpret_cast<uint4*>(dst + (((int64_t)b * NH + h0 + hl) * S + s0 + sl) * HD + ch * 8) = v;
    } else {
      *reinterpret_cast<uint4*>(qkv_out + ((((int64_t)b * S + s0 + sl) * NH + h0 + hl) * 3 + which) * HD + ch * 8) = v;
    }
  }
}

// (HD, ROT) pairs of the GPT-NeoX / GPT-3 presets; anything else takes the vector kernels.
#define DSA_ROTARY_ROW_CASES(X) X(64, 16) X(64, 64) X(80, 20) X(96, 24) X(96, 96) X(128, 32) X(128, 64) X(128, 128)

// --------------------------------------------------------------------------------------
// Softmax over rows of scores [R, C] with row r belonging to query position
// q = r % Sq (causal: keys > q + (C - Sq) masked). Optional additive mask [Bm, Sq, C]
// broadcast over heads (mask row = (r / (heads*Sq)) * Sq + q when mask_batch > 0).
// y = softmax(scale * x + mask). Rows processed one per 256-thread block.
// --------------------------------------------------------------------------------------
template <typename T, int NV>
__global__ void __launch_bounds__(256) softmax_fwd_kernel(const T* __restrict__ x, T* __restrict__ y,
                                                          const T* __restrict__ mask, int64_t R, int C, int Sq,
                                                          int heads, float scale, int causal, int mask_rows) {
  __shared__ float red[32];
  constexpr int VN = 8;
  const int64_t r = blockIdx.x;
  const int q = (int)(r % Sq);
  const int limit = causal ? q + (C - Sq) + 1 : C;  // valid keys [0, limit)
  const T* xr = x + r * C;
  const T* mr = nullptr;
  if (mask) {
    const int64_t bidx = r / ((int64_t)heads * Sq);
    mr = mask + (bidx * mask_rows + (mask_rows == 1 ? 0 : q)) * (int64_t)C;  // [B,1,1|Sq,C]
  }
  float vals[NV][VN];
  float mx = -INFINITY;
#pragma unroll
  for (int kk = 0; kk < NV; ++kk) {
    const int c0 = (threadIdx.x + kk * 256) * VN;
    if (c0 < C) {
      Vec16<T>::load(xr + c0, vals[kk]);
      float mv[VN];
      if (mr) Vec16<T>::load(mr + c0, mv);
#pragma unroll
      for (int j = 0; j < VN; ++j) {
        float s = vals[kk][j] * scale + (mr ? mv[j] : 0.f);
        if (c0 + j >= limit) s = -INFINITY;
        vals[kk][j] = s;
        mx = fmaxf(mx, s);
      }
    } else {
#pragma unroll
      for (int j = 0; j < VN; ++j) vals[kk][j] = -INFINITY;
    }
  }
  // block max
  mx = wave_max(mx);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = mx;
  __syncthreads();
  mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  __syncthreads();
  float sum = 0.f;
#pragma unroll
  for (int kk = 0; kk < NV; ++kk)
#pragma unroll
    for (int j = 0; j < VN; ++j) {
      const float e = (vals[kk][j] == -INFINITY || mx == -INFINITY) ? 0.f : __expf(vals[kk][j] - mx);
      vals[kk][j] = e;
      sum += e;
    }
  sum = block_sum(sum, red);
  const float inv = sum > 0.f ? 1.f / sum : 0.f;
#pragma unroll
  for (int kk = 0; kk < NV; ++kk) {
    const int c0 = (threadIdx.x + kk * 256) * VN;
    if (c0 < C) {
      float o[VN];
#pragma unroll
      for (int j = 0; j < VN; ++j) o[j] = vals[kk][j] * inv;
      Vec16<T>::store(y + r * C + c0, o);
    }
  }
}

// dx = scale * y * (dy - sum(dy*y))
template <typename T, int NV>
__global__ void __launch_bounds__(256) softmax_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ y,
                                                          T* __restrict__ dx, int64_t R, int C, float scale) {
  __shared__ float red[32];
  constexpr int VN = 8;
  const int64_t r = blockIdx.x;
  float yv[NV][VN], gv[NV][VN];
  float dot = 0.f;
#pragma unroll
  for (int kk = 0; kk < NV; ++kk) {
    const int c0 = (threadIdx.x + kk * 256) * VN;
    if (c0 < C) {
      Vec16<T>::load(y + r * C + c0, yv[kk]);
      Vec16<T>::load(dy + r * C + c0, gv[kk]);
#pragma unroll
      for (int j = 0; j < VN; ++j) dot = fmaf(yv[kk][j], gv[kk][j], dot);
    }
  }
  dot = block_sum(dot, red);
#pragma unroll
  for (int kk = 0; kk < NV; ++kk) {
    const int c0 = (threadIdx.x + kk * 256) * VN;
    if (c0 < C) {
      float o[VN];
#pragma unroll
      for (int j = 0; j < VN; ++j) o[j] = scale * yv[kk][j] * (gv[kk][j] - dot);
      Vec16<T>::store(dx + r * C + c0, o);
    }
  }
}

// Short rows (C <= 4096, the BERT / sparse-block regime): a row is owned by a group of G lanes
// inside one wave (G = C/8 rounded up to a power of two, <= 64; each lane holds NV x 8
// elements), 256/G rows per block, reductions are in-wave xor shuffles over the group with no
// LDS and no barrier.  The one-row-per-block kernels above leave 15/16 of the block idle at
// C = 128 (0.2 TB/s measured for BERT-Large scores [64,16,128,128]).
template <int G>
__device__ __forceinline__ float group_max(float v) {
#pragma unroll
  for (int o = G / 2; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
}
template <int G>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
  for (int o = G / 2; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

template <typename T, int G, int NV>
__global__ void __launch_bounds__(256) softmax_fwd_rows_kernel(const T* __restrict__ x, T* __restrict__ y,
                                                               const T* __restrict__ mask, int64_t R, int C, int Sq,
                                                               int heads, float scale, int causal, int mask_rows) {
  constexpr int VN = 8;
  const int lane_g = threadIdx.x % G;
  const int64_t r = (int64_t)blockIdx.x * (256 / G) + threadIdx.x / G;
  const bool live = r < R;  // dead rows still join the shuffles (full EXEC), write nothing
  const int64_t rr = live ? r : R - 1;
  const int q = (int)(rr % Sq);
  const int limit = causal ? q + (C - Sq) + 1 : C;
  const T* xr = x + rr * C;
  const T* mr = nullptr;
  if (mask) {
    const int64_t bidx = rr / ((int64_t)heads * Sq);
    mr = mask + (bidx * mask_rows + (mask_rows == 1 ? 0 : q)) * (int64_t)C;
  }
  float vals[NV][VN];
  float mx = -INFINITY;
#pragma unroll
  for (int kk = 0; kk < NV; ++kk) {
    const int c0 = (lane_g + kk * G) * VN;
    if (c0 < C) {
      Vec16<T>::load(xr + c0, vals[kk]);
      float mv[VN];
      if (mr) Vec16<T>::load(mr + c0, mv);
#pragma unroll
      for (int j = 0; j < VN; ++j) {
        float sv = vals[kk][j] * scale + (mr ? mv[j] : 0.f);
        if (c0 + j >= limit) sv = -INFINITY;
        vals[kk][j] = sv;
        mx = fmaxf(mx, sv);
      }
    } else {
#pragma unroll
      for (int j = 0; j < VN; ++j) vals[kk][j] = -INFINITY;
    }
  }
  mx = group_max<G>(mx);
  float sum = 0.f;
#pragma unroll
  for (int kk = 0; kk < NV; ++kk)
#pragma unroll
    for (int j = 0; j < VN; ++j) {
      const float e = (vals[kk][j] == -INFINITY || mx == -INFINITY) ? 0.f : __expf(vals[kk][j] - mx);
      vals[kk][j] = e;
      sum += e;
    }
  sum = group_sum<G>(sum);
  const float inv = sum > 0.f ? 1.f / sum : 0.f;
  if (!live) return;
#pragma unroll
  for (int kk = 0; kk < NV; ++kk) {
    const int c0 = (lane_g + kk * G) * VN;
    if (c0 < C) {
      float o[VN];
#pragma unroll
      for (int j = 0; j < VN; ++j) o[j] = vals[kk][j] * inv;
      Vec16<T>::store(y + r * C + c0, o);
    }
  }
}

template <typename T, int G, int NV>
__global__ void __launch_bounds__(256) softmax_bwd_rows_kernel(const T* __restrict__ dy, const T* __restrict__ y,
                                                               T* __restrict__ dx, int64_t R, int C, float scale) {
  constexpr int VN = 8;
  const int lane_g = threadIdx.x % G;
  const int64_t r = (int64_t)blockIdx.x * (256 / G) + threadIdx.x / G;
  const bool live = r < R;
  const int64_t rr = live ? r : R - 1;
  float yv[NV][VN], gv[NV][VN];
  float dot = 0.f;
#pragma unroll
  for (int kk = 0; kk < NV; ++kk) {
    const int c0 = (lane_g + kk * G) * VN;
    if (c0 < C) {
      Vec16<T>::load(y + rr * C + c0, yv[kk]);
      Vec16<T>::load(dy + rr * C + c0, gv[kk]);
#pragma unroll
      for (int j = 0; j < VN; ++j) dot = fmaf(yv[kk][j], gv[kk][j], dot);
    }
  }
  dot = group_sum<G>(dot);
  if (!live) return;
#pragma unroll
  for (int kk = 0; kk < NV; ++kk) {
    const int c0 = (lane_g + kk * G) * VN;
    if (c0 < C) {
      float o[VN];
#pragma unroll
      for (int j = 0; j < VN; ++j) o[j] = scale * yv[kk][j] * (gv[kk][j] - dot);
      Vec16<T>::store(dx + r * C + c0, o);
    }
  }
}

// (G, NV) for a row of C columns (C % 8 == 0): G lanes x NV x 8 elements >= C, or 0 when the
// row is long enough for the one-row-per-block kernels
static inline bool softmax_rows_shape(int C, int& G, int& NV) {
  const int chunks = C / 8;
  if (chunks <= 0 || C % 8 != 0 || chunks > 512) return false;
  G = 8;
  while (G < chunks && G < 64) G <<= 1;
  NV = (chunks + G - 1) / G;
  NV = NV <= 1 ? 1 : NV <= 2 ? 2 : NV <= 4 ? 4 : 8;
  return true;
}

#define DSA_SOFTMAX_ROWS(G_, NV_, KERNEL, ...)                                                      \
  switch (G_ * 16 + NV_) {                                                                          \
    case 8 * 16 + 1: { constexpr int GG = 8, VV = 1; __VA_ARGS__; } break;                         \
    case 16 * 16 + 1: { constexpr int GG = 16, VV = 1; __VA_ARGS__; } break;                       \
    case 32 * 16 + 1: { constexpr int GG = 32, VV = 1; __VA_ARGS__; } break;                       \
    case 64 * 16 + 1: { constexpr int GG = 64, VV = 1; __VA_ARGS__; } break;                       \
    case 64 * 16 + 2: { constexpr int GG = 64, VV = 2; __VA_ARGS__; } break;                       \
    case 64 * 16 + 4: { constexpr int GG = 64, VV = 4; __VA_ARGS__; } break;                       \
    default: { constexpr int GG = 64, VV = 8; __VA_ARGS__; } break;                                \
  }

// --------------------------------------------------------------------------------------

#define DSA_DISPATCH_SNV(nv, NV, ...)                                \
  switch (nv) {                                                      \
    case 1: { constexpr int NV = 1; __VA_ARGS__; } break;            \
    case 2: { constexpr int NV = 2; __VA_ARGS__; } break;            \
    case 3: case 4: { constexpr int NV = 4; __VA_ARGS__; } break;    \
    case 5: case 6: case 7: case 8: { constexpr int NV = 8; __VA_ARGS__; } break; \
    default: { constexpr int NV = 16; __VA_ARGS__; } break;          \
  }

static int elem_grid(int64_t work) {
  int64_t g = (work + 255) / 256;
  if (g > 16384) g = 16384;
  return (int)(g < 1 ? 1 : g);
}

void launch_rotary_split_fwd(const void* qkv, void* q, void* k, void* v, const float* cs, int B, int S, int NH,
                             int HD, int ROT, float qscale, int dt, hipStream_t s) {
  const int rows = B * S * NH;
  const int grid = (rows * 3 + 255) / 256;
  const bool tiled = S % ROT_SB == 0 && NH % ROT_HB == 0;
#define DSA_ROT_TILED_FWD(hd, rot)                                                                             \
  if (tiled && HD == hd && ROT == rot) {                                                                       \
    DSA_DISPATCH_16(dt, T,                                                                                     \
        hipLaunchKernelGGL((rotary_split_tiled_kernel<T, hd, rot, false>), dim3(B * (S / ROT_SB) * (NH / ROT_HB)), \
                           dim3(256), 0, s, (const T*)qkv, nullptr, nullptr, nullptr, nullptr, (T*)q, (T*)k, (T*)v, (const float2*)cs, S, NH, qscale));                                                    \
    return;                                                                                                    \
  }
  DSA_ROTARY_ROW_CASES(DSA_ROT_TILED_FWD)
#undef DSA_ROT_TILED_FWD
#define DSA_ROT_FWD(hd, rot)                                                                                   \
  if (HD == hd && ROT == rot) {                                                                                \
    DSA_DISPATCH_16(dt, T,                                                                                     \
      hipLaunchKernelGGL((rotary_split_fwd_row_kernel<T, hd, rot>), dim3(grid), dim3(256), 0, s, (const T*)qkv, \
                         (T*)q, (T*)k, (T*)v, (const float2*)cs, rows, S, NH, qscale));                        \
    return;                                                                                                    \
  }
  if ((int64_t)rows * 3 < (1LL << 31)) { DSA_ROTARY_ROW_CASES(DSA_ROT_FWD) }
#undef DSA_ROT_FWD
  const int64_t work = (int64_t)B * S * NH * 3 * HD / 8;
  DSA_DISPATCH_16(dt, T,
    hipLaunchKernelGGL((rotary_split_fwd_kernel<T>), dim3(elem_grid(work)), dim3(256), 0, s, (const T*)qkv, (T*)q,
                       (T*)k, (T*)v, (const float2*)cs, B, S, NH, HD, ROT, qscale));
}

void launch_rotary_split_bwd(const void* dq, const void* dk, const void* dv, void* dqkv, const float* cs, int B,
                             int S, int NH, int HD, int ROT, float qscale, int dt, hipStream_t s) {
  const int rows = B * S * NH;
  const int grid = (rows * 3 + 255) / 256;
  const bool tiled = S % ROT_SB == 0 && NH % ROT_HB == 0;
#define DSA_ROT_TILED_BWD(hd, rot)                                                                             \
  if (tiled && HD == hd && ROT == rot) {                                                                       \
    DSA_DISPATCH_16(dt, T,                                                                                     \
        hipLaunchKernelGGL((rotary_split_tiled_kernel<T, hd, rot, true>), dim3(B * (S / ROT_SB) * (NH / ROT_HB)), \
                           dim3(256), 0, s, nullptr, (T*)dqkv, (const T*)dq, (const T*)dk, (const T*)dv, nullptr, nullptr, nullptr, (const float2*)cs, S, NH, qscale));                                                    \
    return;                                                                                                    \
  }
  DSA_ROTARY_ROW_CASES(DSA_ROT_TILED_BWD)
#undef DSA_ROT_TILED_BWD
#define DSA_ROT_BWD(hd, rot)                                                                                   \
  if (HD == hd && ROT == rot) {                                                                                \
    DSA_DISPATCH_16(dt, T,                                                                                     \
      hipLaunchKernelGGL((rotary_split_bwd_row_kernel<T, hd, rot>), dim3(grid), dim3(256), 0, s, (const T*)dq,  \
                         (const T*)dk, (const T*)dv, (T*)dqkv, (const float2*)cs, rows, S, NH, qscale));       \
    return;                                                                                                    \
  }
  if ((int64_t)rows * 3 < (1LL << 31)) { DSA_ROTARY_ROW_CASES(DSA_ROT_BWD) }
#undef DSA_ROT_BWD
  const int64_t work = (int64_t)B * S * NH * 3 * HD / 8;
  DSA_DISPATCH_16(dt, T,
    hipLaunchKernelGGL((rotary_split_bwd_kernel<T>), dim3(elem_grid(work)), dim3(256), 0, s, (const T*)dq,
                       (const T*)dk, (const T*)dv, (T*)dqkv, (const float2*)cs, B, S, NH, HD, ROT, qscale));
}

int softmax_max_cols() { return 16 * 256 * 8; }

void launch_softmax_fwd(const void* x, void* y, const void* mask, int64_t R, int C, int Sq, int heads, float scale,
                        int causal, int mask_rows, int dt, hipStream_t s) {
  if (R <= 0) return;
  int G, NVr;
  if (softmax_rows_shape(C, G, NVr)) {
    const unsigned grid = (unsigned)((R + 256 / G - 1) / (256 / G));
    DSA_DISPATCH_16(dt, T, DSA_SOFTMAX_ROWS(G, NVr, 0,
      hipLaunchKernelGGL((softmax_fwd_rows_kernel<T, GG, VV>), dim3(grid), dim3(256), 0, s, (const T*)x, (T*)y,
                         (const T*)mask, R, C, Sq, heads, scale, causal, mask_rows)));
    return;
  }
  const int nv = (C / 8 + 255) / 256;
  DSA_DISPATCH_16(dt, T, DSA_DISPATCH_SNV(nv, NV,
    hipLaunchKernelGGL((softmax_fwd_kernel<T, NV>), dim3((unsigned)R), dim3(256), 0, s, (const T*)x, (T*)y,
                       (const T*)mask, R, C, Sq, heads, scale, causal, mask_rows)));
}

void launch_softmax_bwd(const void* dy, const void* y, void* dx, int64_t R, int C, float scale, int dt,
                        hipStream_t s) {
  if (R <= 0) return;
  int G, NVr;
  if (softmax_rows_shape(C, G, NVr)) {
    const unsigned grid = (unsigned)((R + 256 / G - 1) / (256 / G));
    DSA_DISPATCH_16(dt, T, DSA_SOFTMAX_ROWS(G, NVr, 0,
      hipLaunchKernelGGL((softmax_bwd_rows_kernel<T, GG, VV>), dim3(grid), dim3(256), 0, s, (const T*)dy,
                         (const T*)y, (T*)dx, R, C, scale)));
    return;
  }
  const int nv = (C / 8 + 255) / 256;
  DSA_DISPATCH_16(dt, T, DSA_DISPATCH_SNV(nv, NV,
    hipLaunchKernelGGL((softmax_bwd_kernel<T, NV>), dim3((unsigned)R), dim3(256), 0, s, (const T*)dy,
                       (const T*)y, (T*)dx, R, C, scale)));
}

// --------------------------------------------------------------------------------------
// BERT attention layout moves (reference transform_kernels.cu: bias_add_transform_0213,
// transform4d_0213): one 16-byte vector per thread, reads and writes both coalesced along the
// head dimension.
//   heads_split:  qkv [B, S, 3, NH, HD] -> q, k, v [B, NH, S, HD]   (and heads_merge, its inverse)
//   swap12:       x [A, P, Q, D] -> y [A, Q, P, D]                   (context merge and its backward)
// --------------------------------------------------------------------------------------
template <typename T>
__global__ void __launch_bounds__(256) heads_split_kernel(const uint4* __restrict__ qkv, uint4* __restrict__ q,
                                                          uint4* __restrict__ k, uint4* __restrict__ v, int64_t total,
                                                          int S, int NH, int HV) {
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int dv = (int)(t % HV);
    int64_t r = t / HV;
    const int h = (int)(r % NH); r /= NH;
    const int which = (int)(r % 3); r /= 3;
    const int s = (int)(r % S);
    const int64_t b = r / S;
    uint4* dst = which == 0 ? q : (which == 1 ? k : v);
    dst[((b * NH + h) * S + s) * HV + dv] = qkv[t];
  }
}

template <typename T>
__global__ void __launch_bounds__(256) heads_merge_kernel(const uint4* __restrict__ q, const uint4* __restrict__ k,
                                                          const uint4* __restrict__ v, uint4* __restrict__ qkv,
                                                          int64_t total, int S, int NH, int HV) {
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int dv = (int)(t % HV);
    int64_t r = t / HV;
    const int h = (int)(r % NH); r /= NH;
    const int which = (int)(r % 3); r /= 3;
    const int s = (int)(r % S);
    const int64_t b = r / S;
    const uint4* src = which == 0 ? q : (which == 1 ? k : v);
    qkv[t] = src[((b * NH + h) * S + s) * HV + dv];
  }
}

__global__ void __launch_bounds__(256) swap12_kernel(const uint4* __restrict__ x, uint4* __restrict__ y, int64_t total,
                                                     int P, int Q, int DV) {
  // t enumerates the OUTPUT [A, Q, P, DV] so writes are contiguous
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int dv = (int)(t % DV);
    int64_t r = t / DV;
    const int p = (int)(r % P); r /= P;
    const int q = (int)(r % Q);
    const int64_t a = r / Q;
    y[t] = x[((a * P + p) * Q + q) * DV + dv];
  }
}

static int move_grid(int64_t vecs) {
  int64_t g = (vecs + 255) / 256;
  if (g > 65536) g = 65536;
  return (int)(g < 1 ? 1 : g);
}

void launch_heads_split(const void* qkv, void* q, void* k, void* v, int B, int S, int NH, int HD, hipStream_t s) {
  const int HV = HD / 8;
  const int64_t total = (int64_t)B * S * 3 * NH * HV;
  hipLaunchKernelGGL((heads_split_kernel<bf16_t>), dim3(move_grid(total)), dim3(256), 0, s, (const uint4*)qkv,
                     (uint4*)q, (uint4*)k, (uint4*)v, total, S, NH, HV);
}

void launch_heads_merge(const void* q, const void* k, const void* v, void* qkv, int B, int S, int NH, int HD,
                        hipStream_t s) {
  const int HV = HD / 8;
  const int64_t total = (int64_t)B * S * 3 * NH * HV;
  hipLaunchKernelGGL((heads_merge_kernel<bf16_t>), dim3(move_grid(total)), dim3(256), 0, s, (const uint4*)q,
                     (const uint4*)k, (const uint4*)v, (uint4*)qkv, total, S, NH, HV);
}

void launch_swap12(const void* x, void* y, int64_t A, int P, int Q, int D, hipStream_t s) {
  const int DV = D / 8;
  const int64_t total = A * P * Q * DV;
  hipLaunchKernelGGL(swap12_kernel, dim3(move_grid(total)), dim3(256), 0, s, (const uint4*)x, (uint4*)y, total, P, Q,
                     DV);
}

}  // namespace dsa
