// LayerNorm / bias-GeLU / bias-residual-dropout kernels for CDNA4.
//
// Parity targets: csrc/transformer/normalize_kernels.cu (fused_bias_residual_layer_norm,
// LayerNormBackward1/2), csrc/transformer/gelu_kernels.cu (fused_bias_gelu, d_gelu_func),
// csrc/transformer/general_kernels.cu (column_sum_reduce).
// MI355X design: one 256-thread block (4 waves) per row with the whole row held in
// registers (16-byte vector loads), fp32 statistics, wave64 shuffles + one LDS hop;
// weight/bias gradients are produced as per-block column partials in the same pass
// and folded by a tiny column-reduce kernel (no atomics, deterministic).
#include <algorithm>
#include <cstdlib>

#include "../include/dsa_common.h"
#include "../include/launchers.h"

namespace dsa {

constexpr int LN_THREADS = 256;
constexpr int LN_MAXV = 8;  // up to 8 16-byte vectors per thread: H <= 16384 (bf16), 8192 (fp32)

// ---------------------------------------------------------------------------
// LayerNorm forward: y = (x - mean) * rstd * gamma + beta
// optional: x_out = x + residual (+ bias) is formed first and stored (pre-LN
// residual fusion); when `res` is null the input is used as-is.
// ---------------------------------------------------------------------------
template <typename T, int NV>
__global__ void __launch_bounds__(LN_THREADS) ln_fwd_kernel(const T* __restrict__ x, const T* __restrict__ res,
                                                            const T* __restrict__ bias, T* __restrict__ sum_out,
                                                            const T* __restrict__ gamma, const T* __restrict__ beta,
                                                            T* __restrict__ y, float* __restrict__ mean_out,
                                                            float* __restrict__ rstd_out, int H, float eps) {
  __shared__ float red[32];
  constexpr int VN = Vec16<T>::N;
  const int nvec = H / VN;
  const int64_t row = blockIdx.x;
  const T* xr = x + row * H;
  float vals[NV][VN];
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int vi = threadIdx.x + k * LN_THREADS;
    if (vi < nvec) {
      Vec16<T>::load(xr + vi * VN, vals[k]);
      if (res) {
        float r[VN];
        Vec16<T>::load(res + row * H + vi * VN, r);
#pragma unroll
        for (int j = 0; j < VN; ++j) vals[k][j] += r[j];
        if (bias) {
          float b[VN];
          Vec16<T>::load(bias + vi * VN, b);
#pragma unroll
          for (int j = 0; j < VN; ++j) vals[k][j] += b[j];
        }
        if (sum_out) Vec16<T>::store(sum_out + row * H + vi * VN, vals[k]);
      }
#pragma unroll
      for (int j = 0; j < VN; ++j) s += vals[k][j];
    }
  }
  const float mean = block_sum(s, red) / H;
  float ss = 0.f;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int vi = threadIdx.x + k * LN_THREADS;
    if (vi < nvec) {
#pragma unroll
      for (int j = 0; j < VN; ++j) { float d = vals[k][j] - mean; ss = fmaf(d, d, ss); }
    }
  }
  const float var = block_sum(ss, red) / H;
  const float rstd = rsqrtf(var + eps);
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int vi = threadIdx.x + k * LN_THREADS;
    if (vi < nvec) {
      float gm[VN], bt[VN], o[VN];
      Vec16<T>::load(gamma + vi * VN, gm);
      if (beta) Vec16<T>::load(beta + vi * VN, bt);
#pragma unroll
      for (int j = 0; j < VN; ++j) o[j] = (vals[k][j] - mean) * rstd * gm[j] + (beta ? bt[j] : 0.f);
      Vec16<T>::store(y + row * H + vi * VN, o);
    }
  }
  if (threadIdx.x == 0) { mean_out[row] = mean; rstd_out[row] = rstd; }
}

// ---------------------------------------------------------------------------
// LayerNorm backward. Each block walks rows blockIdx.x, blockIdx.x + gridDim.x, ...
// computes dx per row and accumulates dgamma/dbeta column partials in registers,
// written once per block into partial[blockIdx.x][H] (and [gridDim + blockIdx.x][H]).
// dres (optional): gradient flowing through a residual branch, added into dx.
// ---------------------------------------------------------------------------
template <typename T, int NV>
__global__ void __launch_bounds__(LN_THREADS) ln_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                            const T* __restrict__ gamma,
                                                            const float* __restrict__ mean,
                                                            const float* __restrict__ rstd,
                                                            const T* __restrict__ dres, T* __restrict__ dx,
                                                            float* __restrict__ partial, int64_t rows, int H,
                                                            int pf = 1) {
  __shared__ float red[32];
  constexpr int VN = Vec16<T>::N;
  const int nvec = H / VN;
  float dg[NV][VN], db[NV][VN], gm[NV][VN];
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int vi = threadIdx.x + k * LN_THREADS;
#pragma unroll
    for (int j = 0; j < VN; ++j) { dg[k][j] = 0.f; db[k][j] = 0.f; gm[k][j] = 0.f; }
    if (vi < nvec) Vec16<T>::load(gamma + vi * VN, gm[k]);
  }
  // software-pipelined over the block's rows: the next row's x / dy (and its mean / rstd) are in
  // flight while this row is reduced across the block -- one row per block in flight left the
  // 512-block grid at ~3.7 TB/s on [32768, 2048] (profiles/r4e_neox13b_zero2_mb16_timed_kernel_stats.md)
  float nx[NV][VN], ng[NV][VN];
  float nmu = 0.f, nrs = 0.f;
  auto fetch = [&](int64_t r) {
    nmu = mean[r];
    nrs = rstd[r];
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int vi = threadIdx.x + k * LN_THREADS;
      if (vi < nvec) {
        Vec16<T>::load(x + r * H + vi * VN, nx[k]);
        Vec16<T>::load(dy + r * H + vi * VN, ng[k]);
      }
    }
  };
  if ((int64_t)blockIdx.x < rows) fetch(blockIdx.x);
  for (int64_t row = blockIdx.x; row < rows; row += gridDim.x) {
    if (!pf && row != blockIdx.x) fetch(row);  // pf = 0: load the row just in time (A/B)
    const float mu = nmu, rs = nrs;
    float xh[NV][VN], g[NV][VN], rr[NV][VN];
#pragma unroll
    for (int k = 0; k < NV; ++k)
#pragma unroll
      for (int j = 0; j < VN; ++j) { xh[k][j] = nx[k][j]; g[k][j] = ng[k][j]; }
    if (pf && row + gridDim.x < rows) fetch(row + gridDim.x);
    if (dres) {
#pragma unroll
      for (int k = 0; k < NV; ++k) {
        const int vi = threadIdx.x + k * LN_THREADS;
        if (vi < nvec) Vec16<T>::load(dres + row * H + vi * VN, rr[k]);
      }
    }
    float a = 0.f, b = 0.f;  // sum(dxhat), sum(dxhat * xhat)
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int vi = threadIdx.x + k * LN_THREADS;
      if (vi < nvec) {
#pragma unroll
        for (int j = 0; j < VN; ++j) {
          xh[k][j] = (xh[k][j] - mu) * rs;
          dg[k][j] = fmaf(g[k][j], xh[k][j], dg[k][j]);
          db[k][j] += g[k][j];
          const float dxh = g[k][j] * gm[k][j];
          a += dxh;
          b = fmaf(dxh, xh[k][j], b);
        }
      }
    }
    block_sum2(a, b, red);
    a /= H; b /= H;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int vi = threadIdx.x + k * LN_THREADS;
      if (vi < nvec) {
        float o[VN];
#pragma unroll
        for (int j = 0; j < VN; ++j) o[j] = rs * (g[k][j] * gm[k][j] - a - xh[k][j] * b);
        if (dres) {
#pragma unroll
          for (int j = 0; j < VN; ++j) o[j] += rr[k][j];
        }
        Vec16<T>::store(dx + row * H + vi * VN, o);
      }
    }
  }
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int vi = threadIdx.x + k * LN_THREADS;
    if (vi < nvec) {
      float* pg = partial + (int64_t)blockIdx.x * H + vi * VN;
      float* pb = partial + (int64_t)(gridDim.x + blockIdx.x) * H + vi * VN;
#pragma unroll
      for (int j = 0; j < VN; j += 4) {
        *reinterpret_cast<float4*>(pg + j) = make_float4(dg[k][j], dg[k][j + 1], dg[k][j + 2], dg[k][j + 3]);
        *reinterpret_cast<float4*>(pb + j) = make_float4(db[k][j], db[k][j + 1], db[k][j + 2], db[k][j + 3]);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Wave-per-row LayerNorm for narrow rows (H <= 64 lanes x WV vectors, e.g. BERT's 1024): a
// 256-thread block normalises 4 rows at once with wave-level shuffles only (no LDS hop, no block
// barrier), where the block-per-row kernels would leave half the threads idle and serialise
// every row behind a barrier.  Same math and outputs as ln_fwd_kernel / ln_bwd_kernel.
// ---------------------------------------------------------------------------
template <typename T, int WV>
__global__ void __launch_bounds__(256) ln_fwd_wave_kernel(const T* __restrict__ x, const T* __restrict__ res,
                                                          const T* __restrict__ bias, T* __restrict__ sum_out,
                                                          const T* __restrict__ gamma, const T* __restrict__ beta,
                                                          T* __restrict__ y, float* __restrict__ mean_out,
                                                          float* __restrict__ rstd_out, int64_t rows, int H,
                                                          float eps) {
  constexpr int VN = Vec16<T>::N;
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;  // whole wave
  const int nvec = H / VN;
  const T* xr = x + row * H;
  float vals[WV][VN];
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < WV; ++k) {
    const int vi = lane + 64 * k;
    if (vi < nvec) {
      Vec16<T>::load(xr + vi * VN, vals[k]);
      if (res) {
        float r[VN];
        Vec16<T>::load(res + row * H + vi * VN, r);
#pragma unroll
        for (int j = 0; j < VN; ++j) vals[k][j] += r[j];
        if (bias) {
          float b[VN];
          Vec16<T>::load(bias + vi * VN, b);
#pragma unroll
          for (int j = 0; j < VN; ++j) vals[k][j] += b[j];
        }
        if (sum_out) Vec16<T>::store(sum_out + row * H + vi * VN, vals[k]);
      }
#pragma unroll
      for (int j = 0; j < VN; ++j) s += vals[k][j];
    }
  }
  const float mean = wave_sum(s) / H;
  float ss = 0.f;
#pragma unroll
  for (int k = 0; k < WV; ++k)
    if (lane + 64 * k < nvec) {
#pragma unroll
      for (int j = 0; j < VN; ++j) { const float d = vals[k][j] - mean; ss = fmaf(d, d, ss); }
    }
  const float rstd = rsqrtf(wave_sum(ss) / H + eps);
#pragma unroll
  for (int k = 0; k < WV; ++k) {
    const int vi = lane + 64 * k;
    if (vi < nvec) {
      float gm[VN], bt[VN], o[VN];
      Vec16<T>::load(gamma + vi * VN, gm);
      if (beta) Vec16<T>::load(beta + vi * VN, bt);
#pragma unroll
      for (int j = 0; j < VN; ++j) o[j] = (vals[k][j] - mean) * rstd * gm[j] + (beta ? bt[j] : 0.f);
      Vec16<T>::store(y + row * H + vi * VN, o);
    }
  }
  if (lane == 0) { mean_out[row] = mean; rstd_out[row] = rstd; }
}

// Each wave walks rows (4 * blockIdx.x + wave) + k * 4 * gridDim.x; gamma/beta partials of the
// block's 4 waves are folded through LDS into partial[blockIdx.x] / [gridDim.x + blockIdx.x].
template <typename T, int WV>
__global__ void __launch_bounds__(256) ln_bwd_wave_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                          const T* __restrict__ gamma, const float* __restrict__ mean,
                                                          const float* __restrict__ rstd, const T* __restrict__ dres,
                                                          T* __restrict__ dx, float* __restrict__ partial,
                                                          int64_t rows, int H) {
  extern __shared__ float fold[];  // [4 waves][2][H]
  constexpr int VN = Vec16<T>::N;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int nvec = H / VN;
  float dg[WV][VN], db[WV][VN], gm[WV][VN];
#pragma unroll
  for (int k = 0; k < WV; ++k) {
    const int vi = lane + 64 * k;
#pragma unroll
    for (int j = 0; j < VN; ++j) { dg[k][j] = 0.f; db[k][j] = 0.f; gm[k][j] = 0.f; }
    if (vi < nvec) Vec16<T>::load(gamma + vi * VN, gm[k]);
  }
  // the row loop is software-pipelined: the next row's x / dy / dres / statistics are loaded
  // (raw 16-byte vectors) before the current row's reductions, so each wave keeps two rows of
  // loads in flight -- with ~2 waves per SIMD the loop was latency-bound at ~2.8 TB/s
  const int64_t rstep = (int64_t)gridDim.x * 4;
  int64_t row = (int64_t)blockIdx.x * 4 + w;
  uint4 nx[WV], ng[WV], nr[WV];
  float nmu = 0.f, nrs = 0.f;
  auto fetch = [&](int64_t r) {
    if (r >= rows) return;
    nmu = mean[r];
    nrs = rstd[r];
#pragma unroll
    for (int k = 0; k < WV; ++k) {
      const int vi = lane + 64 * k;
      if (vi < nvec) {
        nx[k] = *reinterpret_cast<const uint4*>(x + r * H + vi * VN);
        ng[k] = *reinterpret_cast<const uint4*>(dy + r * H + vi * VN);
        if (dres) nr[k] = *reinterpret_cast<const uint4*>(dres + r * H + vi * VN);
      }
    }
  };
  fetch(row);
  for (; row < rows; row += rstep) {
    const float mu = nmu, rs = nrs;
    float xh[WV][VN], g[WV][VN], rr[WV][VN];
#pragma unroll
    for (int k = 0; k < WV; ++k) {
      Vec16<T>::unpack(nx[k], xh[k]);
      Vec16<T>::unpack(ng[k], g[k]);
      if (dres) Vec16<T>::unpack(nr[k], rr[k]);
    }
    fetch(row + rstep);
    float a = 0.f, b = 0.f;
#pragma unroll
    for (int k = 0; k < WV; ++k) {
      const int vi = lane + 64 * k;
      if (vi < nvec) {
#pragma unroll
        for (int j = 0; j < VN; ++j) {
          xh[k][j] = (xh[k][j] - mu) * rs;
          dg[k][j] = fmaf(g[k][j], xh[k][j], dg[k][j]);
          db[k][j] += g[k][j];
          const float dxh = g[k][j] * gm[k][j];
          a += dxh;
          b = fmaf(dxh, xh[k][j], b);
        }
      }
    }
    a = wave_sum(a) / H;
    b = wave_sum(b) / H;
#pragma unroll
    for (int k = 0; k < WV; ++k) {
      const int vi = lane + 64 * k;
      if (vi < nvec) {
        float o[VN];
#pragma unroll
        for (int j = 0; j < VN; ++j) o[j] = rs * (g[k][j] * gm[k][j] - a - xh[k][j] * b);
        if (dres) {
#pragma unroll
          for (int j = 0; j < VN; ++j) o[j] += rr[k][j];
        }
        Vec16<T>::store(dx + row * H + vi * VN, o);
      }
    }
  }
#pragma unroll
  for (int k = 0; k < WV; ++k) {
    const int vi = lane + 64 * k;
    if (vi < nvec) {
#pragma unroll
      for (int j = 0; j < VN; ++j) {
        fold[(w * 2) * H + vi * VN + j] = dg[k][j];
        fold[(w * 2 + 1) * H + vi * VN + j] = db[k][j];
      }
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < 2 * H; c += 256) {
    const int which = c / H, col = c - which * H;
    const float v = fold[(0 * 2 + which) * H + col] + fold[(1 * 2 + which) * H + col] +
                    fold[(2 * 2 + which) * H + col] + fold[(3 * 2 + which) * H + col];
    partial[(int64_t)(which * gridDim.x + blockIdx.x) * H + col] = v;
  }
}

// out[c] = sum_r partial[r][c] over R rows, C columns; written in dtype T
// (optionally accumulated into existing out when `accum`).
// blockIdx.y == 1 sums a second partial block (partial + second_off) into out2 in the same launch
// (LayerNorm's gamma and beta gradients).
// blockIdx.y == 2: a third block (partial + 2 * second_off) into out3 with its own accumulate flag
// (the bias gradient of the fused dropout + LayerNorm backward).
template <typename T>
__global__ void __launch_bounds__(256) colsum_kernel(const float* __restrict__ partial, int R, int C,
                                                     T* __restrict__ out, int accum, int64_t second_off = 0,
                                                     T* __restrict__ out2 = nullptr, T* __restrict__ out3 = nullptr,
                                                     int accum3 = 0) {
  if (blockIdx.y == 1) {
    partial += second_off;
    out = out2;
  } else if (blockIdx.y == 2) {
    partial += 2 * second_off;
    out = out3;
    accum = accum3;
  }
  if (out == nullptr) return;
  // 16 columns x 64 row-groups per block: a lane reads 4 columns (float4) of every 64th row
  // (loads issued 4 at a time, all independent), and C / 16 blocks spread the fold over the chip
  // (C % 4 == 0).  The partials are usually L2-resident (written by the previous kernel).
  // Row-groups are folded by shuffles inside each wave (lanes 4 apart share a column quad),
  // then across the 4 waves through LDS.
  __shared__ float4 red[4][4];
  const int q = threadIdx.x & 3, rg = threadIdx.x >> 2;
  const int c = blockIdx.x * 16 + 4 * q;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (c < C) {
    int r = rg;
    for (; r + 192 < R; r += 256) {
      float4 v[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) v[k] = *reinterpret_cast<const float4*>(partial + (int64_t)(r + 64 * k) * C + c);
#pragma unroll
      for (int k = 0; k < 4; ++k) { acc.x += v[k].x; acc.y += v[k].y; acc.z += v[k].z; acc.w += v[k].w; }
    }
    for (; r < R; r += 64) {
      const float4 v = *reinterpret_cast<const float4*>(partial + (int64_t)r * C + c);
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
  }
#pragma unroll
  for (int off = 4; off < 64; off <<= 1) {
    acc.x += __shfl_xor(acc.x, off, 64);
    acc.y += __shfl_xor(acc.y, off, 64);
    acc.z += __shfl_xor(acc.z, off, 64);
    acc.w += __shfl_xor(acc.w, off, 64);
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (lane < 4) red[wv][lane] = acc;
  __syncthreads();
  if (threadIdx.x < 16) {
    const int qq = threadIdx.x >> 2, comp = threadIdx.x & 3;
    const int col = blockIdx.x * 16 + 4 * qq + comp;
    if (col < C) {
      float v = 0.f;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float4 t = red[g][qq];
        v += comp == 0 ? t.x : comp == 1 ? t.y : comp == 2 ? t.z : t.w;
      }
      if (accum) v += Conv<T>::load(out, col);
      Conv<T>::store(out, col, v);
    }
  }
}

// ---------------------------------------------------------------------------
// bias + GeLU (exact erf or tanh approximation)
// ---------------------------------------------------------------------------
// gelu_f / dgelu_f live in dsa_common.h (shared with the transposing GeLU kernels)

// U vectors per thread and pass, all loads issued before the first GeLU: one 16-byte load per lane
// in flight left the kernel latency-bound at ~3.9 TB/s on MI355X (BERT-Large fc1, 8192 x 4096)
template <typename T, int U>
__global__ void __launch_bounds__(256) bias_gelu_fwd_kernel(const T* __restrict__ x, const T* __restrict__ b,
                                                            T* __restrict__ y, int64_t n, int C, int approx) {
  constexpr int VN = Vec16<T>::N;
  const int64_t nvec = n / VN;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i0 < nvec; i0 += stride * U) {
    float v[U][VN], bb[U][VN];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = i0 + u * stride;
      if (i < nvec) {
        Vec16<T>::load(x + i * VN, v[u]);
        if (b) Vec16<T>::load(b + (int)((i * VN) % C), bb[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = i0 + u * stride;
      if (i < nvec) {
#pragma unroll
        for (int j = 0; j < VN; ++j) v[u][j] = gelu_f(v[u][j] + (b ? bb[u][j] : 0.f), approx);
        Vec16<T>::store(y + i * VN, v[u]);
      }
    }
  }
}

// y = a + b (+ c): the residual sums of a transformer block in one pass (reference fused_add2 /
// fused_add3 / fused_add4, general_kernels.cu:89-292), fp32 accumulation, 16-byte vectors.
template <typename T>
__global__ void __launch_bounds__(256) add3_kernel(const T* __restrict__ a, const T* __restrict__ b,
                                                   const T* __restrict__ c, T* __restrict__ y, int64_t n) {
  constexpr int VN = Vec16<T>::N;
  const int64_t nvec = n / VN;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nvec; i += stride) {
    float va[VN], vb[VN], vc[VN];
    Vec16<T>::load(a + i * VN, va);
    Vec16<T>::load(b + i * VN, vb);
    if (c) {
      Vec16<T>::load(c + i * VN, vc);
#pragma unroll
      for (int j = 0; j < VN; ++j) va[j] += vb[j] + vc[j];
    } else {
#pragma unroll
      for (int j = 0; j < VN; ++j) va[j] += vb[j];
    }
    Vec16<T>::store(y + i * VN, va);
  }
}

// dx = dy * gelu'(x + b); per-block column partials of dx for the bias gradient.
// grid: (ceil(C / (256*VN)), row_chunks); each thread owns VN consecutive columns.
template <typename T>
__global__ void __launch_bounds__(256) bias_gelu_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                            const T* __restrict__ b, T* __restrict__ dx,
                                                            float* __restrict__ partial, int64_t rows, int C,
                                                            int approx) {
  constexpr int VN = Vec16<T>::N;
  const int c0 = (blockIdx.x * 256 + threadIdx.x) * VN;
  if (c0 >= C) return;
  const int64_t chunk = (rows + gridDim.y - 1) / gridDim.y;
  const int64_t r0 = blockIdx.y * chunk;
  const int64_t r1 = r0 + chunk < rows ? r0 + chunk : rows;
  float bb[VN], acc[VN];
#pragma unroll
  for (int j = 0; j < VN; ++j) acc[j] = 0.f;
  if (b) Vec16<T>::load(b + c0, bb);
  int64_t r = r0;
  constexpr int U = 4;  // rows per pass, all 2U loads in flight before the first use
  for (; r + U <= r1; r += U) {
    float xv[U][VN], g[U][VN];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      Vec16<T>::load(x + (r + u) * C + c0, xv[u]);
      Vec16<T>::load(dy + (r + u) * C + c0, g[u]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int j = 0; j < VN; ++j) {
        g[u][j] *= dgelu_f(xv[u][j] + (b ? bb[j] : 0.f), approx);
        acc[j] += g[u][j];
      }
      Vec16<T>::store(dx + (r + u) * C + c0, g[u]);
    }
  }
  for (; r < r1; ++r) {
    float xv[VN], g[VN];
    Vec16<T>::load(x + r * C + c0, xv);
    Vec16<T>::load(dy + r * C + c0, g);
#pragma unroll
    for (int j = 0; j < VN; ++j) {
      g[j] *= dgelu_f(xv[j] + (b ? bb[j] : 0.f), approx);
      acc[j] += g[j];
    }
    Vec16<T>::store(dx + r * C + c0, g);
  }
  if (partial) {
    float* p = partial + (int64_t)blockIdx.y * C + c0;
#pragma unroll
    for (int j = 0; j < VN; j += 4) *reinterpret_cast<float4*>(p + j) = make_float4(acc[j], acc[j + 1], acc[j + 2], acc[j + 3]);
  }
}

// ---------------------------------------------------------------------------
// Host launchers
// ---------------------------------------------------------------------------

#define DSA_DISPATCH_NV(nv, NV, ...)                                \
  switch (nv) {                                                      \
    case 1: { constexpr int NV = 1; __VA_ARGS__; } break;            \
    case 2: { constexpr int NV = 2; __VA_ARGS__; } break;            \
    case 3: { constexpr int NV = 3; __VA_ARGS__; } break;            \
    case 4: { constexpr int NV = 4; __VA_ARGS__; } break;            \
    case 5: case 6: { constexpr int NV = 6; __VA_ARGS__; } break;    \
    default: { constexpr int NV = 8; __VA_ARGS__; } break;           \
  }

int ln_max_hidden(int dt) { return LN_THREADS * LN_MAXV * (dt == kF32 ? 4 : 8); }

// rows of at most 64 lanes x 2 vectors (H <= 1024 for 16-bit, 512 for fp32) take the
// wave-per-row kernels, wider rows the block-per-row ones
static bool ln_wave(int H, int dt) { return H <= 64 * 2 * (dt == kF32 ? 4 : 8); }

void launch_ln_fwd(const void* x, const void* res, const void* bias, void* sum_out, const void* gamma,
                   const void* beta, void* y, float* mean, float* rstd, int64_t rows, int H, float eps, int dt,
                   hipStream_t s) {
  if (rows <= 0) return;
  if (ln_wave(H, dt)) {
    DSA_DISPATCH_T(dt, T,
      hipLaunchKernelGGL((ln_fwd_wave_kernel<T, 2>), dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, s,
                         (const T*)x, (const T*)res, (const T*)bias, (T*)sum_out, (const T*)gamma,
                         (const T*)beta, (T*)y, mean, rstd, rows, H, eps));
    return;
  }
  const int nv = (H / (dt == kF32 ? 4 : 8) + LN_THREADS - 1) / LN_THREADS;
  DSA_DISPATCH_T(dt, T, DSA_DISPATCH_NV(nv, NV,
    hipLaunchKernelGGL((ln_fwd_kernel<T, NV>), dim3((unsigned)rows), dim3(LN_THREADS), 0, s,
                       (const T*)x, (const T*)res, (const T*)bias, (T*)sum_out, (const T*)gamma,
                       (const T*)beta, (T*)y, mean, rstd, H, eps)));
}

int ln_bwd_grid(int64_t rows) { return (int)(rows < 512 ? rows : 512); }

// partial workspace: 2 * ln_bwd_grid(rows) * H floats
void launch_ln_bwd(const void* dy, const void* x, const void* gamma, const float* mean, const float* rstd,
                   const void* dres, void* dx, void* dgamma, void* dbeta, float* partial, int64_t rows, int H,
                   int dt, hipStream_t s, int accum) {
  if (rows <= 0) return;
  const bool wave = ln_wave(H, dt);
  // 16-bit rows of up to 64 lanes x 4 vectors (H <= 2048) also take the wave-per-row backward: at
  // NeoX-1.3B's [32768, 2048] 110-115 vs 158-171 us for the block-per-row kernel, one wave per SIMD
  // and all (profiles/r6r_layernorm_bwd_wave4_ab.log)
  const bool wave4 = !wave && dt != kF32 && H <= 64 * 4 * 8;
  // partial rows: one per block (<= ln_bwd_grid(rows), the caller's workspace)
  const int grid = (wave || wave4) ? (int)std::min<int64_t>(ln_bwd_grid(rows), (rows + 3) / 4) : ln_bwd_grid(rows);
  const int nv = (H / (dt == kF32 ? 4 : 8) + LN_THREADS - 1) / LN_THREADS;
  DSA_DISPATCH_T(dt, T,
    if (wave)
      hipLaunchKernelGGL((ln_bwd_wave_kernel<T, 2>), dim3(grid), dim3(256), 8 * H * sizeof(float), s,
                         (const T*)dy, (const T*)x, (const T*)gamma, mean, rstd, (const T*)dres, (T*)dx, partial,
                         rows, H);
    else if (wave4)
      hipLaunchKernelGGL((ln_bwd_wave_kernel<T, 4>), dim3(grid), dim3(256), 8 * H * sizeof(float), s,
                         (const T*)dy, (const T*)x, (const T*)gamma, mean, rstd, (const T*)dres, (T*)dx, partial,
                         rows, H);
    else
      DSA_DISPATCH_NV(nv, NV, hipLaunchKernelGGL((ln_bwd_kernel<T, NV>), dim3(grid), dim3(LN_THREADS), 0, s,
                         (const T*)dy, (const T*)x, (const T*)gamma, mean, rstd, (const T*)dres, (T*)dx,
                         // row prefetch: +5-9 % at hidden 2048 (one vector per thread), -15 % at 6144
                         // (three: the doubled row registers cost more than the latency they hide),
                         // profiles/r4g_notes.md
                         partial, rows, H, (NV == 1) ? 1 : 0));
    hipLaunchKernelGGL((colsum_kernel<T>), dim3((H + 15) / 16, dbeta ? 2 : 1), dim3(256), 0, s, partial, grid, H,
                       (T*)dgamma, accum, (int64_t)grid * H, (T*)dbeta));
}

void launch_add3(const void* a, const void* b, const void* c, void* y, int64_t n, int dt, hipStream_t s) {
  if (n <= 0) return;
  const int vn = dt == kF32 ? 4 : 8;
  int64_t g = (n / vn + 255) / 256;
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  DSA_DISPATCH_T(dt, T,
    hipLaunchKernelGGL((add3_kernel<T>), dim3((unsigned)g), dim3(256), 0, s, (const T*)a, (const T*)b, (const T*)c,
                       (T*)y, n));
}

void launch_bias_gelu_fwd(const void* x, const void* b, void* y, int64_t rows, int C, int approx, int dt,
                          hipStream_t s) {
  const int64_t n = rows * C;
  if (n <= 0) return;
  const int vn = dt == kF32 ? 4 : 8;
  // two vectors per thread and pass: the GeLU math is cheap enough since the sigmoid form that
  // the kernel is bound by HBM, where more loads in flight pay (1 and 4 measured slower, r5h)
  constexpr int U = 2;
  int64_t g = (n / vn + 256 * U - 1) / (256 * U);
  if (g > 16384) g = 16384;
  if (g < 1) g = 1;
  DSA_DISPATCH_T(dt, T,
    hipLaunchKernelGGL((bias_gelu_fwd_kernel<T, U>), dim3((unsigned)g), dim3(256), 0, s,
                       (const T*)x, (const T*)b, (T*)y, n, C, approx));
}

int bias_gelu_row_chunks(int64_t rows, int C, int dt) {
  const int vn = dt == kF32 ? 4 : 8;
  const int cblocks = (C / vn + 255) / 256;
  // aim for ~2048 blocks total, each walking >= 16 rows
  int64_t rc = 2048 / (cblocks > 0 ? cblocks : 1);
  if (rc > rows / 16) rc = rows / 16;
  if (rc < 1) rc = 1;
  return (int)rc;
}

// partial workspace: bias_gelu_row_chunks(rows, C) * C floats (when db != null)
void launch_bias_gelu_bwd(const void* dy, const void* x, const void* b, void* dx, void* db, float* partial,
                          int64_t rows, int C, int approx, int dt, hipStream_t s, int db_accum) {
  if (rows <= 0) return;
  const int vn = dt == kF32 ? 4 : 8;
  const int cblocks = (C / vn + 255) / 256;
  const int rc = bias_gelu_row_chunks(rows, C, dt);
  DSA_DISPATCH_T(dt, T,
    hipLaunchKernelGGL((bias_gelu_bwd_kernel<T>), dim3(cblocks, rc), dim3(256), 0, s,
                       (const T*)dy, (const T*)x, (const T*)b, (T*)dx, db ? partial : nullptr, rows, C, approx);
    if (db) hipLaunchKernelGGL((colsum_kernel<T>), dim3((C + 15) / 16), dim3(256), 0, s, partial, rc, C,
                               (T*)db, db_accum));
}

// Column sum of a [rows, C] tensor into out[C] (bias gradients of plain linears).
template <typename T>
__global__ void __launch_bounds__(256) colsum_partial_kernel(const T* __restrict__ x, float* __restrict__ partial,
                                                             int64_t rows, int C) {
  constexpr int VN = Vec16<T>::N;
  const int c0 = (blockIdx.x * 256 + threadIdx.x) * VN;
  if (c0 >= C) return;
  const int64_t chunk = (rows + gridDim.y - 1) / gridDim.y;
  const int64_t r0 = blockIdx.y * chunk;
  const int64_t r1 = r0 + chunk < rows ? r0 + chunk : rows;
  float acc[VN];
#pragma unroll
  for (int j = 0; j < VN; ++j) acc[j] = 0.f;
  for (int64_t r = r0; r < r1; ++r) {
    float v[VN];
    Vec16<T>::load(x + r * C + c0, v);
#pragma unroll
    for (int j = 0; j < VN; ++j) acc[j] += v[j];
  }
  float* p = partial + (int64_t)blockIdx.y * C + c0;
#pragma unroll
  for (int j = 0; j < VN; j += 4) *reinterpret_cast<float4*>(p + j) = make_float4(acc[j], acc[j + 1], acc[j + 2], acc[j + 3]);
}

// out[i] (+)= sum_s part[s][i]: the split-K weight-gradient partials folded in one pass with fp32
// accumulation; out in the partials' dtype or fp32 (OUTF).  n % (16 / sizeof(T)) == 0.
template <typename T, bool OUTF>
__global__ void __launch_bounds__(256) sum_slices_kernel(const T* __restrict__ part, int S, int64_t n,
                                                         void* __restrict__ out, int accum) {
  constexpr int VN = Vec16<T>::N;
  const int64_t nvec = n / VN;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nvec; i += stride) {
    float acc[VN];
    if (accum) {
      if constexpr (OUTF) {
#pragma unroll
        for (int j = 0; j < VN; j += 4) {
          const float4 o = *reinterpret_cast<const float4*>((const float*)out + i * VN + j);
          acc[j] = o.x; acc[j + 1] = o.y; acc[j + 2] = o.z; acc[j + 3] = o.w;
        }
      } else {
        Vec16<T>::load((const T*)out + i * VN, acc);
      }
    } else {
#pragma unroll
      for (int j = 0; j < VN; ++j) acc[j] = 0.f;
    }
    for (int sl = 0; sl < S; ++sl) {
      float v[VN];
      Vec16<T>::load(part + sl * n + i * VN, v);
#pragma unroll
      for (int j = 0; j < VN; ++j) acc[j] += v[j];
    }
    if constexpr (OUTF) {
#pragma unroll
      for (int j = 0; j < VN; j += 4)
        *reinterpret_cast<float4*>((float*)out + i * VN + j) = make_float4(acc[j], acc[j + 1], acc[j + 2], acc[j + 3]);
    } else {
      Vec16<T>::store((T*)out + i * VN, acc);
    }
  }
}

void launch_sum_slices(const void* part, int S, int64_t n, void* out, bool out_f32, int accum, int dt,
                       hipStream_t s) {
  if (n <= 0) return;
  const int vn = dt == kF32 ? 4 : 8;
  int64_t g = (n / vn + 255) / 256;
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  DSA_DISPATCH_T(dt, T,
    if (out_f32)
      hipLaunchKernelGGL((sum_slices_kernel<T, true>), dim3((unsigned)g), dim3(256), 0, s, (const T*)part, S, n, out,
                         accum);
    else
      hipLaunchKernelGGL((sum_slices_kernel<T, false>), dim3((unsigned)g), dim3(256), 0, s, (const T*)part, S, n, out,
                         accum));
}

// fp32 partials (the split-K GEMMs write fp32: no bf16 rounding before the sum): out[i] (+)=
// sum_s part[s][i] with out in bf16 / f16 / fp32 (T).
template <typename T>
__global__ void __launch_bounds__(256) sum_slices_f32_kernel(const float* __restrict__ part, int S, int64_t n,
                                                             T* __restrict__ out, int accum) {
  constexpr int VN = Vec16<T>::N;
  const int64_t nvec = n / VN;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nvec; i += stride) {
    float acc[VN];
    if (accum) {
      Vec16<T>::load(out + i * VN, acc);
    } else {
#pragma unroll
      for (int j = 0; j < VN; ++j) acc[j] = 0.f;
    }
    for (int sl = 0; sl < S; ++sl) {
      const float* src = part + sl * n + i * VN;
#pragma unroll
      for (int j = 0; j < VN; j += 4) {
        const float4 v = *reinterpret_cast<const float4*>(src + j);
        acc[j] += v.x; acc[j + 1] += v.y; acc[j + 2] += v.z; acc[j + 3] += v.w;
      }
    }
    Vec16<T>::store(out + i * VN, acc);
  }
}

void launch_sum_slices_f32(const float* part, int S, int64_t n, void* out, int accum, int out_dt, hipStream_t s) {
  if (n <= 0) return;
  const int vn = out_dt == kF32 ? 4 : 8;
  int64_t g = (n / vn + 255) / 256;
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  DSA_DISPATCH_T(out_dt, T,
    hipLaunchKernelGGL((sum_slices_f32_kernel<T>), dim3((unsigned)g), dim3(256), 0, s, part, S, n, (T*)out, accum));
}

void launch_colsum_partials(const float* partial, int R, int C, void* out, int accum, int dt, hipStream_t s) {
  DSA_DISPATCH_T(dt, T,
    hipLaunchKernelGGL((colsum_kernel<T>), dim3((C + 15) / 16), dim3(256), 0, s, partial, R, C, (T*)out, accum));
}

void launch_colsum3(const float* partial, int R, int C, void* out1, void* out2, void* out3, int accum12, int accum3,
                    int dt, hipStream_t s) {
  DSA_DISPATCH_T(dt, T,
    hipLaunchKernelGGL((colsum_kernel<T>), dim3((C + 15) / 16, 3), dim3(256), 0, s, partial, R, C, (T*)out1, accum12,
                       (int64_t)R * C, (T*)out2, (T*)out3, accum3));
}

void launch_colsum(const void* x, void* out, float* partial, int64_t rows, int C, int accum, int dt,
                   hipStream_t s) {
  if (rows <= 0) return;
  const int vn = dt == kF32 ? 4 : 8;
  const int cblocks = (C / vn + 255) / 256;
  const int rc = bias_gelu_row_chunks(rows, C, dt);
  DSA_DISPATCH_T(dt, T,
    hipLaunchKernelGGL((colsum_partial_kernel<T>), dim3(cblocks, rc), dim3(256), 0, s, (const T*)x, partial,
                       rows, C);
    hipLaunchKernelGGL((colsum_kernel<T>), dim3((C + 15) / 16), dim3(256), 0, s, partial, rc, C, (T*)out,
                       accum));
}

// Empty kernel whose only purpose is its name in a kernel trace: bench.py launches it with
// tag 1 right before and tag 2 right after the timed steps, so scripts/prof_summary.py --timed
// can restrict a rocprofv3 trace to the timed region (no init / warmup / memory-fit kernels).
__global__ void dsa_profile_marker_kernel(int tag) { (void)tag; }

void launch_profile_marker(int tag, hipStream_t s) {
  hipLaunchKernelGGL(dsa_profile_marker_kernel, dim3(1), dim3(64), 0, s, tag);
}

}  // namespace dsa
