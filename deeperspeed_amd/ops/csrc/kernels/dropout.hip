// Dropout with a counter-based Philox4x32-10 generator (replaces csrc/transformer/dropout_kernels.cu,
// which draws from curand with a (seed, offset) context).  Element i uses counter
// (offset + i/4) under key = seed, so any launch is reproducible from (seed, offset) alone:
// activation-checkpoint recomputation and the backward pass never need stored RNG state.
// Masks are stored as uint8 (1 = keep); kept values are scaled by 1/(1-p).
#include <initializer_list>

#include "../include/dsa_common.h"
#include "../include/launchers.h"

namespace dsa {

__device__ __forceinline__ uint4 philox4x32_10(uint4 ctr, uint2 key) {
  const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u, W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t hi0 = __umulhi(M0, ctr.x), lo0 = M0 * ctr.x;
    const uint32_t hi1 = __umulhi(M1, ctr.z), lo1 = M1 * ctr.z;
    ctr = make_uint4(hi1 ^ ctr.y ^ key.x, lo1, hi0 ^ ctr.w ^ key.y, lo0);
    key.x += W0;
    key.y += W1;
  }
  return ctr;
}

// 4 uniform draws in [0, 1) for element group g (elements 4g..4g+3)
__device__ __forceinline__ void uniform4(uint64_t seed, uint64_t offset, uint64_t g, float (&u)[4]) {
  const uint64_t c = offset + g;
  const uint4 r = philox4x32_10(make_uint4((uint32_t)c, (uint32_t)(c >> 32), 0u, 0u),
                                make_uint2((uint32_t)seed, (uint32_t)(seed >> 32)));
  const float k = 2.3283064365386963e-10f;  // 2^-32
  u[0] = r.x * k; u[1] = r.y * k; u[2] = r.z * k; u[3] = r.w * k;
}

// Graph-replayable seeds: with `rng` (device int64 [seed, step]) the seed is read on the GPU and
// the step shifts the Philox counter by 2^40 per increment, so a captured HIP graph draws fresh
// masks on every replay (the host-side seed / offset then only separate the call sites).
__device__ __forceinline__ void rng_apply(const int64_t* __restrict__ rng, uint64_t& seed, uint64_t& offset) {
  if (rng) {
    seed ^= (uint64_t)rng[0];
    offset += (uint64_t)rng[1] << 40;
  }
}

template <typename T>
__global__ void __launch_bounds__(256) dropout_fwd_kernel(const T* __restrict__ x, T* __restrict__ y,
                                                          uint8_t* __restrict__ mask, int64_t n, float p,
                                                          uint64_t seed, uint64_t offset, const int64_t* __restrict__ rng = nullptr) {
  rng_apply(rng, seed, offset);
  const float scale = 1.f / (1.f - p);
  const int64_t ngroups = (n + 3) / 4;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < ngroups; g += stride) {
    float u[4];
    uniform4(seed, offset, g, u);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int64_t i = 4 * g + k;
      if (i < n) {
        const bool keep = u[k] >= p;
        mask[i] = keep;
        Conv<T>::store(y, i, keep ? Conv<T>::load(x, i) * scale : 0.f);
      }
    }
  }
}

template <typename T>
__global__ void __launch_bounds__(256) bias_dropout_residual_kernel(const T* __restrict__ x, const T* __restrict__ b,
                                                                    const T* __restrict__ res, T* __restrict__ y,
                                                                    uint8_t* __restrict__ mask, int64_t n, int C,
                                                                    float p, uint64_t seed, uint64_t offset, const int64_t* __restrict__ rng = nullptr) {
  rng_apply(rng, seed, offset);
  const float scale = 1.f / (1.f - p);
  const int64_t ngroups = (n + 3) / 4;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < ngroups; g += stride) {
    float u[4];
    uniform4(seed, offset, g, u);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int64_t i = 4 * g + k;
      if (i < n) {
        const bool keep = u[k] >= p;
        mask[i] = keep;
        const float v = Conv<T>::load(x, i) + Conv<T>::load(b, (int)(i % C));
        Conv<T>::store(y, i, Conv<T>::load(res, i) + (keep ? v * scale : 0.f));
      }
    }
  }
}

template <typename T>
__global__ void __launch_bounds__(256) dropout_bwd_kernel(const T* __restrict__ dy, const uint8_t* __restrict__ mask,
                                                          T* __restrict__ dx, int64_t n, float scale) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    Conv<T>::store(dx, i, mask[i] ? Conv<T>::load(dy, i) * scale : 0.f);
}

// ---- 16-byte vector forms (VN = 8 for 16-bit types, 4 for fp32): the same element -> Philox
// counter mapping as above, so masks and outputs are bit-identical to the scalar kernels; the
// mask of a vector is stored as one 8- (or 4-) byte word.  Need n % VN == 0 (and C % VN == 0
// for the bias) and 16-byte aligned tensors; the launchers fall back to the scalar kernels.
template <int VN>
__device__ __forceinline__ void draws(uint64_t seed, uint64_t offset, int64_t v, float (&u)[VN]) {
#pragma unroll
  for (int q = 0; q < VN / 4; ++q) {
    float t[4];
    uniform4(seed, offset, (uint64_t)v * (VN / 4) + q, t);
#pragma unroll
    for (int k = 0; k < 4; ++k) u[4 * q + k] = t[k];
  }
}

template <int VN>
__device__ __forceinline__ void store_mask(uint8_t* m, const bool (&keep)[VN]) {
  uint32_t w[2] = {0u, 0u};
#pragma unroll
  for (int k = 0; k < VN; ++k) w[k >> 2] |= (uint32_t)keep[k] << (8 * (k & 3));
  if constexpr (VN == 8) *reinterpret_cast<uint2*>(m) = make_uint2(w[0], w[1]);
  else *reinterpret_cast<uint32_t*>(m) = w[0];
}

template <int VN>
__device__ __forceinline__ void load_mask(const uint8_t* m, bool (&keep)[VN]) {
  uint32_t w[2];
  if constexpr (VN == 8) {
    const uint2 v = *reinterpret_cast<const uint2*>(m);
    w[0] = v.x; w[1] = v.y;
  } else {
    w[0] = *reinterpret_cast<const uint32_t*>(m);
    w[1] = 0u;
  }
#pragma unroll
  for (int k = 0; k < VN; ++k) keep[k] = ((w[k >> 2] >> (8 * (k & 3))) & 0xffu) != 0u;
}

template <typename T>
__global__ void __launch_bounds__(256) dropout_fwd_vec_kernel(const T* __restrict__ x, T* __restrict__ y,
                                                              uint8_t* __restrict__ mask, int64_t n, float p,
                                                              uint64_t seed, uint64_t offset, const int64_t* __restrict__ rng = nullptr) {
  rng_apply(rng, seed, offset);
  constexpr int VN = Vec16<T>::N;
  const float scale = 1.f / (1.f - p);
  const int64_t nvec = n / VN, stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += stride) {
    float u[VN], a[VN];
    bool keep[VN];
    draws<VN>(seed, offset, v, u);
    Vec16<T>::load(x + v * VN, a);
#pragma unroll
    for (int k = 0; k < VN; ++k) {
      keep[k] = u[k] >= p;
      a[k] = keep[k] ? a[k] * scale : 0.f;
    }
    Vec16<T>::store(y + v * VN, a);
    store_mask<VN>(mask + v * VN, keep);
  }
}

template <typename T>
__global__ void __launch_bounds__(256) bias_dropout_residual_vec_kernel(const T* __restrict__ x,
                                                                        const T* __restrict__ b,
                                                                        const T* __restrict__ res,
                                                                        T* __restrict__ y, uint8_t* __restrict__ mask,
                                                                        int64_t n, int C, float p, uint64_t seed,
                                                                        uint64_t offset, const int64_t* __restrict__ rng = nullptr) {
  rng_apply(rng, seed, offset);
  constexpr int VN = Vec16<T>::N;
  const float scale = 1.f / (1.f - p);
  const int64_t nvec = n / VN, stride = (int64_t)gridDim.x * blockDim.x;
  const int cvec = C / VN;
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += stride) {
    float u[VN], a[VN], bb[VN], r[VN];
    bool keep[VN];
    draws<VN>(seed, offset, v, u);
    Vec16<T>::load(x + v * VN, a);
    Vec16<T>::load(b + (int)(v % cvec) * VN, bb);
    Vec16<T>::load(res + v * VN, r);
#pragma unroll
    for (int k = 0; k < VN; ++k) {
      keep[k] = u[k] >= p;
      a[k] = r[k] + (keep[k] ? (a[k] + bb[k]) * scale : 0.f);
    }
    Vec16<T>::store(y + v * VN, a);
    store_mask<VN>(mask + v * VN, keep);
  }
}

template <typename T>
__global__ void __launch_bounds__(256) dropout_bwd_vec_kernel(const T* __restrict__ dy,
                                                              const uint8_t* __restrict__ mask, T* __restrict__ dx,
                                                              int64_t n, float scale) {
  constexpr int VN = Vec16<T>::N;
  const int64_t nvec = n / VN, stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += stride) {
    float g[VN];
    bool keep[VN];
    Vec16<T>::load(dy + v * VN, g);
    load_mask<VN>(mask + v * VN, keep);
#pragma unroll
    for (int k = 0; k < VN; ++k) g[k] = keep[k] ? g[k] * scale : 0.f;
    Vec16<T>::store(dx + v * VN, g);
  }
}

// dropout backward of a bias + dropout + residual block that also yields the bias gradient:
// dx = dy * mask / (1 - p) and per-(block, row-lane) column partials of dx, folded afterwards by
// colsum_kernel, so dx is not read a second time for its column sums.  A block covers tpr
// threads x VN columns and 256 / tpr rows at a time (narrow rows keep every thread busy).
template <typename T>
__global__ void __launch_bounds__(256) dropout_bwd_colsum_kernel(const T* __restrict__ dy,
                                                                 const uint8_t* __restrict__ mask,
                                                                 T* __restrict__ dx, float* __restrict__ partial,
                                                                 int64_t rows, int C, float scale) {
  constexpr int VN = Vec16<T>::N;
  const int cv = C / VN;
  const int tpr = cv < 256 ? cv : 256, rpb = 256 / tpr;
  const int t = threadIdx.x % tpr, rs = threadIdx.x / tpr;
  const int c0 = (blockIdx.x * tpr + t) * VN;
  if (rs >= rpb || c0 >= C) return;
  const int64_t chunk = (rows + gridDim.y - 1) / gridDim.y;
  const int64_t r0 = blockIdx.y * chunk;
  const int64_t r1 = r0 + chunk < rows ? r0 + chunk : rows;
  float acc[VN];
#pragma unroll
  for (int j = 0; j < VN; ++j) acc[j] = 0.f;
  for (int64_t r = r0 + rs; r < r1; r += rpb) {
    float g[VN];
    bool keep[VN];
    Vec16<T>::load(dy + r * C + c0, g);
    load_mask<VN>(mask + r * C + c0, keep);
#pragma unroll
    for (int k = 0; k < VN; ++k) {
      g[k] = keep[k] ? g[k] * scale : 0.f;
      acc[k] += g[k];
    }
    Vec16<T>::store(dx + r * C + c0, g);
  }
  float* pp = partial + ((int64_t)blockIdx.y * rpb + rs) * C + c0;
#pragma unroll
  for (int j = 0; j < VN; j += 4) *reinterpret_cast<float4*>(pp + j) = make_float4(acc[j], acc[j + 1], acc[j + 2], acc[j + 3]);
}

// partial rows for dropout_bwd_colsum: row chunks x rows-per-block
void dropout_bwd_colsum_dims(int64_t rows, int C, int dt, int* cblocks, int* rchunks, int* prows) {
  const int vn = dt == kF32 ? 4 : 8;
  const int cv = C / vn, tpr = cv < 256 ? cv : 256, rpb = 256 / tpr;
  *cblocks = (cv + tpr - 1) / tpr;
  int64_t rc = 1024 / *cblocks;  // ~1024 blocks, each walking >= 16 rows
  if (rc > rows / (16 * rpb)) rc = rows / (16 * rpb);
  if (rc < 1) rc = 1;
  *rchunks = (int)rc;
  *prows = (int)rc * rpb;
}

void launch_dropout_bwd_colsum(const void* dy, const uint8_t* mask, void* dx, void* db, float* partial, int64_t rows,
                               int C, float p, int dt, hipStream_t s) {
  if (rows <= 0) return;
  int cb, rc, pr;
  dropout_bwd_colsum_dims(rows, C, dt, &cb, &rc, &pr);
  DSA_DISPATCH_T(dt, T,
    hipLaunchKernelGGL((dropout_bwd_colsum_kernel<T>), dim3(cb, rc), dim3(256), 0, s, (const T*)dy, mask, (T*)dx,
                       partial, rows, C, 1.f / (1.f - p)));
  launch_colsum_partials(partial, pr, C, db, 0, dt, s);
}

// ---------------------------------------------------------------------------
// bias + dropout + residual fused with the LayerNorm that reads its output (pre-LN blocks:
// out = res + dropout(x + b) is the next sub-layer's LayerNorm input and its residual).  One wave
// per row (H <= 64 lanes x WV vectors): the row stays in registers between the residual sum and
// the statistics, so `out` is not read back by a separate LayerNorm launch.  Masks use the same
// element -> Philox counter map as bias_dropout_residual_vec_kernel and the statistics are taken
// over the ROUNDED out (what a LayerNorm kernel reading it would see): y, out and the mask are
// bit-identical to the two-kernel path.
// ---------------------------------------------------------------------------
template <typename T, int WV>
__global__ void __launch_bounds__(256) bdr_ln_fwd_wave_kernel(
    const T* __restrict__ x, const T* __restrict__ b, const T* __restrict__ res, T* __restrict__ out,
    uint8_t* __restrict__ mask, const T* __restrict__ gamma, const T* __restrict__ beta, T* __restrict__ y,
    float* __restrict__ mean_out, float* __restrict__ rstd_out, int64_t rows, int H, float p, float eps,
    uint64_t seed, uint64_t offset, const int64_t* __restrict__ rng) {
  rng_apply(rng, seed, offset);
  constexpr int VN = Vec16<T>::N;
  const float scale = 1.f / (1.f - p);
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;  // whole wave
  const int nvec = H / VN;
  float vals[WV][VN];
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < WV; ++k) {
    const int vi = lane + 64 * k;
    if (vi < nvec) {
      const int64_t v = row * nvec + vi;  // flat vector index = the unfused kernel's Philox group
      float u[VN], a[VN], bb[VN], r[VN];
      bool keep[VN];
      draws<VN>(seed, offset, v, u);
      Vec16<T>::load(x + v * VN, a);
      Vec16<T>::load(b + vi * VN, bb);
      Vec16<T>::load(res + v * VN, r);
#pragma unroll
      for (int j = 0; j < VN; ++j) {
        keep[j] = u[j] >= p;
        a[j] = r[j] + (keep[j] ? (a[j] + bb[j]) * scale : 0.f);
      }
      const uint4 pk = Vec16<T>::pack(a);
      *reinterpret_cast<uint4*>(out + v * VN) = pk;
      store_mask<VN>(mask + v * VN, keep);
      Vec16<T>::unpack(pk, vals[k]);
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

// Backward of bdr_ln_fwd: the LayerNorm backward (dy, with the residual-path gradient dres added)
// gives dtot = d(out), which is also the residual input's gradient; the same pass applies the
// dropout mask (dxb = dtot * mask / (1 - p), the branch gradient) and gathers three column
// partials per block -- gamma, beta and the bias (sum of dxb) -- folded by one colsum launch.
// Replaces ln_bwd_wave + colsum + dropout_bwd_colsum + colsum (dtot is not re-read).
template <typename T, int WV>
__global__ void __launch_bounds__(256) bdr_ln_bwd_wave_kernel(
    const T* __restrict__ dy, const T* __restrict__ xo, const T* __restrict__ gamma, const float* __restrict__ mean,
    const float* __restrict__ rstd, const T* __restrict__ dres, const uint8_t* __restrict__ mask,
    T* __restrict__ dtot, T* __restrict__ dxb, float* __restrict__ partial, int64_t rows, int H, float scale) {
  extern __shared__ float fold[];  // [4 waves][3][H]
  constexpr int VN = Vec16<T>::N;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int nvec = H / VN;
  float dg[WV][VN], dbt[WV][VN], dbi[WV][VN], gm[WV][VN];
#pragma unroll
  for (int k = 0; k < WV; ++k) {
    const int vi = lane + 64 * k;
#pragma unroll
    for (int j = 0; j < VN; ++j) { dg[k][j] = 0.f; dbt[k][j] = 0.f; dbi[k][j] = 0.f; gm[k][j] = 0.f; }
    if (vi < nvec) Vec16<T>::load(gamma + vi * VN, gm[k]);
  }
  // software-pipelined like ln_bwd_wave_kernel: the next row's loads are in flight during this
  // row's reductions
  const int64_t rstep = (int64_t)gridDim.x * 4;
  int64_t row = (int64_t)blockIdx.x * 4 + w;
  uint4 nx[WV], ng[WV], nr[WV];
  uint2 nk[WV];  // raw mask bytes (one per element; VN == 4 uses .x only)
  float nmu = 0.f, nrs = 0.f;
  auto fetch = [&](int64_t r) {
    if (r >= rows) return;
    nmu = mean[r];
    nrs = rstd[r];
#pragma unroll
    for (int k = 0; k < WV; ++k) {
      const int vi = lane + 64 * k;
      if (vi < nvec) {
        nx[k] = *reinterpret_cast<const uint4*>(xo + r * H + vi * VN);
        ng[k] = *reinterpret_cast<const uint4*>(dy + r * H + vi * VN);
        if (dres) nr[k] = *reinterpret_cast<const uint4*>(dres + r * H + vi * VN);
        if constexpr (VN == 8) nk[k] = *reinterpret_cast<const uint2*>(mask + r * H + vi * VN);
        else nk[k] = make_uint2(*reinterpret_cast<const uint32_t*>(mask + r * H + vi * VN), 0u);
      }
    }
  };
  fetch(row);
  for (; row < rows; row += rstep) {
    const float mu = nmu, rs = nrs;
    float xh[WV][VN], g[WV][VN], rr[WV][VN];
    uint2 keep[WV];
#pragma unroll
    for (int k = 0; k < WV; ++k) {
      Vec16<T>::unpack(nx[k], xh[k]);
      Vec16<T>::unpack(ng[k], g[k]);
      if (dres) Vec16<T>::unpack(nr[k], rr[k]);
      keep[k] = nk[k];
    }
    fetch(row + rstep);
    float a = 0.f, bsum = 0.f;
#pragma unroll
    for (int k = 0; k < WV; ++k) {
      const int vi = lane + 64 * k;
      if (vi < nvec) {
#pragma unroll
        for (int j = 0; j < VN; ++j) {
          xh[k][j] = (xh[k][j] - mu) * rs;
          dg[k][j] = fmaf(g[k][j], xh[k][j], dg[k][j]);
          dbt[k][j] += g[k][j];
          const float dxh = g[k][j] * gm[k][j];
          a += dxh;
          bsum = fmaf(dxh, xh[k][j], bsum);
        }
      }
    }
    a = wave_sum(a) / H;
    bsum = wave_sum(bsum) / H;
#pragma unroll
    for (int k = 0; k < WV; ++k) {
      const int vi = lane + 64 * k;
      if (vi < nvec) {
        float o[VN];
#pragma unroll
        for (int j = 0; j < VN; ++j) o[j] = rs * (g[k][j] * gm[k][j] - a - xh[k][j] * bsum);
        if (dres) {
#pragma unroll
          for (int j = 0; j < VN; ++j) o[j] += rr[k][j];
        }
        const uint4 pk = Vec16<T>::pack(o);
        *reinterpret_cast<uint4*>(dtot + row * H + vi * VN) = pk;
        Vec16<T>::unpack(pk, o);  // the rounded dtot, as the unfused dropout backward reads it
#pragma unroll
        for (int j = 0; j < VN; ++j) {
          const uint32_t wd = j < 4 ? keep[k].x : keep[k].y;
          o[j] = ((wd >> (8 * (j & 3))) & 0xffu) ? o[j] * scale : 0.f;
          dbi[k][j] += o[j];
        }
        Vec16<T>::store(dxb + row * H + vi * VN, o);
      }
    }
  }
#pragma unroll
  for (int k = 0; k < WV; ++k) {
    const int vi = lane + 64 * k;
    if (vi < nvec) {
#pragma unroll
      for (int j = 0; j < VN; ++j) {
        fold[(w * 3) * H + vi * VN + j] = dg[k][j];
        fold[(w * 3 + 1) * H + vi * VN + j] = dbt[k][j];
        fold[(w * 3 + 2) * H + vi * VN + j] = dbi[k][j];
      }
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < 3 * H; c += 256) {
    const int which = c / H, col = c - which * H;
    const float v = fold[(0 * 3 + which) * H + col] + fold[(1 * 3 + which) * H + col] +
                    fold[(2 * 3 + which) * H + col] + fold[(3 * 3 + which) * H + col];
    partial[(int64_t)(which * gridDim.x + blockIdx.x) * H + col] = v;
  }
}

bool bdr_ln_supported(int H, int dt) { return dt != kF32 && H % 8 == 0 && H <= 64 * 2 * 8; }

int bdr_ln_bwd_grid(int64_t rows) {
  const int64_t g = (rows + 3) / 4;
  return (int)(g < 512 ? (g < 1 ? 1 : g) : 512);
}

void launch_bdr_ln_fwd(const void* x, const void* bias, const void* res, void* out, uint8_t* mask, const void* gamma,
                       const void* beta, void* y, float* mean, float* rstd, int64_t rows, int H, float p, float eps,
                       uint64_t seed, uint64_t offset, int dt, hipStream_t s, const int64_t* rng) {
  if (rows <= 0) return;
  DSA_DISPATCH_T(dt, T,
    hipLaunchKernelGGL((bdr_ln_fwd_wave_kernel<T, 2>), dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, s,
                       (const T*)x, (const T*)bias, (const T*)res, (T*)out, mask, (const T*)gamma, (const T*)beta,
                       (T*)y, mean, rstd, rows, H, p, eps, seed, offset, rng));
}

// partial workspace: 3 * bdr_ln_bwd_grid(rows) * H floats
void launch_bdr_ln_bwd(const void* dy, const void* xo, const void* gamma, const float* mean, const float* rstd,
                       const void* dres, const uint8_t* mask, void* dtot, void* dxb, void* dgamma, void* dbeta,
                       void* dbias, float* partial, int64_t rows, int H, float p, int accum, int accum_bias, int dt,
                       hipStream_t s) {
  if (rows <= 0) return;
  const int grid = bdr_ln_bwd_grid(rows);
  DSA_DISPATCH_T(dt, T,
    hipLaunchKernelGGL((bdr_ln_bwd_wave_kernel<T, 2>), dim3(grid), dim3(256), 12 * H * sizeof(float), s,
                       (const T*)dy, (const T*)xo, (const T*)gamma, mean, rstd, (const T*)dres, mask, (T*)dtot,
                       (T*)dxb, partial, rows, H, 1.f / (1.f - p)));
  launch_colsum3(partial, grid, H, dgamma, dbeta, dbias, accum, accum_bias, dt, s);
}

static inline bool vec_ok(int64_t n, int vn, std::initializer_list<const void*> ptrs) {
  if (n % vn) return false;
  for (const void* q : ptrs)
    if (q && (reinterpret_cast<uintptr_t>(q) & 15)) return false;
  return true;
}

static inline unsigned dgrid(int64_t work) {
  int64_t g = (work + 255) / 256;
  return (unsigned)(g < 1 ? 1 : (g > 8192 ? 8192 : g));
}

void launch_dropout_fwd(const void* x, void* y, uint8_t* mask, int64_t n, float p, uint64_t seed, uint64_t offset,
                        int dt, hipStream_t s, const int64_t* rng) {
  if (n <= 0) return;
  const int vn = dt == kF32 ? 4 : 8;
  if (vec_ok(n, vn, {x, y}) && (reinterpret_cast<uintptr_t>(mask) & 7) == 0) {
    DSA_DISPATCH_T(dt, T,
      hipLaunchKernelGGL((dropout_fwd_vec_kernel<T>), dim3(dgrid(n / vn)), dim3(256), 0, s, (const T*)x, (T*)y, mask,
                         n, p, seed, offset, rng));
    return;
  }
  DSA_DISPATCH_T(dt, T,
    hipLaunchKernelGGL((dropout_fwd_kernel<T>), dim3(dgrid((n + 3) / 4)), dim3(256), 0, s, (const T*)x, (T*)y, mask,
                       n, p, seed, offset, rng));
}

void launch_bias_dropout_residual(const void* x, const void* bias, const void* res, void* y, uint8_t* mask,
                                  int64_t rows, int C, float p, uint64_t seed, uint64_t offset, int dt,
                                  hipStream_t s, const int64_t* rng) {
  const int64_t n = rows * C;
  if (n <= 0) return;
  const int vn = dt == kF32 ? 4 : 8;
  if (vec_ok(n, vn, {x, bias, res, y}) && C % vn == 0 && (reinterpret_cast<uintptr_t>(mask) & 7) == 0) {
    DSA_DISPATCH_T(dt, T,
      hipLaunchKernelGGL((bias_dropout_residual_vec_kernel<T>), dim3(dgrid(n / vn)), dim3(256), 0, s, (const T*)x,
                         (const T*)bias, (const T*)res, (T*)y, mask, n, C, p, seed, offset, rng));
    return;
  }
  DSA_DISPATCH_T(dt, T,
    hipLaunchKernelGGL((bias_dropout_residual_kernel<T>), dim3(dgrid((n + 3) / 4)), dim3(256), 0, s, (const T*)x,
                       (const T*)bias, (const T*)res, (T*)y, mask, n, C, p, seed, offset, rng));
}

void launch_dropout_bwd(const void* dy, const uint8_t* mask, void* dx, int64_t n, float p, int dt, hipStream_t s) {
  if (n <= 0) return;
  const int vn = dt == kF32 ? 4 : 8;
  if (vec_ok(n, vn, {dy, dx}) && (reinterpret_cast<uintptr_t>(mask) & 7) == 0) {
    DSA_DISPATCH_T(dt, T,
      hipLaunchKernelGGL((dropout_bwd_vec_kernel<T>), dim3(dgrid(n / vn)), dim3(256), 0, s, (const T*)dy, mask, (T*)dx,
                         n, 1.f / (1.f - p)));
    return;
  }
  DSA_DISPATCH_T(dt, T,
    hipLaunchKernelGGL((dropout_bwd_kernel<T>), dim3(dgrid(n)), dim3(256), 0, s, (const T*)dy, mask, (T*)dx, n,
                       1.f / (1.f - p)));
}

}  // namespace dsa
