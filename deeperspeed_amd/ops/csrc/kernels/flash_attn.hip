// Fused (flash-style) attention forward + backward for CDNA4 (gfx950) on bf16/fp16 MFMA.
//
// Replaces the reference's materialised attention path (QK^T strided-batched GEMM ->
// attn_softmax -> PV GEMM, csrc/transformer/softmax_kernels.cu, strided_batch_gemm.h) and
// its S<8192 limit: scores never leave the CU.  Layout: q,k,v,o [B*H, S, D] row-major,
// lse [B*H, S] fp32 (natural log of the scaled row sum), D in {64, 96, 128}.
//
// MFMA mapping (v_mfma_f32_16x16x32_bf16, wave64): lane l, g = l>>4, i = l&15
//   A fragment: A[row i][k 8g..8g+7]      B fragment: B[k 8g..8g+7][col i]
//   C/D:        C[row 4g+r][col i], r = 0..3
// Every operand tile is staged in LDS in its natural [row][D] layout (rows padded by 16 B
// so 16-lane row reads are conflict-free).  Operands needed "down a column" are read with
// ds_read_b64_tr_b16 (hardware transpose, two 4-row blocks per 8-deep fragment), and the
// softmax/dS tiles produced in C layout are re-laid out through a per-wave LDS scratch to
// become A operands.  Workgroup = 4 waves = 64 rows (queries for fwd/dQ, keys for dK/dV).
// Backward is FA2-style without atomics: one kernel owns dK/dV per key block, one owns dQ
// per query block (both recompute P from the saved LSE).
#include "../include/dsa_common.h"
#include "../include/launchers.h"

namespace dsa {
namespace fa {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

constexpr int BM = 64;  // rows per workgroup (16 per wave)
constexpr int BN = 64;  // columns (keys or queries) per inner iteration

template <typename T> struct Mfma;
template <> struct Mfma<bf16_t> {
  __device__ __forceinline__ static f32x4 run(s16x8 a, s16x8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c,
                                                   0, 0, 0);
  }
};
template <> struct Mfma<f16_t> {
  __device__ __forceinline__ static f32x4 run(s16x8 a, s16x8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0,
                                                  0, 0);
  }
};

template <typename T> __device__ __forceinline__ uint16_t to16(float f);
template <> __device__ __forceinline__ uint16_t to16<bf16_t>(float f) { return f32_to_bf16(f); }
template <> __device__ __forceinline__ uint16_t to16<f16_t>(float f) { return f32_to_f16(f); }

// 8 consecutive 16-bit elements of an LDS row (A fragment / B-from-transposed-storage)
__device__ __forceinline__ s16x8 lds_row8(const uint16_t* p) { return *reinterpret_cast<const s16x8*>(p); }

// B fragment read "down a column": rows r0+8g..r0+8g+7, column c0+i of a [rows][stride] tile.
__device__ __forceinline__ s16x8 lds_col8(const uint16_t* base, int stride, int r0, int c0, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const uint16_t* a0 = base + (r0 + 8 * g + q) * stride + c0 + 4 * p;
  const uint16_t* a1 = a0 + 4 * stride;
  s16x4 x = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0));
  s16x4 y = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a1));
  return s16x8{x[0], x[1], x[2], x[3], y[0], y[1], y[2], y[3]};
}

// Cooperative stage of `rows` rows of a [S, D] tensor (row base r0) into an LDS tile with
// row stride D+8; out-of-range rows are zero-filled (keeps EXEC full for tr reads).
template <int D>
__device__ __forceinline__ void stage_rows(uint16_t* lds, const uint16_t* __restrict__ g, int r0, int S) {
  constexpr int CH = D / 8;  // 16-byte chunks per row
  for (int c = threadIdx.x; c < BN * CH; c += blockDim.x) {
    const int r = c / CH, ch = c - r * CH;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (r0 + r < S) v = *reinterpret_cast<const uint4*>(g + (int64_t)(r0 + r) * D + ch * 8);
    *reinterpret_cast<uint4*>(lds + r * (D + 8) + ch * 8) = v;
  }
}

__device__ __forceinline__ float rowgroup_max(float v) {  // across the 16 lanes sharing g
  v = fmaxf(v, __shfl_xor(v, 1, 64));
  v = fmaxf(v, __shfl_xor(v, 2, 64));
  v = fmaxf(v, __shfl_xor(v, 4, 64));
  v = fmaxf(v, __shfl_xor(v, 8, 64));
  return v;
}
__device__ __forceinline__ float rowgroup_sum(float v) {
  v += __shfl_xor(v, 1, 64);
  v += __shfl_xor(v, 2, 64);
  v += __shfl_xor(v, 4, 64);
  v += __shfl_xor(v, 8, 64);
  return v;
}

// ======================================================================== forward
template <typename T, int D, bool CAUSAL>
__global__ void __launch_bounds__(256) fwd_kernel(const uint16_t* __restrict__ Q, const uint16_t* __restrict__ K,
                                                  const uint16_t* __restrict__ V, uint16_t* __restrict__ O,
                                                  float* __restrict__ LSE, int S, float scale) {
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  uint16_t* Ks = smem;                       // [BN][D+8]
  uint16_t* Vs = Ks + BN * (D + 8);          // [BN][D+8]
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint16_t* Ps = Vs + BN * (D + 8) + w * 16 * (BN + 8);  // per wave [16][BN+8]
  const int g = lane >> 4, i = lane & 15;
  const int64_t bh = blockIdx.y;
  const int qb = blockIdx.x * BM;
  const int qrow0 = qb + 16 * w;
  const uint16_t* Qb = Q + bh * (int64_t)S * D;
  const uint16_t* Kb = K + bh * (int64_t)S * D;
  const uint16_t* Vb = V + bh * (int64_t)S * D;

  s16x8 qf[D / 32];
#pragma unroll
  for (int kk = 0; kk < D / 32; ++kk) {
    const int row = qrow0 + i;
    qf[kk] = row < S ? *reinterpret_cast<const s16x8*>(Qb + (int64_t)row * D + 32 * kk + 8 * g) : s16x8{};
  }
  f32x4 o[D / 16];
#pragma unroll
  for (int dt = 0; dt < D / 16; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m[4], l[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) { m[r] = -INFINITY; l[r] = 0.f; }
  const float sl2 = scale * 1.4426950408889634f;  // exp(x) = exp2(x * log2 e)

  const int kend = CAUSAL ? min(S, qb + BM) : S;
  for (int j0 = 0; j0 < kend; j0 += BN) {
    __syncthreads();
    stage_rows<D>(Ks, Kb, j0, S);
    stage_rows<D>(Vs, Vb, j0, S);
    __syncthreads();
    f32x4 s[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      s[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < D / 32; ++kk)
        s[t] = Mfma<T>::run(qf[kk], lds_row8(Ks + (16 * t + i) * (D + 8) + 32 * kk + 8 * g), s[t]);
    }
    // mask + online softmax (rows 4g+r of this wave, keys j0+16t+i)
    float mx[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int qrow = qrow0 + 4 * g + r;
      float v = -INFINITY;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int key = j0 + 16 * t + i;
        float x = s[t][r] * sl2;
        if (key >= S || (CAUSAL && key > qrow)) x = -INFINITY;
        s[t][r] = x;
        v = fmaxf(v, x);
      }
      mx[r] = rowgroup_max(v);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float mn = fmaxf(m[r], mx[r]);
      const float alpha = (mn == -INFINITY) ? 1.f : exp2f(m[r] - mn);
      float ps = 0.f;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const float p = (mn == -INFINITY) ? 0.f : exp2f(s[t][r] - mn);
        s[t][r] = p;
        ps += p;
      }
      l[r] = l[r] * alpha + rowgroup_sum(ps);
      m[r] = mn;
#pragma unroll
      for (int dt = 0; dt < D / 16; ++dt) o[dt][r] *= alpha;
    }
    // P (C layout) -> per-wave LDS [16][BN+8] -> A fragments
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) Ps[(4 * g + r) * (BN + 8) + 16 * t + i] = to16<T>(s[t][r]);
    __syncthreads();
#pragma unroll
    for (int c = 0; c < BN / 32; ++c) {
      const s16x8 pa = lds_row8(Ps + i * (BN + 8) + 32 * c + 8 * g);
#pragma unroll
      for (int dt = 0; dt < D / 16; ++dt) o[dt] = Mfma<T>::run(pa, lds_col8(Vs, D + 8, 32 * c, 16 * dt, lane), o[dt]);
    }
  }
  // epilogue
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int qrow = qrow0 + 4 * g + r;
    const float inv = l[r] > 0.f ? 1.f / l[r] : 0.f;
    if (qrow < S) {
      uint16_t* orow = O + (bh * (int64_t)S + qrow) * D;
#pragma unroll
      for (int dt = 0; dt < D / 16; ++dt) orow[16 * dt + i] = to16<T>(o[dt][r] * inv);
      if (i == 0) LSE[bh * (int64_t)S + qrow] = (m[r] == -INFINITY) ? -INFINITY : (m[r] + log2f(l[r])) * 0.6931471805599453f;
    }
  }
}

// ======================================================================== backward: delta
template <typename T, int D>
__global__ void __launch_bounds__(256) delta_kernel(const uint16_t* __restrict__ dO, const uint16_t* __restrict__ O,
                                                    float* __restrict__ delta, int64_t rows) {
  // 8 lanes per row, 16-byte loads
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t row = t >> 3;
  const int sub = t & 7;
  float acc = 0.f;
  if (row < rows) {
    for (int c = sub; c < D / 8; c += 8) {
      float a[8], b[8];
      Vec16<T>::load(reinterpret_cast<const T*>(dO) + row * D + c * 8, a);
      Vec16<T>::load(reinterpret_cast<const T*>(O) + row * D + c * 8, b);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc = fmaf(a[j], b[j], acc);
    }
  }
  acc += __shfl_xor(acc, 1, 64);
  acc += __shfl_xor(acc, 2, 64);
  acc += __shfl_xor(acc, 4, 64);
  if (row < rows && sub == 0) delta[row] = acc;
}

// ======================================================================== backward: dK, dV
template <typename T, int D, bool CAUSAL>
__global__ void __launch_bounds__(256) bwd_dkdv_kernel(const uint16_t* __restrict__ Q, const uint16_t* __restrict__ K,
                                                       const uint16_t* __restrict__ V, const uint16_t* __restrict__ dO,
                                                       const float* __restrict__ LSE, const float* __restrict__ DELTA,
                                                       uint16_t* __restrict__ dK, uint16_t* __restrict__ dV, int S,
                                                       float scale) {
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  uint16_t* Qs = smem;                   // [BN queries][D+8]
  uint16_t* dOs = Qs + BN * (D + 8);     // [BN][D+8]
  float* lse_s = reinterpret_cast<float*>(dOs + BN * (D + 8));  // [BN]
  float* del_s = lse_s + BN;                                     // [BN]
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint16_t* Pt = reinterpret_cast<uint16_t*>(del_s + BN) + w * 2 * 16 * (BN + 8);  // per wave P^T [16][BN+8]
  uint16_t* dSt = Pt + 16 * (BN + 8);                                             // per wave dS^T [16][BN+8]
  const int g = lane >> 4, i = lane & 15;
  const int64_t bh = blockIdx.y;
  const int kb = blockIdx.x * BM;
  const int krow0 = kb + 16 * w;
  const int64_t base = bh * (int64_t)S * D;
  const float sl2 = scale * 1.4426950408889634f;

  s16x8 kf[D / 32], vf[D / 32];
#pragma unroll
  for (int kk = 0; kk < D / 32; ++kk) {
    const int row = krow0 + i;
    kf[kk] = row < S ? *reinterpret_cast<const s16x8*>(K + base + (int64_t)row * D + 32 * kk + 8 * g) : s16x8{};
    vf[kk] = row < S ? *reinterpret_cast<const s16x8*>(V + base + (int64_t)row * D + 32 * kk + 8 * g) : s16x8{};
  }
  f32x4 dk[D / 16], dv[D / 16];
#pragma unroll
  for (int dt = 0; dt < D / 16; ++dt) { dk[dt] = f32x4{0.f, 0.f, 0.f, 0.f}; dv[dt] = dk[dt]; }

  const int qstart = CAUSAL ? kb : 0;
  for (int i0 = qstart; i0 < S; i0 += BN) {
    __syncthreads();
    stage_rows<D>(Qs, Q + base, i0, S);
    stage_rows<D>(dOs, dO + base, i0, S);
    if (threadIdx.x < BN) {
      const int q = i0 + threadIdx.x;
      lse_s[threadIdx.x] = q < S ? LSE[bh * (int64_t)S + q] : 0.f;
      del_s[threadIdx.x] = q < S ? DELTA[bh * (int64_t)S + q] : 0.f;
    }
    __syncthreads();
    // S^T = K Q^T, dP^T = V dO^T  (rows: keys 4g+r of this wave; cols: queries 16t+i)
    f32x4 s[4], dp[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      s[t] = f32x4{0.f, 0.f, 0.f, 0.f};
      dp[t] = s[t];
#pragma unroll
      for (int kk = 0; kk < D / 32; ++kk) {
        s[t] = Mfma<T>::run(kf[kk], lds_row8(Qs + (16 * t + i) * (D + 8) + 32 * kk + 8 * g), s[t]);
        dp[t] = Mfma<T>::run(vf[kk], lds_row8(dOs + (16 * t + i) * (D + 8) + 32 * kk + 8 * g), dp[t]);
      }
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int qc = 16 * t + i;
      const int q = i0 + qc;
      const float lse2 = lse_s[qc] * 1.4426950408889634f;
      const float dl = del_s[qc];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = krow0 + 4 * g + r;
        float p = exp2f(s[t][r] * sl2 - lse2);
        if (q >= S || key >= S || (CAUSAL && key > q)) p = 0.f;
        const float ds = p * (dp[t][r] - dl);
        Pt[(4 * g + r) * (BN + 8) + qc] = to16<T>(p);
        dSt[(4 * g + r) * (BN + 8) + qc] = to16<T>(ds);
      }
    }
    __syncthreads();
    // dV += P^T dO ; dK += dS^T Q   (contraction over the BN queries)
#pragma unroll
    for (int c = 0; c < BN / 32; ++c) {
      const s16x8 pa = lds_row8(Pt + i * (BN + 8) + 32 * c + 8 * g);
      const s16x8 sa = lds_row8(dSt + i * (BN + 8) + 32 * c + 8 * g);
#pragma unroll
      for (int dt = 0; dt < D / 16; ++dt) {
        dv[dt] = Mfma<T>::run(pa, lds_col8(dOs, D + 8, 32 * c, 16 * dt, lane), dv[dt]);
        dk[dt] = Mfma<T>::run(sa, lds_col8(Qs, D + 8, 32 * c, 16 * dt, lane), dk[dt]);
      }
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int key = krow0 + 4 * g + r;
    if (key < S) {
      uint16_t* dkr = dK + base + (int64_t)key * D;
      uint16_t* dvr = dV + base + (int64_t)key * D;
#pragma unroll
      for (int dt = 0; dt < D / 16; ++dt) {
        dkr[16 * dt + i] = to16<T>(dk[dt][r] * scale);
        dvr[16 * dt + i] = to16<T>(dv[dt][r]);
      }
    }
  }
}

// ======================================================================== backward: dQ
template <typename T, int D, bool CAUSAL>
__global__ void __launch_bounds__(256) bwd_dq_kernel(const uint16_t* __restrict__ Q, const uint16_t* __restrict__ K,
                                                     const uint16_t* __restrict__ V, const uint16_t* __restrict__ dO,
                                                     const float* __restrict__ LSE, const float* __restrict__ DELTA,
                                                     uint16_t* __restrict__ dQ, int S, float scale) {
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  uint16_t* Ks = smem;                 // [BN keys][D+8]
  uint16_t* Vs = Ks + BN * (D + 8);    // [BN][D+8]
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint16_t* dSs = Vs + BN * (D + 8) + w * 16 * (BN + 8);  // per wave dS [16][BN+8]
  const int g = lane >> 4, i = lane & 15;
  const int64_t bh = blockIdx.y;
  const int qb = blockIdx.x * BM;
  const int qrow0 = qb + 16 * w;
  const int64_t base = bh * (int64_t)S * D;
  const float sl2 = scale * 1.4426950408889634f;

  s16x8 qf[D / 32], of[D / 32];
#pragma unroll
  for (int kk = 0; kk < D / 32; ++kk) {
    const int row = qrow0 + i;
    qf[kk] = row < S ? *reinterpret_cast<const s16x8*>(Q + base + (int64_t)row * D + 32 * kk + 8 * g) : s16x8{};
    of[kk] = row < S ? *reinterpret_cast<const s16x8*>(dO + base + (int64_t)row * D + 32 * kk + 8 * g) : s16x8{};
  }
  float lse2[4], dl[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int q = qrow0 + 4 * g + r;
    lse2[r] = q < S ? LSE[bh * (int64_t)S + q] * 1.4426950408889634f : 0.f;
    dl[r] = q < S ? DELTA[bh * (int64_t)S + q] : 0.f;
  }
  f32x4 dq[D / 16];
#pragma unroll
  for (int dt = 0; dt < D / 16; ++dt) dq[dt] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int kend = CAUSAL ? min(S, qb + BM) : S;
  for (int j0 = 0; j0 < kend; j0 += BN) {
    __syncthreads();
    stage_rows<D>(Ks, K + base, j0, S);
    stage_rows<D>(Vs, V + base, j0, S);
    __syncthreads();
    f32x4 s[4], dp[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      s[t] = f32x4{0.f, 0.f, 0.f, 0.f};
      dp[t] = s[t];
#pragma unroll
      for (int kk = 0; kk < D / 32; ++kk) {
        s[t] = Mfma<T>::run(qf[kk], lds_row8(Ks + (16 * t + i) * (D + 8) + 32 * kk + 8 * g), s[t]);
        dp[t] = Mfma<T>::run(of[kk], lds_row8(Vs + (16 * t + i) * (D + 8) + 32 * kk + 8 * g), dp[t]);
      }
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int key = j0 + 16 * t + i;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int q = qrow0 + 4 * g + r;
        float p = exp2f(s[t][r] * sl2 - lse2[r]);
        if (q >= S || key >= S || (CAUSAL && key > q)) p = 0.f;
        dSs[(4 * g + r) * (BN + 8) + 16 * t + i] = to16<T>(p * (dp[t][r] - dl[r]));
      }
    }
    __syncthreads();
#pragma unroll
    for (int c = 0; c < BN / 32; ++c) {
      const s16x8 sa = lds_row8(dSs + i * (BN + 8) + 32 * c + 8 * g);
#pragma unroll
      for (int dt = 0; dt < D / 16; ++dt) dq[dt] = Mfma<T>::run(sa, lds_col8(Ks, D + 8, 32 * c, 16 * dt, lane), dq[dt]);
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int q = qrow0 + 4 * g + r;
    if (q < S) {
      uint16_t* dqr = dQ + base + (int64_t)q * D;
#pragma unroll
      for (int dt = 0; dt < D / 16; ++dt) dqr[16 * dt + i] = to16<T>(dq[dt][r] * scale);
    }
  }
}

template <int D> constexpr int fwd_lds() { return (2 * BN * (D + 8) + 4 * 16 * (BN + 8)) * 2; }
template <int D> constexpr int dkdv_lds() { return (2 * BN * (D + 8)) * 2 + 2 * BN * 4 + 4 * 2 * 16 * (BN + 8) * 2; }
template <int D> constexpr int dq_lds() { return (2 * BN * (D + 8) + 4 * 16 * (BN + 8)) * 2; }

}  // namespace fa

#define FA_DISPATCH(dt, D, causal, ...)                                                              \
  do {                                                                                               \
    auto _go = [&](auto tt, auto dd, auto cc) {                                                      \
      using T = decltype(tt);                                                                        \
      constexpr int DD = decltype(dd)::value;                                                        \
      constexpr bool CC = decltype(cc)::value;                                                       \
      __VA_ARGS__;                                                                                   \
    };                                                                                               \
    auto _d = [&](auto tt, auto cc) {                                                                \
      if (D == 64) _go(tt, std::integral_constant<int, 64>{}, cc);                                  \
      else if (D == 96) _go(tt, std::integral_constant<int, 96>{}, cc);                             \
      else _go(tt, std::integral_constant<int, 128>{}, cc);                                         \
    };                                                                                               \
    auto _c = [&](auto tt) {                                                                         \
      if (causal) _d(tt, std::true_type{}); else _d(tt, std::false_type{});                          \
    };                                                                                               \
    if (dt == kBF16) _c(bf16_t{}); else _c(f16_t{});                                                 \
  } while (0)

bool flash_supported(int D) { return D == 64 || D == 96 || D == 128; }

void launch_flash_fwd(const void* q, const void* k, const void* v, void* o, float* lse, int BH, int S, int D,
                      bool causal, float scale, int dt, hipStream_t s) {
  dim3 grid((S + fa::BM - 1) / fa::BM, BH);
  FA_DISPATCH(dt, D, causal,
    hipLaunchKernelGGL((fa::fwd_kernel<T, DD, CC>), grid, dim3(256), fa::fwd_lds<DD>(), s, (const uint16_t*)q,
                       (const uint16_t*)k, (const uint16_t*)v, (uint16_t*)o, lse, S, scale));
}

void launch_flash_bwd(const void* dout, const void* q, const void* k, const void* v, const void* o, const float* lse,
                      float* delta, void* dq, void* dk, void* dv, int BH, int S, int D, bool causal, float scale,
                      int dt, hipStream_t s) {
  const int64_t rows = (int64_t)BH * S;
  FA_DISPATCH(dt, D, causal,
    hipLaunchKernelGGL((fa::delta_kernel<T, DD>), dim3((unsigned)((rows * 8 + 255) / 256)), dim3(256), 0, s,
                       (const uint16_t*)dout, (const uint16_t*)o, delta, rows);
    hipLaunchKernelGGL((fa::bwd_dkdv_kernel<T, DD, CC>), dim3((S + fa::BM - 1) / fa::BM, BH), dim3(256),
                       fa::dkdv_lds<DD>(), s, (const uint16_t*)q, (const uint16_t*)k, (const uint16_t*)v,
                       (const uint16_t*)dout, lse, delta, (uint16_t*)dk, (uint16_t*)dv, S, scale);
    hipLaunchKernelGGL((fa::bwd_dq_kernel<T, DD, CC>), dim3((S + fa::BM - 1) / fa::BM, BH), dim3(256),
                       fa::dq_lds<DD>(), s, (const uint16_t*)q, (const uint16_t*)k, (const uint16_t*)v,
                       (const uint16_t*)dout, lse, delta, (uint16_t*)dq, S, scale));
}

}  // namespace dsa
