// Block-sparse MatMul / Softmax API kernels (the reference's Triton matmul.tr / softmax_*.tr,
// deepspeed/ops/sparse_attention/trsrc, driven by host LUTs from ops/sparse_attention).  The
// fused attention path (SparseSelfAttention) uses flash_attn.hip instead; these kernels serve
// direct users of MatMul(sdd|dsd|dds, trans_a, trans_b) and Softmax.
//
// Sparse storage (same as the reference): x[z][n][block][block], n = index of the non-zero
// block in torch.nonzero(layout) order (head, block-row, block-col).
//
// Both products stage every operand tile into LDS in its NATURAL memory orientation with
// 16-byte loads and stores, and pick the MFMA fragment reader per orientation: rows whose k is
// contiguous read 8 elements straight from LDS, rows whose k is strided read them through
// ds_read_b64_tr_b16 (hardware transpose).  So transposed dense operands (trans_a/trans_b,
// the dds and backward products) and transposed sparse operands (layout^T walk via perm) need
// no gather or transpose copy, and the output is written either row- or column-major through
// the MFMA operand order (each lane stores 4 consecutive elements, 8 bytes).
//
// * sdd: C[z][n] = alpha * A[rows of r(n)] . B[rows of c(n)]^T, one workgroup per non-zero
//        block, K in 64-deep stages (32 at block 128), double-buffered LDS with register prefetch.
// * dsd: C[z,h, rows of r, :] = sum_{p in CSR row r} S_p . D[rows of c_p, :], one workgroup
//        per (row segment, 64 output columns); 64-deep k stages hold max(1, 64/block) blocks.
//        Rows much longer than the mean are split into segments (host LUT, longest first)
//        whose fp32 partials a finish kernel sums, so one long row no longer sets the tail.
// * softmax fwd/bwd: 8..64 lanes per row (short rows share a wave), 16-byte chunks; the row
//        is held in registers (up to 4096 elements) so scale/RPE/masks are evaluated once and x
//        read once; longer rows use an online (max, sum) pass plus a write pass.  Out of place.
#include "../include/dsa_common.h"
#include "../include/launchers.h"

namespace dsa {
namespace sp {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

template <typename T> struct M;
template <> struct M<bf16_t> {
  __device__ __forceinline__ static f32x4 k32(s16x8 a, s16x8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c,
                                                   0, 0, 0);
  }
  __device__ __forceinline__ static uint16_t st(float f) { return f32_to_bf16(f); }
  __device__ __forceinline__ static float ld(uint16_t h) { return bf16_to_f32(h); }
};
template <> struct M<f16_t> {
  __device__ __forceinline__ static f32x4 k32(s16x8 a, s16x8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0,
                                                  0, 0);
  }
  __device__ __forceinline__ static uint16_t st(float f) { return f32_to_f16(f); }
  __device__ __forceinline__ static float ld(uint16_t h) { return f16_to_f32(h); }
};

// MFMA 16x16x32 fragment of a matrix X[i][k]: lane (g = lane/16, i = lane%16) holds
// X[i0 + i][k0 + 8g .. k0 + 8g + 7].  The LDS tile holds X either i-major ([i][k], KMAJ=false)
// or k-major ([k][i], KMAJ=true, read through the hardware transpose; needs a full EXEC mask).
template <bool KMAJ>
__device__ __forceinline__ s16x8 frag(const uint16_t* t, int stride, int i0, int k0, int lane) {
  const int g = lane >> 4, i = lane & 15;
  if constexpr (!KMAJ) {
    return *reinterpret_cast<const s16x8*>(t + (i0 + i) * stride + k0 + 8 * g);
  } else {
    const int q = i >> 2, p = i & 3;
    const uint16_t* a0 = t + (k0 + 8 * g + q) * stride + i0 + 4 * p;
    const s16x4 x = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0));
    const s16x4 y = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0 + 4 * stride));
    return s16x8{x[0], x[1], x[2], x[3], y[0], y[1], y[2], y[3]};
  }
}

// 4 consecutive output elements (one lane's MFMA accumulator) as one 8-byte store
template <typename T>
__device__ __forceinline__ void store4(uint16_t* p, f32x4 v, float alpha) {
  const uint32_t lo = (uint32_t)M<T>::st(v[0] * alpha) | ((uint32_t)M<T>::st(v[1] * alpha) << 16);
  const uint32_t hi = (uint32_t)M<T>::st(v[2] * alpha) | ((uint32_t)M<T>::st(v[3] * alpha) << 16);
  *reinterpret_cast<uint2*>(p) = make_uint2(lo, hi);
}

// ---------------------------------------------------------------------------------- SDD
// A element (z, h, row, k) at z*sz + h*sh + row*sr + k*sk, with sk == 1 (AT=false, tile staged
// [row][k]) or sr == 1 (AT=true, staged [k][row]); B likewise.  C [Z, nnz, BLK, BLK].
struct Mat {
  const uint16_t* p;
  int64_t sz, sh, sr, sk;
};

template <typename T, int BLK, bool AT, bool BT>
__global__ void __launch_bounds__(BLK == 16 ? 64 : 256)
    sdd_kernel(Mat A, Mat B, uint16_t* __restrict__ C, const int* __restrict__ nz, int nnz, int K, float alpha) {
  constexpr int NT = BLK == 16 ? 64 : 256;
  constexpr int KC = BLK == 128 ? 32 : 64;  // keeps the two double-buffered tiles <= 41 KB
  constexpr int AR = AT ? KC : BLK, AW = AT ? BLK : KC, AS = AW + 8;  // tile rows, width, LDS stride
  constexpr int BR = BT ? KC : BLK, BW = BT ? BLK : KC, BS = BW + 8;
  constexpr int ACH = AR * AW / 8, BCH = BR * BW / 8;  // 16-byte chunks per tile
  constexpr int LA = (ACH + NT - 1) / NT, LB = (BCH + NT - 1) / NT;
  // waves: 2x2 over the block's 16x16 sub-tiles (1 wave for BLK 16)
  constexpr int WM = BLK == 16 ? 1 : 2, SUB = BLK / 16, RM = SUB / WM;
  __shared__ __attribute__((aligned(16))) uint16_t As[2][AR * AS];
  __shared__ __attribute__((aligned(16))) uint16_t Bs[2][BR * BS];

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int z = blockIdx.x / nnz, n = blockIdx.x - z * nnz;
  const int h = nz[3 * n], r = nz[3 * n + 1], c = nz[3 * n + 2];
  const uint16_t* ab = A.p + z * A.sz + h * A.sh + (int64_t)r * BLK * A.sr;
  const uint16_t* bb = B.p + z * B.sz + h * B.sh + (int64_t)c * BLK * B.sr;

  uint4 ra[LA], rb[LB];
  auto load = [&](int k0) {
#pragma unroll
    for (int l = 0; l < LA; ++l) {
      const int ch = tid + l * NT, row = ch / (AW / 8), col = (ch % (AW / 8)) * 8;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (ch < ACH) {
        if constexpr (!AT) {
          if (k0 + col < K) v = *reinterpret_cast<const uint4*>(ab + row * A.sr + k0 + col);
        } else {
          if (k0 + row < K) v = *reinterpret_cast<const uint4*>(ab + (int64_t)(k0 + row) * A.sk + col);
        }
      }
      ra[l] = v;
    }
#pragma unroll
    for (int l = 0; l < LB; ++l) {
      const int ch = tid + l * NT, row = ch / (BW / 8), col = (ch % (BW / 8)) * 8;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (ch < BCH) {
        if constexpr (!BT) {
          if (k0 + col < K) v = *reinterpret_cast<const uint4*>(bb + row * B.sr + k0 + col);
        } else {
          if (k0 + row < K) v = *reinterpret_cast<const uint4*>(bb + (int64_t)(k0 + row) * B.sk + col);
        }
      }
      rb[l] = v;
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int l = 0; l < LA; ++l) {
      const int ch = tid + l * NT;
      if (ch < ACH) *reinterpret_cast<uint4*>(&As[buf][(ch / (AW / 8)) * AS + (ch % (AW / 8)) * 8]) = ra[l];
    }
#pragma unroll
    for (int l = 0; l < LB; ++l) {
      const int ch = tid + l * NT;
      if (ch < BCH) *reinterpret_cast<uint4*>(&Bs[buf][(ch / (BW / 8)) * BS + (ch % (BW / 8)) * 8]) = rb[l];
    }
  };

  const int wm = w / WM, wn = w % WM;  // wave's sub-tile block: rows wm*RM.., cols wn*RM..
  f32x4 acc[RM][RM];
#pragma unroll
  for (int a = 0; a < RM; ++a)
#pragma unroll
    for (int b = 0; b < RM; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nst = (K + KC - 1) / KC;
  load(0);
  store(0);
  __syncthreads();
  for (int s = 0; s < nst; ++s) {
    const int buf = s & 1;
    if (s + 1 < nst) load((s + 1) * KC);
#pragma unroll
    for (int kk = 0; kk < KC; kk += 32) {
      s16x8 fb[RM], fa[RM];
#pragma unroll
      for (int j = 0; j < RM; ++j) fb[j] = frag<BT>(Bs[buf], BS, (wn * RM + j) * 16, kk, lane);
#pragma unroll
      for (int i = 0; i < RM; ++i) fa[i] = frag<AT>(As[buf], AS, (wm * RM + i) * 16, kk, lane);
      // out[a][b] = sum_k B[a][k] A[b][k] = C^T: each lane ends with 4 consecutive columns of a row
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int j = 0; j < RM; ++j) acc[i][j] = M<T>::k32(fb[j], fa[i], acc[i][j]);
    }
    if (s + 1 < nst) store(buf ^ 1);
    __syncthreads();
  }
  const int g = lane >> 4, i = lane & 15;
  uint16_t* cb = C + (int64_t)blockIdx.x * BLK * BLK;
#pragma unroll
  for (int a = 0; a < RM; ++a)
#pragma unroll
    for (int b = 0; b < RM; ++b)
      store4<T>(cb + ((wm * RM + a) * 16 + i) * BLK + (wn * RM + b) * 16 + 4 * g, acc[a][b], alpha);
}

// ---------------------------------------------------------------------------------- DSD
// C[z,h, r*BLK + m, n] = sum_{p in CSR row (h, r)} S_eff(p)[m][k] . D[z,h, cols[p]*BLK + k, n]
// S [Z, nnz, BLK, BLK]; TS: S_eff(p) is stored block perm[p] transposed (walk of layout^T).
// D element (z,h,k,n) at z*sz + h*sh + k*sr + n*sk with sk == 1 (DT=false, staged [k][n]) or
// sr == 1 (DT=true, staged [n][k]).  C element (z,h,m,n) at z*sz + h*sh + m*sr + n*sk with
// sk == 1 (CT=false) or sr == 1 (CT=true).
template <typename T, int BLK, bool TS, bool DT, bool CT>
__global__ void __launch_bounds__(256)
    dsd_kernel(const uint16_t* __restrict__ S, const int4* __restrict__ seg, const int* __restrict__ cols,
               const int* __restrict__ perm, Mat D, Mat Cm, float* __restrict__ ws, int nslots, int Np, int nnz,
               int nbr, int N) {
  constexpr int NT = 256, BN = 64;
  constexpr int KS = BLK < 64 ? 64 : BLK, BPS = KS / BLK;  // k depth / blocks per stage
  constexpr int SR = TS ? KS : BLK, SW = TS ? BLK : KS, SST = SW + 8;
  constexpr int DR = DT ? BN : KS, DW = DT ? KS : BN, DST = DW + 8;
  constexpr int BCH = BLK * BLK / 8, DCH = KS * BN / 8;  // chunks: one S block, the D tile
  constexpr int LS = (BPS * BCH + NT - 1) / NT, LD = (DCH + NT - 1) / NT;
  constexpr int RS = BLK / 16;
  __shared__ __attribute__((aligned(16))) uint16_t Ss[2][SR * SST];
  __shared__ __attribute__((aligned(16))) uint16_t Ds[2][DR * DST];

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int ntile = blockIdx.x, n0 = ntile * BN, z = blockIdx.z;
  const int4 sg = seg[blockIdx.y];  // (h*nbr + r, first block, end block, partial slot or -1)
  const int r = sg.x % nbr, h = sg.x / nbr, p0 = sg.y, p1 = sg.z, slot = sg.w;
  const uint16_t* sb = S + (int64_t)z * nnz * BLK * BLK;
  const uint16_t* db = D.p + z * D.sz + h * D.sh;

  uint4 rs[LS], rd[LD];
  auto load = [&](int pst) {  // blocks pst .. pst + BPS - 1 of the row
#pragma unroll
    for (int l = 0; l < LS; ++l) {
      const int ch = tid + l * NT, b = ch / BCH, e = (ch - b * BCH) * 8;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (ch < BPS * BCH && pst + b < p1) {
        const int blk = TS ? perm[pst + b] : pst + b;
        v = *reinterpret_cast<const uint4*>(sb + (int64_t)blk * BLK * BLK + e);
      }
      rs[l] = v;
    }
#pragma unroll
    for (int l = 0; l < LD; ++l) {
      const int ch = tid + l * NT;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (ch < DCH) {
        if constexpr (!DT) {  // tile [k][n]: KS rows of 64 columns
          const int k = ch / (BN / 8), nn = (ch % (BN / 8)) * 8, b = k / BLK;
          if (pst + b < p1 && n0 + nn < N)
            v = *reinterpret_cast<const uint4*>(db + (int64_t)(cols[pst + b] * BLK + k - b * BLK) * D.sr + n0 + nn);
        } else {  // tile [n][k]: 64 rows of KS
          const int nn = ch / (KS / 8), k = (ch % (KS / 8)) * 8, b = k / BLK;
          if (pst + b < p1 && n0 + nn < N)
            v = *reinterpret_cast<const uint4*>(db + (int64_t)(n0 + nn) * D.sk + cols[pst + b] * BLK + k - b * BLK);
        }
      }
      rd[l] = v;
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int l = 0; l < LS; ++l) {
      const int ch = tid + l * NT;
      if (ch < BPS * BCH) {
        const int b = ch / BCH, e = (ch - b * BCH) * 8, br = e / BLK, bc = e % BLK;
        // block b sits at k offset b*BLK: columns of an [m][k] tile, rows of a [k][m] tile
        const int off = TS ? (b * BLK + br) * SST + bc : br * SST + b * BLK + bc;
        *reinterpret_cast<uint4*>(&Ss[buf][off]) = rs[l];
      }
    }
#pragma unroll
    for (int l = 0; l < LD; ++l) {
      const int ch = tid + l * NT;
      if (ch < DCH) *reinterpret_cast<uint4*>(&Ds[buf][(ch / (DW / 8)) * DST + (ch % (DW / 8)) * 8]) = rd[l];
    }
  };

  f32x4 acc[RS];
#pragma unroll
  for (int a = 0; a < RS; ++a) acc[a] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nst = (p1 - p0 + BPS - 1) / BPS;
  if (nst > 0) {
    load(p0);
    store(0);
  }
  __syncthreads();
  for (int s = 0; s < nst; ++s) {
    const int buf = s & 1;
    if (s + 1 < nst) load(p0 + (s + 1) * BPS);
#pragma unroll
    for (int kk = 0; kk < KS; kk += 32) {
      // D^T rows n: a [k][n] tile is k-major, an [n][k] tile i-major
      const s16x8 fd = frag<!DT>(Ds[buf], DST, w * 16, kk, lane);
#pragma unroll
      for (int a = 0; a < RS; ++a) {
        const s16x8 fs = frag<TS>(Ss[buf], SST, a * 16, kk, lane);
        acc[a] = CT ? M<T>::k32(fs, fd, acc[a]) : M<T>::k32(fd, fs, acc[a]);
      }
    }
    if (s + 1 < nst) store(buf ^ 1);
    __syncthreads();
  }
  const int g = lane >> 4, i = lane & 15;
  if (slot >= 0) {  // one segment of a split row: fp32 partial [BLK][Np], summed by dsd_finish
    float* wb = ws + ((int64_t)z * nslots + slot) * BLK * Np;
#pragma unroll
    for (int a = 0; a < RS; ++a) {
      if constexpr (!CT) {
        *reinterpret_cast<f32x4*>(wb + (a * 16 + i) * Np + n0 + w * 16 + 4 * g) = acc[a];
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) wb[(a * 16 + 4 * g + q) * Np + n0 + w * 16 + i] = acc[a][q];
      }
    }
    return;
  }
  uint16_t* cb = const_cast<uint16_t*>(Cm.p) + z * Cm.sz + h * Cm.sh + (int64_t)r * BLK * Cm.sr;
#pragma unroll
  for (int a = 0; a < RS; ++a) {
    if constexpr (!CT) {  // lane: row a*16+i, columns n0 + w*16 + 4g .. +3
      const int nn = n0 + w * 16 + 4 * g;
      if (nn < N) store4<T>(cb + (int64_t)(a * 16 + i) * Cm.sr + nn, acc[a], 1.f);
    } else {  // lane: rows a*16+4g .. +3 of column n0 + w*16 + i
      const int nn = n0 + w * 16 + i;
      if (nn < N) store4<T>(cb + (int64_t)nn * Cm.sk + a * 16 + 4 * g, acc[a], 1.f);
    }
  }
}

// Rows split into several segments (long rows of an unbalanced layout, e.g. the global columns
// of BigBird walked transposed): sum the fp32 partials of row fin = (h*nbr + r, slot0, nslots).
template <typename T, int BLK, bool CT>
__global__ void __launch_bounds__(256) dsd_finish_kernel(const float* __restrict__ ws, const int4* __restrict__ fin,
                                                         Mat Cm, int nslots, int Np, int nbr, int N) {
  const int4 f = fin[blockIdx.x];
  const int z = blockIdx.y, r = f.x % nbr, h = f.x / nbr;
  const float* wb = ws + ((int64_t)z * nslots + f.y) * BLK * Np;
  uint16_t* cb = const_cast<uint16_t*>(Cm.p) + z * Cm.sz + h * Cm.sh + (int64_t)r * BLK * Cm.sr;
  const int nq = N / 4;
  for (int idx = threadIdx.x; idx < BLK * nq; idx += 256) {
    const int m = idx / nq, n = (idx - m * nq) * 4;
    f32x4 v = *reinterpret_cast<const f32x4*>(wb + m * Np + n);
    for (int j = 1; j < f.z; ++j) v += *reinterpret_cast<const f32x4*>(wb + ((int64_t)j * BLK + m) * Np + n);
    if constexpr (!CT) {
      store4<T>(cb + (int64_t)m * Cm.sr + n, v, 1.f);
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q) cb[(int64_t)(n + q) * Cm.sk + m] = M<T>::st(v[q]);
    }
  }
}

// ---------------------------------------------------------------------------------- softmax
// x [Z, nnz, blk, blk]. rpe: dense [.,.,S,S] via strides (z, h, row); kpm [Z, S] (stride_z),
// attn [S, S]; modes: 0 = add, 1 = mul (0 -> -inf).
struct SoftmaxArgs {
  const uint16_t* rpe; int64_t rpe_sz, rpe_sh, rpe_sr;
  const uint16_t* kpm; int64_t kpm_sz;
  const uint16_t* attn; int64_t attn_sr;
  int kpm_mul, attn_mul;
  float scale;
  int causal;  // extension: col > row -> -inf (causal LM without a dense S x S mask)
};

// the 8 biased, scaled scores of one 16-byte chunk (columns col .. col+7 of `row`)
template <typename T>
__device__ __forceinline__ void sm_chunk(const uint4 raw, int z, int h, int row, int col, const SoftmaxArgs& a,
                                         float* v) {
  const uint16_t* e = reinterpret_cast<const uint16_t*>(&raw);
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = M<T>::ld(e[j]) * a.scale;
  if (a.rpe) {
    const uint16_t* p = a.rpe + z * a.rpe_sz + h * a.rpe_sh + (int64_t)row * a.rpe_sr + col;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] += M<T>::ld(p[j]);
  }
  if (a.kpm) {
    const uint16_t* p = a.kpm + z * a.kpm_sz + col;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float m = M<T>::ld(p[j]);
      v[j] += a.kpm_mul ? (m == 0.f ? -INFINITY : 0.f) : m;
    }
  }
  if (a.attn) {
    const uint16_t* p = a.attn + (int64_t)row * a.attn_sr + col;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float m = M<T>::ld(p[j]);
      v[j] += a.attn_mul ? (m == 0.f ? -INFINITY : 0.f) : m;
    }
  }
  if (a.causal) {
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (col + j > row) v[j] = -INFINITY;
  }
}

__device__ __forceinline__ int64_t sm_off(int z, int nnz, int p0, int blk, int rr, int e) {
  return (((int64_t)z * nnz + p0 + e / blk) * blk + rr) * blk + e % blk;
}

template <typename T>
__device__ __forceinline__ uint4 pack8(const float* v, float mul) {
  uint32_t w[4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
    w[j] = (uint32_t)M<T>::st(v[2 * j] * mul) | ((uint32_t)M<T>::st(v[2 * j + 1] * mul) << 16);
  return make_uint4(w[0], w[1], w[2], w[3]);
}

template <int LPR>
__device__ __forceinline__ float group_max(float v) {
#pragma unroll
  for (int o = LPR / 2; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
template <int LPR>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
  for (int o = LPR / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Row bookkeeping: a group of LPR lanes owns one row (64/LPR consecutive rows per wave, so the
// short rows of a sparse layout -- adjacent in memory inside each block -- share a wave).
struct SmRow {
  int z, h, row, rr, p0, nch, sub;
};
__device__ __forceinline__ SmRow sm_row(const int* rowptr, int H, int nbr, int blk, int64_t total, int lpr) {
  const int lane = threadIdx.x & 63;
  int64_t task = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * (64 / lpr) + lane / lpr;
  const bool valid = task < total;
  if (!valid) task = total - 1;
  const int S = nbr * blk;
  SmRow r;
  r.row = (int)(task % S);
  r.h = (int)((task / S) % H);
  r.z = (int)(task / ((int64_t)S * H));
  const int br = r.row / blk;
  r.rr = r.row - br * blk;
  r.p0 = rowptr[r.h * nbr + br];
  r.nch = valid ? (rowptr[r.h * nbr + br + 1] - r.p0) * blk / 8 : 0;
  r.sub = lane % lpr;
  return r;
}

// NC > 0: up to NC chunks of 8 per lane held in registers (rows <= 8*LPR*NC elements).
// NC == 0 (LPR 64): online (max, sum) pass, then a recompute-and-write pass.
template <typename T, int LPR, int NC>
__global__ void __launch_bounds__(256) sparse_softmax_fwd_kernel(const uint16_t* __restrict__ x,
                                                                 uint16_t* __restrict__ y,
                                                                 const int* __restrict__ rowptr,
                                                                 const int* __restrict__ cols, int nnz, int H,
                                                                 int nbr, int blk, int64_t total, SoftmaxArgs a) {
  const SmRow R = sm_row(rowptr, H, nbr, blk, total, LPR);
  const int z = R.z, h = R.h, row = R.row, rr = R.rr, p0 = R.p0, nch = R.nch;
  auto colof = [&](int e) { return cols[p0 + e / blk] * blk + e % blk; };
  if constexpr (NC > 0) {
    float v[NC][8];
    float mx = -INFINITY;
#pragma unroll
    for (int q = 0; q < NC; ++q) {
      const int ch = R.sub + LPR * q;
      if (ch < nch) {
        const int e = 8 * ch;
        const uint4 raw = *reinterpret_cast<const uint4*>(x + sm_off(z, nnz, p0, blk, rr, e));
        sm_chunk<T>(raw, z, h, row, colof(e), a, v[q]);
#pragma unroll
        for (int j = 0; j < 8; ++j) mx = fmaxf(mx, v[q][j]);
      }
    }
    mx = group_max<LPR>(mx);
    float sum = 0.f;
#pragma unroll
    for (int q = 0; q < NC; ++q)
      if (R.sub + LPR * q < nch) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          v[q][j] = mx == -INFINITY ? 0.f : __expf(v[q][j] - mx);
          sum += v[q][j];
        }
      }
    sum = group_sum<LPR>(sum);
    const float inv = sum > 0.f ? 1.f / sum : 0.f;
#pragma unroll
    for (int q = 0; q < NC; ++q) {
      const int ch = R.sub + LPR * q;
      if (ch < nch) *reinterpret_cast<uint4*>(y + sm_off(z, nnz, p0, blk, rr, 8 * ch)) = pack8<T>(v[q], inv);
    }
  } else {
    float mx = -INFINITY, sum = 0.f, v[8];
    for (int ch = R.sub; ch < nch; ch += LPR) {
      const int e = 8 * ch;
      sm_chunk<T>(*reinterpret_cast<const uint4*>(x + sm_off(z, nnz, p0, blk, rr, e)), z, h, row, colof(e), a, v);
      float cm = v[0];
#pragma unroll
      for (int j = 1; j < 8; ++j) cm = fmaxf(cm, v[j]);
      if (cm > mx) {
        sum = mx == -INFINITY ? 0.f : sum * __expf(mx - cm);
        mx = cm;
      }
      if (mx != -INFINITY) {
#pragma unroll
        for (int j = 0; j < 8; ++j) sum += __expf(v[j] - mx);
      }
    }
    const float gmx = group_max<LPR>(mx);
    sum = group_sum<LPR>(mx == -INFINITY ? 0.f : sum * __expf(mx - gmx));
    const float inv = sum > 0.f ? 1.f / sum : 0.f;
    for (int ch = R.sub; ch < nch; ch += LPR) {
      const int e = 8 * ch;
      const int64_t off = sm_off(z, nnz, p0, blk, rr, e);
      sm_chunk<T>(*reinterpret_cast<const uint4*>(x + off), z, h, row, colof(e), a, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = gmx == -INFINITY ? 0.f : __expf(v[j] - gmx);
      *reinterpret_cast<uint4*>(y + off) = pack8<T>(v, inv);
    }
  }
}

// dx = scale * y * (dy - sum(dy*y)) over the row's non-zero blocks.  LPR / NC as in the forward.
template <typename T, int LPR, int NC>
__global__ void __launch_bounds__(256) sparse_softmax_bwd_kernel(const uint16_t* __restrict__ y,
                                                                 const uint16_t* __restrict__ dy,
                                                                 uint16_t* __restrict__ dx,
                                                                 const int* __restrict__ rowptr, int nnz, int H,
                                                                 int nbr, int blk, int64_t total, float scale) {
  const SmRow R = sm_row(rowptr, H, nbr, blk, total, LPR);
  const int z = R.z, rr = R.rr, p0 = R.p0, nch = R.nch;
  auto dot8 = [](uint4 a, uint4 b) {
    const uint16_t *ea = reinterpret_cast<const uint16_t*>(&a), *eb = reinterpret_cast<const uint16_t*>(&b);
    float d = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) d += M<T>::ld(ea[j]) * M<T>::ld(eb[j]);
    return d;
  };
  auto grad8 = [&](uint4 a, uint4 b, float dot) {
    const uint16_t *ea = reinterpret_cast<const uint16_t*>(&a), *eb = reinterpret_cast<const uint16_t*>(&b);
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = M<T>::ld(ea[j]) * (M<T>::ld(eb[j]) - dot);
    return pack8<T>(v, scale);
  };
  float dot = 0.f;
  if constexpr (NC > 0) {
    uint4 ry[NC], rg[NC];
#pragma unroll
    for (int q = 0; q < NC; ++q) {
      const int ch = R.sub + LPR * q;
      if (ch < nch) {
        const int64_t off = sm_off(z, nnz, p0, blk, rr, 8 * ch);
        ry[q] = *reinterpret_cast<const uint4*>(y + off);
        rg[q] = *reinterpret_cast<const uint4*>(dy + off);
        dot += dot8(ry[q], rg[q]);
      }
    }
    dot = group_sum<LPR>(dot);
#pragma unroll
    for (int q = 0; q < NC; ++q) {
      const int ch = R.sub + LPR * q;
      if (ch < nch) *reinterpret_cast<uint4*>(dx + sm_off(z, nnz, p0, blk, rr, 8 * ch)) = grad8(ry[q], rg[q], dot);
    }
  } else {
    for (int ch = R.sub; ch < nch; ch += LPR) {
      const int64_t off = sm_off(z, nnz, p0, blk, rr, 8 * ch);
      dot += dot8(*reinterpret_cast<const uint4*>(y + off), *reinterpret_cast<const uint4*>(dy + off));
    }
    dot = group_sum<LPR>(dot);
    for (int ch = R.sub; ch < nch; ch += LPR) {
      const int64_t off = sm_off(z, nnz, p0, blk, rr, 8 * ch);
      *reinterpret_cast<uint4*>(dx + off) =
          grad8(*reinterpret_cast<const uint4*>(y + off), *reinterpret_cast<const uint4*>(dy + off), dot);
    }
  }
}

}  // namespace sp

static inline unsigned waves_grid(int64_t waves) { return (unsigned)((waves + 3) / 4); }

static inline sp::Mat mat(const void* p, const int64_t* st) {
  return sp::Mat{(const uint16_t*)p, st[0], st[1], st[2], st[3]};
}

#define DSA_SPARSE_BLK(blk, BLK, ...)                   \
  switch (blk) {                                         \
    case 16: { constexpr int BLK = 16; __VA_ARGS__; } break;   \
    case 32: { constexpr int BLK = 32; __VA_ARGS__; } break;   \
    case 64: { constexpr int BLK = 64; __VA_ARGS__; } break;   \
    case 128: { constexpr int BLK = 128; __VA_ARGS__; } break; \
    default: break;                                      \
  }
#define DSA_BOOL(v, B, ...)                       \
  if (v) { constexpr bool B = true; __VA_ARGS__; } \
  else { constexpr bool B = false; __VA_ARGS__; }

void launch_sparse_sdd(const void* A, const int64_t* sa, bool at, const void* B, const int64_t* sb, bool bt, void* C,
                       const int* nz, int nnz, int Z, int K, int blk, float alpha, int dt, hipStream_t s) {
  const int64_t wgs = (int64_t)Z * nnz;
  if (wgs == 0) return;
  const sp::Mat ma = mat(A, sa), mb = mat(B, sb);
  DSA_DISPATCH_16(dt, T, DSA_SPARSE_BLK(blk, BLK, DSA_BOOL(at, AT, DSA_BOOL(bt, BT,
    hipLaunchKernelGGL((sp::sdd_kernel<T, BLK, AT, BT>), dim3((unsigned)wgs), dim3(BLK == 16 ? 64 : 256), 0, s, ma,
                       mb, (uint16_t*)C, nz, nnz, K, alpha)))));
}

void launch_sparse_dsd(const void* S, const int* seg, int nseg, const int* fin, int nfin, const int* cols,
                       const int* perm, const void* D, const int64_t* sd, bool dtr, void* C, const int64_t* sc,
                       bool ctr, float* ws, int nslots, int nnz, int Z, int nbr, int N, int blk, int dt,
                       hipStream_t s) {
  if (Z == 0 || nseg == 0 || N == 0) return;
  const sp::Mat md = mat(D, sd), mc = mat(C, sc);
  const int Np = (N + 63) / 64 * 64;
  const dim3 grid((unsigned)(Np / 64), (unsigned)nseg, (unsigned)Z);
  const bool ts = perm != nullptr;
  DSA_DISPATCH_16(dt, T, DSA_SPARSE_BLK(blk, BLK, DSA_BOOL(ts, TS, DSA_BOOL(dtr, DT, DSA_BOOL(ctr, CT,
    hipLaunchKernelGGL((sp::dsd_kernel<T, BLK, TS, DT, CT>), grid, dim3(256), 0, s, (const uint16_t*)S,
                       (const int4*)seg, cols, perm, md, mc, ws, nslots, Np, nnz, nbr, N))))));
  if (nfin == 0) return;
  DSA_DISPATCH_16(dt, T, DSA_SPARSE_BLK(blk, BLK, DSA_BOOL(ctr, CT,
    hipLaunchKernelGGL((sp::dsd_finish_kernel<T, BLK, CT>), dim3((unsigned)nfin, (unsigned)Z), dim3(256), 0, s,
                       ws, (const int4*)fin, mc, nslots, Np, nbr, N))));
}

// (lanes per row, cached chunks per lane) for the longest row: short rows share a wave,
// rows up to 4096 elements stay in registers, longer ones take the online two-pass path.
static inline int softmax_variant(int max_row) {
  const int nch = (max_row + 7) / 8;
  if (nch <= 8) return 8 * 16 + 1;
  if (nch <= 16) return 16 * 16 + 1;
  if (nch <= 32) return 32 * 16 + 1;
  if (nch <= 64) return 64 * 16 + 1;
  if (nch <= 128) return 64 * 16 + 2;
  if (nch <= 256) return 64 * 16 + 4;
  if (nch <= 512) return 64 * 16 + 8;
  return 64 * 16;
}
#define DSA_SOFTMAX_VARIANT(var, LPR, NC, ...)                                           \
  switch (var) {                                                                         \
    case 8 * 16 + 1: { constexpr int LPR = 8, NC = 1; __VA_ARGS__; } break;              \
    case 16 * 16 + 1: { constexpr int LPR = 16, NC = 1; __VA_ARGS__; } break;            \
    case 32 * 16 + 1: { constexpr int LPR = 32, NC = 1; __VA_ARGS__; } break;            \
    case 64 * 16 + 1: { constexpr int LPR = 64, NC = 1; __VA_ARGS__; } break;            \
    case 64 * 16 + 2: { constexpr int LPR = 64, NC = 2; __VA_ARGS__; } break;            \
    case 64 * 16 + 4: { constexpr int LPR = 64, NC = 4; __VA_ARGS__; } break;            \
    case 64 * 16 + 8: { constexpr int LPR = 64, NC = 8; __VA_ARGS__; } break;            \
    default: { constexpr int LPR = 64, NC = 0; __VA_ARGS__; } break;                     \
  }

static inline unsigned softmax_grid(int64_t rows, int var) {
  const int rows_per_wave = 64 / (var / 16);
  return waves_grid((rows + rows_per_wave - 1) / rows_per_wave);
}

void launch_sparse_softmax_fwd(const void* x, void* y, const int* rowptr, const int* cols, int nnz, int Z, int H,
                               int nbr, int blk, int max_row, const void* rpe, int64_t rpe_sz, int64_t rpe_sh,
                               int64_t rpe_sr, const void* kpm, int64_t kpm_sz, const void* attn, int64_t attn_sr,
                               int kpm_mul, int attn_mul, float scale, int causal, int dt, hipStream_t s) {
  const int64_t total = (int64_t)Z * H * nbr * blk;
  if (total == 0) return;
  sp::SoftmaxArgs a{(const uint16_t*)rpe, rpe_sz, rpe_sh, rpe_sr, (const uint16_t*)kpm, kpm_sz,
                    (const uint16_t*)attn, attn_sr, kpm_mul, attn_mul, scale, causal};
  const int var = softmax_variant(max_row);
  DSA_DISPATCH_16(dt, T, DSA_SOFTMAX_VARIANT(var, LPR, NC,
    hipLaunchKernelGGL((sp::sparse_softmax_fwd_kernel<T, LPR, NC>), dim3(softmax_grid(total, var)), dim3(256), 0,
                       s, (const uint16_t*)x, (uint16_t*)y, rowptr, cols, nnz, H, nbr, blk, total, a)));
}

void launch_sparse_softmax_bwd(const void* y, const void* dy, void* dx, const int* rowptr, int nnz, int Z, int H,
                               int nbr, int blk, int max_row, float scale, int dt, hipStream_t s) {
  const int64_t total = (int64_t)Z * H * nbr * blk;
  if (total == 0) return;
  const int var = softmax_variant(max_row);
  DSA_DISPATCH_16(dt, T, DSA_SOFTMAX_VARIANT(var, LPR, NC,
    hipLaunchKernelGGL((sp::sparse_softmax_bwd_kernel<T, LPR, NC>), dim3(softmax_grid(total, var)), dim3(256), 0,
                       s, (const uint16_t*)y, (const uint16_t*)dy, (uint16_t*)dx, rowptr, nnz, H, nbr, blk, total,
                       scale)));
}

}  // namespace dsa
