// Block-sparse attention kernels (replaces the reference's Triton matmul.tr / softmax_*.tr,
// deepspeed/ops/sparse_attention/trsrc, driven by host LUTs from ops/sparse_attention).
//
// Sparse storage (same as the reference): x[z][n][block][block], n = index of the non-zero
// block in torch.nonzero(layout) order (head, block-row, block-col).
//
// * sdd_nt:  C_sparse[z][n] = A[z,h, rows of r] . B[z,h, rows of c]^T   (QK^T)
//            one wave per 16x16 sub-tile of a non-zero block, MFMA 16x16x32, operands read
//            straight from HBM with 16-byte lane loads (the A rows of a block-row are shared by
//            all its blocks and stay L2-resident).
// * dsd:     C[z,h, rows of r] = sum_{n in row r} S[z][n] . D[z,h, rows of c]   (P V)
//            D is passed transposed (Dt [z,h,N,K]) so both MFMA operands are 8-byte row reads;
//            one wave per (16-row sub-tile, 16-col tile) of an output block-row, MFMA 16x16x16.
// * softmax fwd/bwd over the non-zero blocks of each row: one wave per (z, h, row), scale,
//   relative-position embedding, key-padding mask and attention mask (add or mul modes).
#include "../include/dsa_common.h"
#include "../include/launchers.h"

namespace dsa {
namespace sp {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <typename T> struct M;
template <> struct M<bf16_t> {
  __device__ __forceinline__ static f32x4 k32(s16x8 a, s16x8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c,
                                                   0, 0, 0);
  }
  __device__ __forceinline__ static f32x4 k16(s16x4 a, s16x4 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b, c, 0, 0, 0);
  }
  __device__ __forceinline__ static uint16_t st(float f) { return f32_to_bf16(f); }
  __device__ __forceinline__ static float ld(uint16_t h) { return bf16_to_f32(h); }
};
template <> struct M<f16_t> {
  __device__ __forceinline__ static f32x4 k32(s16x8 a, s16x8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0,
                                                  0, 0);
  }
  __device__ __forceinline__ static f32x4 k16(s16x4 a, s16x4 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x16f16(__builtin_bit_cast(f16x4, a), __builtin_bit_cast(f16x4, b), c, 0,
                                                 0, 0);
  }
  __device__ __forceinline__ static uint16_t st(float f) { return f32_to_f16(f); }
  __device__ __forceinline__ static float ld(uint16_t h) { return f16_to_f32(h); }
};

// ---------------------------------------------------------------------------------- SDD
// A [Z,H,Mr,K], B [Z,H,Nr,K] (K % 32 == 0), nz [nnz][3] = (h, r, c); C [Z, nnz, blk, blk]
template <typename T>
__global__ void __launch_bounds__(256) sdd_nt_kernel(const uint16_t* __restrict__ A, const uint16_t* __restrict__ B,
                                                     uint16_t* __restrict__ C, const int* __restrict__ nz, int nnz,
                                                     int H, int Mr, int Nr, int K, int blk, int64_t total,
                                                     float alpha) {
  const int lane = threadIdx.x & 63;
  const int64_t task = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (task >= total) return;  // wave-uniform
  const int ts = blk >> 4, t2 = ts * ts;
  const int64_t zn = task / t2;
  const int sub = (int)(task - zn * t2);
  const int z = (int)(zn / nnz), n = (int)(zn - (int64_t)z * nnz);
  const int ti = sub / ts, tj = sub - ti * ts;
  const int h = nz[3 * n], r = nz[3 * n + 1], c = nz[3 * n + 2];
  const int g = lane >> 4, i = lane & 15;
  const uint16_t* ap = A + (((int64_t)z * H + h) * Mr + (int64_t)r * blk + ti * 16 + i) * K + 8 * g;
  const uint16_t* bp = B + (((int64_t)z * H + h) * Nr + (int64_t)c * blk + tj * 16 + i) * K + 8 * g;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int k = 0; k < K; k += 32)
    acc = M<T>::k32(*reinterpret_cast<const s16x8*>(ap + k), *reinterpret_cast<const s16x8*>(bp + k), acc);
  uint16_t* cp = C + (((int64_t)z * nnz + n) * blk + ti * 16 + 4 * g) * blk + tj * 16 + i;
#pragma unroll
  for (int q = 0; q < 4; ++q) cp[(int64_t)q * blk] = M<T>::st(acc[q] * alpha);
}

// ---------------------------------------------------------------------------------- DSD
// S [Z, nnz, blk, blk]; rowptr [H*nbr+1], cols [nnz] (block-col of each non-zero, CSR by row)
// Dt [Z,H,N,Kd] (= dense operand transposed, Kd = nbc*blk); C [Z,H,nbr*blk,N]
template <typename T>
__global__ void __launch_bounds__(256) dsd_kernel(const uint16_t* __restrict__ S, const int* __restrict__ rowptr,
                                                  const int* __restrict__ cols, const uint16_t* __restrict__ Dt,
                                                  uint16_t* __restrict__ C, int nnz, int H, int nbr, int N, int Kd,
                                                  int blk, int64_t total) {
  const int lane = threadIdx.x & 63;
  const int64_t task = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (task >= total) return;
  const int ts = blk >> 4, tn_count = N >> 4;
  int64_t t = task;
  const int tn = (int)(t % tn_count); t /= tn_count;
  const int ti = (int)(t % ts); t /= ts;
  const int r = (int)(t % nbr); t /= nbr;
  const int h = (int)(t % H);
  const int z = (int)(t / H);
  const int g = lane >> 4, i = lane & 15;
  const int p0 = rowptr[h * nbr + r], p1 = rowptr[h * nbr + r + 1];
  const uint16_t* dbase = Dt + (((int64_t)z * H + h) * N + tn * 16 + i) * Kd + 4 * g;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int p = p0; p < p1; ++p) {
    const int c = cols[p];
    const uint16_t* sp = S + (((int64_t)z * nnz + p) * blk + ti * 16 + i) * blk + 4 * g;
    const uint16_t* dp = dbase + (int64_t)c * blk;
    for (int kc = 0; kc < blk; kc += 16)
      acc = M<T>::k16(*reinterpret_cast<const s16x4*>(sp + kc), *reinterpret_cast<const s16x4*>(dp + kc), acc);
  }
  uint16_t* cp = C + (((int64_t)z * H + h) * nbr * blk + (int64_t)r * blk + ti * 16 + 4 * g) * N + tn * 16 + i;
#pragma unroll
  for (int q = 0; q < 4; ++q) cp[(int64_t)q * N] = M<T>::st(acc[q]);
}

// ---------------------------------------------------------------------------------- softmax
// x [Z, nnz, blk, blk] in place. rpe: dense [.,.,S,S] via strides (z, h, row); kpm [Z, S]
// (stride_z), attn [S, S]; modes: 0 = add, 1 = mul (0 -> -inf).
struct SoftmaxArgs {
  const uint16_t* rpe; int64_t rpe_sz, rpe_sh, rpe_sr;
  const uint16_t* kpm; int64_t kpm_sz;
  const uint16_t* attn; int64_t attn_sr;
  int kpm_mul, attn_mul;
  float scale;
  int causal;  // extension: col > row -> -inf (causal LM without a dense S x S mask)
};

template <typename T>
__device__ __forceinline__ float sm_val(const uint16_t* x, int64_t off, int z, int h, int row, int col,
                                        const SoftmaxArgs& a) {
  if (a.causal && col > row) return -INFINITY;
  float v = M<T>::ld(x[off]) * a.scale;
  if (a.rpe) v += M<T>::ld(a.rpe[z * a.rpe_sz + h * a.rpe_sh + (int64_t)row * a.rpe_sr + col]);
  if (a.kpm) {
    const float m = M<T>::ld(a.kpm[z * a.kpm_sz + col]);
    v += a.kpm_mul ? (m == 0.f ? -INFINITY : 0.f) : m;
  }
  if (a.attn) {
    const float m = M<T>::ld(a.attn[(int64_t)row * a.attn_sr + col]);
    v += a.attn_mul ? (m == 0.f ? -INFINITY : 0.f) : m;
  }
  return v;
}

template <typename T>
__global__ void __launch_bounds__(256) sparse_softmax_fwd_kernel(uint16_t* __restrict__ x,
                                                                 const int* __restrict__ rowptr,
                                                                 const int* __restrict__ cols, int nnz, int H,
                                                                 int nbr, int blk, int64_t total, SoftmaxArgs a) {
  const int lane = threadIdx.x & 63;
  const int64_t task = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (task >= total) return;
  const int S = nbr * blk;
  const int row = (int)(task % S);
  const int h = (int)((task / S) % H);
  const int z = (int)(task / ((int64_t)S * H));
  const int r = row / blk, rr = row - r * blk;
  const int p0 = rowptr[h * nbr + r], p1 = rowptr[h * nbr + r + 1];
  const int len = (p1 - p0) * blk;
  float mx = -INFINITY;
  for (int e = lane; e < len; e += 64) {
    const int p = p0 + e / blk, j = e % blk;
    const int64_t off = (((int64_t)z * nnz + p) * blk + rr) * blk + j;
    mx = fmaxf(mx, sm_val<T>(x, off, z, h, row, cols[p] * blk + j, a));
  }
  mx = wave_max(mx);
  float sum = 0.f;
  for (int e = lane; e < len; e += 64) {
    const int p = p0 + e / blk, j = e % blk;
    const int64_t off = (((int64_t)z * nnz + p) * blk + rr) * blk + j;
    const float v = sm_val<T>(x, off, z, h, row, cols[p] * blk + j, a);
    sum += (mx == -INFINITY) ? 0.f : __expf(v - mx);
  }
  sum = wave_sum(sum);
  const float inv = sum > 0.f ? 1.f / sum : 0.f;
  for (int e = lane; e < len; e += 64) {
    const int p = p0 + e / blk, j = e % blk;
    const int64_t off = (((int64_t)z * nnz + p) * blk + rr) * blk + j;
    const float v = sm_val<T>(x, off, z, h, row, cols[p] * blk + j, a);
    x[off] = M<T>::st((mx == -INFINITY) ? 0.f : __expf(v - mx) * inv);
  }
}

// dx = scale * y * (dy - sum(dy*y)) over the row's non-zero blocks (written into dy)
template <typename T>
__global__ void __launch_bounds__(256) sparse_softmax_bwd_kernel(const uint16_t* __restrict__ y,
                                                                 uint16_t* __restrict__ dy,
                                                                 const int* __restrict__ rowptr, int nnz, int H,
                                                                 int nbr, int blk, int64_t total, float scale) {
  const int lane = threadIdx.x & 63;
  const int64_t task = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (task >= total) return;
  const int S = nbr * blk;
  const int row = (int)(task % S);
  const int h = (int)((task / S) % H);
  const int z = (int)(task / ((int64_t)S * H));
  const int r = row / blk, rr = row - r * blk;
  const int p0 = rowptr[h * nbr + r], p1 = rowptr[h * nbr + r + 1];
  const int len = (p1 - p0) * blk;
  float dot = 0.f;
  for (int e = lane; e < len; e += 64) {
    const int64_t off = (((int64_t)z * nnz + p0 + e / blk) * blk + rr) * blk + e % blk;
    dot += M<T>::ld(y[off]) * M<T>::ld(dy[off]);
  }
  dot = wave_sum(dot);
  for (int e = lane; e < len; e += 64) {
    const int64_t off = (((int64_t)z * nnz + p0 + e / blk) * blk + rr) * blk + e % blk;
    dy[off] = M<T>::st(scale * M<T>::ld(y[off]) * (M<T>::ld(dy[off]) - dot));
  }
}

}  // namespace sp

static inline unsigned waves_grid(int64_t waves) { return (unsigned)((waves + 3) / 4); }

void launch_sparse_sdd(const void* A, const void* B, void* C, const int* nz, int nnz, int Z, int H, int Mr, int Nr,
                       int K, int blk, float alpha, int dt, hipStream_t s) {
  const int64_t total = (int64_t)Z * nnz * (blk / 16) * (blk / 16);
  if (total == 0) return;
  DSA_DISPATCH_16(dt, T,
    hipLaunchKernelGGL((sp::sdd_nt_kernel<T>), dim3(waves_grid(total)), dim3(256), 0, s, (const uint16_t*)A,
                       (const uint16_t*)B, (uint16_t*)C, nz, nnz, H, Mr, Nr, K, blk, total, alpha));
}

void launch_sparse_dsd(const void* S, const int* rowptr, const int* cols, const void* Dt, void* C, int nnz, int Z,
                       int H, int nbr, int N, int Kd, int blk, int dt, hipStream_t s) {
  const int64_t total = (int64_t)Z * H * nbr * (blk / 16) * (N / 16);
  if (total == 0) return;
  DSA_DISPATCH_16(dt, T,
    hipLaunchKernelGGL((sp::dsd_kernel<T>), dim3(waves_grid(total)), dim3(256), 0, s, (const uint16_t*)S, rowptr,
                       cols, (const uint16_t*)Dt, (uint16_t*)C, nnz, H, nbr, N, Kd, blk, total));
}

void launch_sparse_softmax_fwd(void* x, const int* rowptr, const int* cols, int nnz, int Z, int H, int nbr, int blk,
                               const void* rpe, int64_t rpe_sz, int64_t rpe_sh, int64_t rpe_sr, const void* kpm,
                               int64_t kpm_sz, const void* attn, int64_t attn_sr, int kpm_mul, int attn_mul,
                               float scale, int causal, int dt, hipStream_t s) {
  const int64_t total = (int64_t)Z * H * nbr * blk;
  if (total == 0) return;
  sp::SoftmaxArgs a{(const uint16_t*)rpe, rpe_sz, rpe_sh, rpe_sr, (const uint16_t*)kpm, kpm_sz,
                    (const uint16_t*)attn, attn_sr, kpm_mul, attn_mul, scale, causal};
  DSA_DISPATCH_16(dt, T,
    hipLaunchKernelGGL((sp::sparse_softmax_fwd_kernel<T>), dim3(waves_grid(total)), dim3(256), 0, s, (uint16_t*)x,
                       rowptr, cols, nnz, H, nbr, blk, total, a));
}

void launch_sparse_softmax_bwd(const void* y, void* dy, const int* rowptr, int nnz, int Z, int H, int nbr, int blk,
                               float scale, int dt, hipStream_t s) {
  const int64_t total = (int64_t)Z * H * nbr * blk;
  if (total == 0) return;
  DSA_DISPATCH_16(dt, T,
    hipLaunchKernelGGL((sp::sparse_softmax_bwd_kernel<T>), dim3(waves_grid(total)), dim3(256), 0, s,
                       (const uint16_t*)y, (uint16_t*)dy, rowptr, nnz, H, nbr, blk, total, scale));
}

}  // namespace dsa
