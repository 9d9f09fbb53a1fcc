// 2-D transpose of 16-bit matrices, y[C][R] = x[R][C], with an optional fused column sum of x.
//
// Used to hand the weight-gradient GEMM dW[N,K] = dY^T X (reduction over the M tokens) its
// operands in the layout hipBLASLt runs fastest on gfx950 (both operands contiguous along the
// reduction: ~1.45 PF/s at the GPT-NeoX-20B shapes vs ~1.1 PF/s for the token-major operands,
// profiles/aux/wgrad_dgrad_variants_neox20b.jsonl).  The column sum of dY is the bias gradient,
// so the transpose of dY also produces it (fp32 partial per 128-row tile, reduced by
// colsum_kernel), replacing a separate full read of dY.
//
// The same tile walk also runs the MLP's bias + GeLU with a transposed output: forward (the
// activation recompute, where fc2's forward value is never read and its weight gradient wants
// gelu(u + b)^T) and backward (du = dy * gelu'(u + b) row-major for fc1's input gradient, du^T
// + its column sum for fc1's weight / bias gradients), each replacing an elementwise pass plus a
// separate transpose of a [tokens, 4h] tensor.
//
// Reference counterpart: `Transpose_Kernel` / `transform_0213` (csrc/transformer/
// transform_kernels.cu:7,56) and `column_sum_reduce` (csrc/transformer/general_kernels.cu:6).
//
// Tile 128 rows x 64 columns, 256 threads (4 waves).  Loads are 16-byte row chunks staged in
// LDS (128-B rows, XOR-swizzled 16-B chunks); each output 16-byte chunk (8 consecutive x rows
// of one column) comes from two ds_read_b64_tr_b16 (hardware 4x16 transpose).  Swizzle: the
// physical chunk of logical chunk cc in row r is cc ^ 2*h(r), h(r) = bit1(r) | bit3(r) << 1,
// which makes every transposed read conflict-free (the two 16-lane groups of a half-wave read
// rows 8 apart; their 8 rows then land on 8 distinct 32-byte bank windows).
#include "../include/dsa_common.h"
#include "../include/launchers.h"

namespace dsa {
namespace {

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

constexpr int TR = 128;  // rows (x) per tile = output columns
constexpr int TC = 64;   // columns (x) per tile = output rows

__device__ __forceinline__ int swz(int row, int cc) {
  return cc ^ ((((row >> 1) & 1) | (((row >> 3) & 1) << 1)) << 1);
}

template <typename T> __device__ __forceinline__ float h2f(short v);
template <> __device__ __forceinline__ float h2f<bf16_t>(short v) { return bf16_to_f32((uint16_t)v); }
template <> __device__ __forceinline__ float h2f<f16_t>(short v) { return f16_to_f32((uint16_t)v); }
template <typename T> __device__ __forceinline__ uint16_t f2h(float v);
template <> __device__ __forceinline__ uint16_t f2h<bf16_t>(float v) { return f32_to_bf16(v); }
template <> __device__ __forceinline__ uint16_t f2h<f16_t>(float v) { return f32_to_f16(v); }

// Elementwise op applied to each loaded 8-element chunk before it is staged for the transpose.
enum TrOp : int {
  kCopy = 0,     // y^T = x^T
  kGeluFwd = 1,  // y^T = gelu(x + b)^T  (only the transposed output is written)
  kGeluBwd = 2,  // g = x * gelu'(x2 + b): g written row-major to yr AND transposed to y
};

template <typename T>
__device__ __forceinline__ void unpack8(const uint4& v, float* f) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    f[2 * j] = h2f<T>((short)(w[j] & 0xffff));
    f[2 * j + 1] = h2f<T>((short)(w[j] >> 16));
  }
}

template <typename T>
__device__ __forceinline__ uint4 pack8(const float* f) {
  uint4 o;
  o.x = (uint32_t)f2h<T>(f[0]) | ((uint32_t)f2h<T>(f[1]) << 16);
  o.y = (uint32_t)f2h<T>(f[2]) | ((uint32_t)f2h<T>(f[3]) << 16);
  o.z = (uint32_t)f2h<T>(f[4]) | ((uint32_t)f2h<T>(f[5]) << 16);
  o.w = (uint32_t)f2h<T>(f[6]) | ((uint32_t)f2h<T>(f[7]) << 16);
  return o;
}

// x2 / bias / yr / approx are used by the GeLU ops only (x2: the GeLU input of kGeluBwd, same
// layout as x; yr: row-major output [R][C], row stride C).
template <typename T, bool SUM, int OP>
__global__ void __launch_bounds__(256) transpose_kernel(const uint16_t* __restrict__ x, uint16_t* __restrict__ y,
                                                        float* __restrict__ partial, int64_t R, int C, int64_t ldx,
                                                        const uint16_t* __restrict__ x2,
                                                        const uint16_t* __restrict__ bias,
                                                        uint16_t* __restrict__ yr, int approx) {
  __shared__ __attribute__((aligned(16))) uint16_t tile[TR * TC];
  const int t = threadIdx.x;
  if (gridDim.z > 1) {  // batched plain copy (launch_transpose_batched): slot z of [L][R][ldx] -> [L][C][R]
    x += (int64_t)blockIdx.z * R * ldx;
    y += (int64_t)blockIdx.z * R * C;
  }
  const int64_t r0 = (int64_t)blockIdx.y * TR;
  const int c0 = blockIdx.x * TC;
  uint4 v[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = t + 256 * i, row = c >> 3, cc = c & 7;
    v[i] = *reinterpret_cast<const uint4*>(x + (r0 + row) * ldx + c0 + cc * 8);
  }
  if constexpr (OP != kCopy) {
    uint4 u[4];
    if constexpr (OP == kGeluBwd) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int c = t + 256 * i, row = c >> 3, cc = c & 7;
        u[i] = *reinterpret_cast<const uint4*>(x2 + (r0 + row) * ldx + c0 + cc * 8);
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = t + 256 * i, row = c >> 3, cc = c & 7;
      float f[8], b[8];
      unpack8<T>(v[i], f);
      if (bias) {
        unpack8<T>(*reinterpret_cast<const uint4*>(bias + c0 + cc * 8), b);
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) b[j] = 0.f;
      }
      if constexpr (OP == kGeluFwd) {
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] = gelu_f(f[j] + b[j], approx);
      } else {
        float xi[8];
        unpack8<T>(u[i], xi);
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] *= dgelu_f(xi[j] + b[j], approx);
      }
      v[i] = pack8<T>(f);
      if constexpr (OP == kGeluBwd)
        *reinterpret_cast<uint4*>(yr + (r0 + row) * (int64_t)C + c0 + cc * 8) = v[i];
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = t + 256 * i, row = c >> 3, cc = c & 7;
    *reinterpret_cast<uint4*>(tile + row * TC + swz(row, cc) * 8) = v[i];
  }
  __syncthreads();
  const int lane = t & 63, w = t >> 6, g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  // lane (q, p) of a 16-lane group addresses row rb+q, logical columns 16w+4p .. 16w+4p+3;
  // it receives column 16w+i of the 4 rows.
  const int cc = (16 * w + 4 * p) >> 3, half = p & 1;
  uint16_t* yrow = y + (int64_t)(c0 + 16 * w + i) * R + r0;
  float s = 0.f;
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const int rb = 8 * g + 32 * it;
    const int ra = rb + q, rc = rb + 4 + q;
    s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(tile + ra * TC + swz(ra, cc) * 8 + half * 4));
    s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(tile + rc * TC + swz(rc, cc) * 8 + half * 4));
    uint4 o;
    o.x = (uint32_t)(uint16_t)lo[0] | ((uint32_t)(uint16_t)lo[1] << 16);
    o.y = (uint32_t)(uint16_t)lo[2] | ((uint32_t)(uint16_t)lo[3] << 16);
    o.z = (uint32_t)(uint16_t)hi[0] | ((uint32_t)(uint16_t)hi[1] << 16);
    o.w = (uint32_t)(uint16_t)hi[2] | ((uint32_t)(uint16_t)hi[3] << 16);
    *reinterpret_cast<uint4*>(yrow + rb) = o;
    if constexpr (SUM) {
#pragma unroll
      for (int j = 0; j < 4; ++j) s += h2f<T>(lo[j]) + h2f<T>(hi[j]);
    }
  }
  if constexpr (SUM) {
    s += __shfl_xor(s, 16);
    s += __shfl_xor(s, 32);
    if (g == 0) partial[(int64_t)blockIdx.y * C + c0 + 16 * w + i] = s;
  }
}

}  // namespace

bool transpose_supported(int64_t R, int64_t C) { return R > 0 && C > 0 && R % TR == 0 && C % TC == 0; }

int64_t transpose_partial_rows(int64_t R) { return R / TR; }

void launch_transpose_batched(const void* x, void* y, int L, int64_t R, int C, int64_t ldx, int dt, hipStream_t s) {
  const dim3 grid(C / TC, (unsigned)(R / TR), (unsigned)L);
  DSA_DISPATCH_16(dt, T,
    hipLaunchKernelGGL((transpose_kernel<T, false, kCopy>), grid, dim3(256), 0, s, (const uint16_t*)x, (uint16_t*)y,
                       nullptr, R, C, ldx, nullptr, nullptr, nullptr, 0));
}

void launch_transpose(const void* x, void* y, float* partial, void* colsum_out, int colsum_accum, int64_t R, int C,
                      int64_t ldx, int dt, hipStream_t s) {
  const dim3 grid(C / TC, (unsigned)(R / TR));
  DSA_DISPATCH_16(dt, T,
    if (partial) {
      hipLaunchKernelGGL((transpose_kernel<T, true, kCopy>), grid, dim3(256), 0, s, (const uint16_t*)x, (uint16_t*)y,
                         partial, R, C, ldx, nullptr, nullptr, nullptr, 0);
      launch_colsum_partials(partial, (int)(R / TR), C, colsum_out, colsum_accum, dt, s);
    } else {
      hipLaunchKernelGGL((transpose_kernel<T, false, kCopy>), grid, dim3(256), 0, s, (const uint16_t*)x, (uint16_t*)y,
                         nullptr, R, C, ldx, nullptr, nullptr, nullptr, 0);
    });
}

void launch_bias_gelu_fwd_t(const void* x, const void* b, void* yt, int64_t R, int C, int approx, int dt,
                            hipStream_t s) {
  const dim3 grid(C / TC, (unsigned)(R / TR));
  DSA_DISPATCH_16(dt, T,
    hipLaunchKernelGGL((transpose_kernel<T, false, kGeluFwd>), grid, dim3(256), 0, s, (const uint16_t*)x,
                       (uint16_t*)yt, nullptr, R, C, (int64_t)C, nullptr, (const uint16_t*)b, nullptr, approx));
}

void launch_bias_gelu_bwd_t(const void* dy, const void* x, const void* b, void* dx, void* dxt, float* partial,
                            void* db, int64_t R, int C, int approx, int dt, hipStream_t s) {
  const dim3 grid(C / TC, (unsigned)(R / TR));
  DSA_DISPATCH_16(dt, T,
    if (partial) {
      hipLaunchKernelGGL((transpose_kernel<T, true, kGeluBwd>), grid, dim3(256), 0, s, (const uint16_t*)dy,
                         (uint16_t*)dxt, partial, R, C, (int64_t)C, (const uint16_t*)x, (const uint16_t*)b,
                         (uint16_t*)dx, approx);
      launch_colsum_partials(partial, (int)(R / TR), C, db, 0, dt, s);
    } else {
      hipLaunchKernelGGL((transpose_kernel<T, false, kGeluBwd>), grid, dim3(256), 0, s, (const uint16_t*)dy,
                         (uint16_t*)dxt, nullptr, R, C, (int64_t)C, (const uint16_t*)x, (const uint16_t*)b,
                         (uint16_t*)dx, approx);
    });
}

}  // namespace dsa
