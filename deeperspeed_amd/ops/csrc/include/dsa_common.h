// Shared device helpers for the deeperspeed_amd CDNA4 (gfx950) kernels.
//
// Design rules (MI355X): wave = 64 lanes, block sizes are multiples of 64,
// bf16/fp16 memory traffic is always vectorised to 16 bytes per lane, math is
// done in fp32, reductions use wave64 shuffles then one LDS hop.
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <hip/hip_fp16.h>
#include <stdint.h>

namespace dsa {

constexpr int kWave = 64;

// ---------------------------------------------------------------------------
// dtype tags. The host side passes an integer code; kernels are templated.
// ---------------------------------------------------------------------------
enum DType : int { kF32 = 0, kBF16 = 1, kF16 = 2 };

struct bf16_t { uint16_t x; };
struct f16_t { uint16_t x; };

__device__ __forceinline__ float bf16_to_f32(uint16_t v) {
  return __uint_as_float(((uint32_t)v) << 16);
}
// Round-to-nearest-even; a plain cast lowers to v_cvt_pk_bf16_f32 on gfx950
// and keeps NaNs NaN.
__device__ __forceinline__ uint16_t f32_to_bf16(float f) {
  __hip_bfloat16 h = __float2bfloat16(f);
  return *reinterpret_cast<uint16_t*>(&h);
}
__device__ __forceinline__ float f16_to_f32(uint16_t v) {
  __half h = *reinterpret_cast<__half*>(&v);
  return __half2float(h);
}
__device__ __forceinline__ uint16_t f32_to_f16(float f) {
  __half h = __float2half(f);
  return *reinterpret_cast<uint16_t*>(&h);
}

// GeLU (exact erf, or the tanh approximation) and its derivative, fp32.
// tanh GeLU as x * sigmoid(2u) (0.5 (1 + tanh u) == sigmoid(2u)), u = k0 (x + k1 x^3): one v_exp_f32
// and one v_rcp_f32 instead of libm's tanhf, whose ~25 VALU instructions per element made the
// BERT-Large GeLU kernels VALU-bound (fc1 output 8192 x 4096: 33 us forward, 46 us backward).
// Accurate in both tails: exp overflows to inf for x << 0 and the rcp gives 0.
__device__ __forceinline__ float gelu_sig2u(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f, m2log2e = -2.f * 1.4426950408889634f;
  const float u = k0 * fmaf(k1 * x, x * x, x);
  return __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(m2log2e * u));
}
// exact GeLU's Phi(x) = 0.5 (1 + erf(x / sqrt 2)) from erfc(|z|) ~= q(t) exp(-z^2), t = 1 / (1 + p|z|)
// (Abramowitz & Stegun 7.1.26, |error| <= 1.5e-7): Phi = 1 - q/2 for x >= 0, q/2 below, so neither
// tail cancels; one v_exp_f32 + one v_rcp_f32 + a degree-5 polynomial instead of libm's erff.
// e = exp(-x^2 / 2) is returned for the derivative's pdf.
__device__ __forceinline__ float gelu_phi(float x, float& e) {
  const float z = fabsf(x) * 0.7071067811865476f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, z, 1.f));
  const float q = t * fmaf(t, fmaf(t, fmaf(t, fmaf(t, 1.061405429f, -1.453152027f), 1.421413741f), -0.284496736f),
                           0.254829592f);
  e = __builtin_amdgcn_exp2f(-1.4426950408889634f * z * z);
  const float h = 0.5f * q * e;
  return x >= 0.f ? 1.f - h : h;
}
__device__ __forceinline__ float gelu_f(float x, bool approx) {
  if (approx) return x * gelu_sig2u(x);
  float e;
  return x * gelu_phi(x, e);
}
__device__ __forceinline__ float dgelu_f(float x, bool approx) {
  if (approx) {  // d/dx x s(2u) = s + 2 x s (1 - s) u'
    const float k0 = 0.7978845608028654f, k1 = 0.044715f;
    const float sg = gelu_sig2u(x);
    return fmaf(2.f * x * sg * (1.f - sg), k0 * fmaf(3.f * k1 * x, x, 1.f), sg);
  }
  float e;
  const float cdf = gelu_phi(x, e);
  return fmaf(x * 0.3989422804014327f, e, cdf);  // Phi + x * pdf, pdf = exp(-x^2/2) / sqrt(2 pi)
}

template <typename T> struct Conv;
template <> struct Conv<float> {
  __device__ __forceinline__ static float load(const float* p, int64_t i) { return p[i]; }
  __device__ __forceinline__ static void store(float* p, int64_t i, float v) { p[i] = v; }
};
template <> struct Conv<bf16_t> {
  __device__ __forceinline__ static float load(const bf16_t* p, int64_t i) {
    return bf16_to_f32(p[i].x);
  }
  __device__ __forceinline__ static void store(bf16_t* p, int64_t i, float v) {
    p[i].x = f32_to_bf16(v);
  }
};
template <> struct Conv<f16_t> {
  __device__ __forceinline__ static float load(const f16_t* p, int64_t i) {
    return f16_to_f32(p[i].x);
  }
  __device__ __forceinline__ static void store(f16_t* p, int64_t i, float v) {
    p[i].x = f32_to_f16(v);
  }
};

// 16-byte vector load/store of N elements of T converted to/from fp32.
// N * sizeof(T) must be 16 (8 x 16-bit, or 4 x fp32).
template <typename T> struct Vec16;
template <> struct Vec16<float> {
  static constexpr int N = 4;
  __device__ __forceinline__ static void load(const float* p, float (&o)[4]) {
    float4 v = *reinterpret_cast<const float4*>(p);
    o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w;
  }
  __device__ __forceinline__ static void store(float* p, const float (&o)[4]) {
    *reinterpret_cast<float4*>(p) = make_float4(o[0], o[1], o[2], o[3]);
  }
  // the raw 16-byte vector of o (pack + unpack = the values a store / load round trip yields)
  __device__ __forceinline__ static uint4 pack(const float (&o)[4]) {
    return make_uint4(__float_as_uint(o[0]), __float_as_uint(o[1]), __float_as_uint(o[2]), __float_as_uint(o[3]));
  }
  // the elements of a raw 16-byte vector already in registers (software-pipelined loads)
  __device__ __forceinline__ static void unpack(const uint4& v, float (&o)[4]) {
    o[0] = __uint_as_float(v.x); o[1] = __uint_as_float(v.y); o[2] = __uint_as_float(v.z); o[3] = __uint_as_float(v.w);
  }
};

template <typename T16, float (*TO)(uint16_t), uint16_t (*FROM)(float)>
struct Vec16Half {
  static constexpr int N = 8;
  __device__ __forceinline__ static void load(const T16* p, float (&o)[8]) {
    unpack(*reinterpret_cast<const uint4*>(p), o);
  }
  __device__ __forceinline__ static void unpack(const uint4& v, float (&o)[8]) {
    uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      o[2 * i] = TO((uint16_t)(w[i] & 0xffff));
      o[2 * i + 1] = TO((uint16_t)(w[i] >> 16));
    }
  }
  __device__ __forceinline__ static uint4 pack(const float (&o)[8]) {
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
      w[i] = (uint32_t)FROM(o[2 * i]) | ((uint32_t)FROM(o[2 * i + 1]) << 16);
    return make_uint4(w[0], w[1], w[2], w[3]);
  }
  __device__ __forceinline__ static void store(T16* p, const float (&o)[8]) {
    *reinterpret_cast<uint4*>(p) = pack(o);
  }
};
template <> struct Vec16<bf16_t> : Vec16Half<bf16_t, bf16_to_f32, f32_to_bf16> {};
template <> struct Vec16<f16_t> : Vec16Half<f16_t, f16_to_f32, f32_to_f16> {};

// Generic N-element (N = 4 or 8) vector IO for mixed-dtype elementwise kernels:
// loads N contiguous elements as fp32 irrespective of storage type.
template <typename T, int N>
__device__ __forceinline__ void load_n(const T* p, float (&o)[N]) {
  if constexpr (Vec16<T>::N == N) {
    Vec16<T>::load(p, o);
  } else if constexpr (Vec16<T>::N * 2 == N) {
    float a[N / 2], b[N / 2];
    Vec16<T>::load(p, a);
    Vec16<T>::load(p + N / 2, b);
#pragma unroll
    for (int i = 0; i < N / 2; ++i) { o[i] = a[i]; o[i + N / 2] = b[i]; }
  } else {  // 8-byte half load for 16-bit types with N == 4
    static_assert(N == 4, "unsupported vector width");
    uint2 v = *reinterpret_cast<const uint2*>(p);
    float t[8];
    uint32_t w[2] = {v.x, v.y};
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      t[2 * i] = Conv<T>::load(reinterpret_cast<const T*>(&w[i]), 0);
      t[2 * i + 1] = Conv<T>::load(reinterpret_cast<const T*>(&w[i]), 1);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) o[i] = t[i];
  }
}
template <typename T, int N>
__device__ __forceinline__ void store_n(T* p, const float (&o)[N]) {
  if constexpr (Vec16<T>::N == N) {
    Vec16<T>::store(p, o);
  } else if constexpr (Vec16<T>::N * 2 == N) {
    float a[N / 2], b[N / 2];
#pragma unroll
    for (int i = 0; i < N / 2; ++i) { a[i] = o[i]; b[i] = o[i + N / 2]; }
    Vec16<T>::store(p, a);
    Vec16<T>::store(p + N / 2, b);
  } else {
    static_assert(N == 4, "unsupported vector width");
    uint32_t w[2];
    T* t = reinterpret_cast<T*>(w);
#pragma unroll
    for (int i = 0; i < 4; ++i) Conv<T>::store(t, i, o[i]);
    *reinterpret_cast<uint2*>(p) = make_uint2(w[0], w[1]);
  }
}

// ---------------------------------------------------------------------------
// wave64 / block reductions
// ---------------------------------------------------------------------------
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Sum over the whole block (blockDim.x a multiple of 64, <= 1024). `red` must
// hold >= 16 floats of LDS. Result is broadcast to every thread.
__device__ __forceinline__ float block_sum(float v, float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int nw = blockDim.x >> 6;
  v = wave_sum(v);
  __syncthreads();  // protect `red` reuse across consecutive calls
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float r = 0.f;
  for (int i = 0; i < nw; ++i) r += red[i];
  return r;
}
// Two sums at once (one LDS round trip).
__device__ __forceinline__ void block_sum2(float& a, float& b, float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int nw = blockDim.x >> 6;
  a = wave_sum(a);
  b = wave_sum(b);
  __syncthreads();
  if (lane == 0) { red[wid] = a; red[16 + wid] = b; }
  __syncthreads();
  float ra = 0.f, rb = 0.f;
  for (int i = 0; i < nw; ++i) { ra += red[i]; rb += red[16 + i]; }
  a = ra; b = rb;
}

// Bijective XCD-aware remap of a flat block id (cdna_hip_programming T1): blocks
// dealt round-robin over the 8 XCDs are renumbered so that each XCD receives
// a contiguous range of logical tiles (neighbouring tiles share its L2).
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  constexpr int NX = 8;
  if (nwg < NX) return orig;
  const int q = nwg / NX, r = nwg % NX;
  const int xcd = orig % NX, idx = orig / NX;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

}  // namespace dsa

#define DSA_CHECK_LAUNCH() (void)hipGetLastError()

// dtype-code -> type dispatch for host launchers (codes: DType above)
#define DSA_DISPATCH_T(code, T, ...)                      \
  switch (code) {                                          \
    case dsa::kF32: { using T = float; __VA_ARGS__; } break;    \
    case dsa::kBF16: { using T = dsa::bf16_t; __VA_ARGS__; } break;  \
    case dsa::kF16: { using T = dsa::f16_t; __VA_ARGS__; } break;    \
    default: break;                                        \
  }

#define DSA_DISPATCH_16(code, T, ...)                      \
  switch (code) {                                          \
    case dsa::kBF16: { using T = dsa::bf16_t; __VA_ARGS__; } break;  \
    case dsa::kF16: { using T = dsa::f16_t; __VA_ARGS__; } break;    \
    default: break;                                        \
  }
