// Fused optimizer kernels for CDNA4: Adam/AdamW (flat + multi-tensor), LAMB,
// fused grad-norm / overflow reductions, scaled copies.
//
// Parity targets: the reference's multi-tensor Adam (csrc/adam/multi_tensor_adam.cu:18-128,
// L2 vs decoupled weight decay) and fused LAMB (csrc/lamb/fused_lamb_cuda_kernel.cu:185-310).
// Design here is MI355X-first: ZeRO keeps each parameter group as one flat,
// 256-byte aligned arena, so the hot path is a single grid-stride launch over a
// flat shard with 16-byte vector IO, fp32 state, and an optional bf16/fp16 model
// copy written in the same pass (no separate cast kernel).
#include "../include/dsa_common.h"
#include "../include/launchers.h"

namespace dsa {

// AdamArgs (launchers.h): bc1/bc2 = 1 - beta^t (1 without bias correction);
// grad_scale multiplies incoming grads (1/loss_scale * clip coefficient);
// adamw = 1 decoupled weight decay, 0 = L2 added to the gradient.

__device__ __forceinline__ void adam_elem(float& w, float g, float& m, float& v, const AdamArgs& a) {
  g *= a.grad_scale;
  if (!a.adamw && a.weight_decay != 0.f) g = fmaf(a.weight_decay, w, g);
  m = fmaf(a.beta1, m, (1.f - a.beta1) * g);
  v = fmaf(a.beta2, v, (1.f - a.beta2) * g * g);
  const float denom = sqrtf(v / a.bc2) + a.eps;
  float upd = (m / a.bc1) / denom;
  if (a.adamw && a.weight_decay != 0.f) upd = fmaf(a.weight_decay, w, upd);
  w = fmaf(-a.lr, upd, w);
}

// W  : storage of the weights being updated (fp32 master, or the param itself)
// TG : gradient storage
// TO : optional low-precision model copy written after the update (may be null)
template <typename TW, typename TG, typename TO>
__global__ void __launch_bounds__(256) adam_flat_kernel(TW* __restrict__ w, const TG* __restrict__ g,
                                                        float* __restrict__ m, float* __restrict__ v,
                                                        TO* __restrict__ out, int64_t n, AdamArgs a) {
  const int64_t nvec = n / 4;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nvec; i += stride) {
    const int64_t e = i * 4;
    float wf[4], gf[4], mf[4], vf[4];
    load_n<TW, 4>(w + e, wf);
    load_n<TG, 4>(g + e, gf);
    load_n<float, 4>(m + e, mf);
    load_n<float, 4>(v + e, vf);
#pragma unroll
    for (int k = 0; k < 4; ++k) adam_elem(wf[k], gf[k], mf[k], vf[k], a);
    store_n<TW, 4>(w + e, wf);
    store_n<float, 4>(m + e, mf);
    store_n<float, 4>(v + e, vf);
    if (out) store_n<TO, 4>(out + e, wf);
  }
  // tail (n % 4 elements) handled by block 0
  if (blockIdx.x == 0) {
    for (int64_t e = nvec * 4 + threadIdx.x; e < n; e += blockDim.x) {
      float wf = Conv<TW>::load(w, e), gf = Conv<TG>::load(g, e), mf = m[e], vf = v[e];
      adam_elem(wf, gf, mf, vf, a);
      Conv<TW>::store(w, e, wf);
      m[e] = mf; v[e] = vf;
      if (out) Conv<TO>::store(out, e, wf);
    }
  }
}

// Compact fp32 master: the master is held EXACTLY as (bf16 high half, int16 residual):
//   bits(master) = (hi << 16) + residual,  hi = (bits + 0x8000) >> 16  (round half away on the
//   magnitude, i.e. RNE except on exact ties), residual in [-32768, 32767].
// The bf16 high half IS the model weight, so the fp32 master costs 2 B/param instead of 4.
__device__ __forceinline__ float compact_decode(uint16_t hi, int16_t r) {
  return __uint_as_float((uint32_t)((int32_t)((uint32_t)hi << 16) + (int32_t)r));
}
__device__ __forceinline__ void compact_encode(float f, uint16_t& hi, int16_t& r) {
  const uint32_t b = __float_as_uint(f);
  const uint32_t h = (b + 0x8000u) >> 16;
  hi = (uint16_t)h;
  r = (int16_t)(int32_t)(b - (h << 16));
}

template <typename TG>
__global__ void __launch_bounds__(256) adam_compact_kernel(uint16_t* __restrict__ hi, int16_t* __restrict__ res,
                                                           const TG* __restrict__ g, float* __restrict__ m,
                                                           float* __restrict__ v, int64_t n, AdamArgs a) {
  const int64_t nvec = n / 4;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nvec; i += stride) {
    const int64_t e = i * 4;
    const ushort4 h4 = *reinterpret_cast<const ushort4*>(hi + e);
    const short4 r4 = *reinterpret_cast<const short4*>(res + e);
    float wf[4] = {compact_decode(h4.x, r4.x), compact_decode(h4.y, r4.y), compact_decode(h4.z, r4.z),
                   compact_decode(h4.w, r4.w)};
    float gf[4], mf[4], vf[4];
    load_n<TG, 4>(g + e, gf);
    load_n<float, 4>(m + e, mf);
    load_n<float, 4>(v + e, vf);
#pragma unroll
    for (int k = 0; k < 4; ++k) adam_elem(wf[k], gf[k], mf[k], vf[k], a);
    ushort4 ho;
    short4 ro;
    compact_encode(wf[0], ho.x, ro.x);
    compact_encode(wf[1], ho.y, ro.y);
    compact_encode(wf[2], ho.z, ro.z);
    compact_encode(wf[3], ho.w, ro.w);
    *reinterpret_cast<ushort4*>(hi + e) = ho;
    *reinterpret_cast<short4*>(res + e) = ro;
    store_n<float, 4>(m + e, mf);
    store_n<float, 4>(v + e, vf);
  }
  if (blockIdx.x == 0) {
    for (int64_t e = nvec * 4 + threadIdx.x; e < n; e += blockDim.x) {
      float wf = compact_decode(hi[e], res[e]), gf = Conv<TG>::load(g, e), mf = m[e], vf = v[e];
      adam_elem(wf, gf, mf, vf, a);
      compact_encode(wf, hi[e], res[e]);
      m[e] = mf; v[e] = vf;
    }
  }
}

// Multi-tensor form: one launch covers a list of (possibly unaligned) tensors.
// `meta` is a device int64 table:
//   [0,T) w ptrs, [T,2T) g ptrs, [2T,3T) m ptrs, [3T,4T) v ptrs, [4T,5T) out ptrs,
//   [5T,6T) numel, [6T,7T+1) chunk prefix (chunks of `chunk` elements)
template <typename TW, typename TG, typename TO>
__global__ void __launch_bounds__(256) adam_multi_kernel(const int64_t* __restrict__ meta, int T,
                                                         int64_t chunk, AdamArgs a) {
  const int64_t* pref = meta + 6 * T;
  const int64_t c = blockIdx.x;
  int lo = 0, hi = T - 1;
  while (lo < hi) {  // last t with pref[t] <= c
    int mid = (lo + hi + 1) >> 1;
    if (pref[mid] <= c) lo = mid; else hi = mid - 1;
  }
  const int t = lo;
  TW* w = reinterpret_cast<TW*>(meta[t]);
  const TG* g = reinterpret_cast<const TG*>(meta[T + t]);
  float* m = reinterpret_cast<float*>(meta[2 * T + t]);
  float* v = reinterpret_cast<float*>(meta[3 * T + t]);
  TO* out = reinterpret_cast<TO*>(meta[4 * T + t]);
  const int64_t n = meta[5 * T + t];
  const int64_t start = (c - pref[t]) * chunk;
  const int64_t end = start + chunk < n ? start + chunk : n;
  for (int64_t e = start + threadIdx.x; e < end; e += blockDim.x) {
    float wf = Conv<TW>::load(w, e), gf = Conv<TG>::load(g, e), mf = m[e], vf = v[e];
    adam_elem(wf, gf, mf, vf, a);
    Conv<TW>::store(w, e, wf);
    m[e] = mf; v[e] = vf;
    if (out) Conv<TO>::store(out, e, wf);
  }
}

// ---------------------------------------------------------------------------
// Sum of squares (fp32 accumulate) over a flat tensor; partials per block then
// a one-block finish. NaN/Inf propagate into the result (overflow detection).
// ---------------------------------------------------------------------------
template <typename T>
__global__ void __launch_bounds__(256) sumsq_partial_kernel(const T* __restrict__ x, int64_t n,
                                                            float* __restrict__ partial) {
  __shared__ float red[32];
  float acc = 0.f;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  constexpr int N = Vec16<T>::N;
  const int64_t nvec = n / N;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nvec; i += stride) {
    float f[N];
    Vec16<T>::load(x + i * N, f);
#pragma unroll
    for (int k = 0; k < N; ++k) acc = fmaf(f[k], f[k], acc);
  }
  if (blockIdx.x == 0)
    for (int64_t e = nvec * N + threadIdx.x; e < n; e += blockDim.x) {
      float f = Conv<T>::load(x, e);
      acc = fmaf(f, f, acc);
    }
  acc = block_sum(acc, red);
  if (threadIdx.x == 0) partial[blockIdx.x] = acc;
}

// Accumulates (adds) the finished sum into out[0] so several tensors can share one
// result slot without host syncs.
__global__ void __launch_bounds__(256) sum_finish_kernel(const float* __restrict__ partial, int n,
                                                         float* __restrict__ out) {
  __shared__ float red[32];
  float acc = 0.f;
  for (int i = threadIdx.x; i < n; i += blockDim.x) acc += partial[i];
  acc = block_sum(acc, red);
  if (threadIdx.x == 0) out[0] += acc;
}

// Multi-tensor sum of squares (the global gradient norm of a per-tensor optimizer): one block per
// `chunk` elements of one tensor (meta = [T pointers | T numels | T+1 chunk prefix], the layout of
// the multi-tensor LAMB), fp32 partial per block, reduced by sum_finish_kernel.  Replaces torch's
// _foreach_norm (one multi_tensor_apply launch per ~100 tensors plus stack / square / sum kernels).
template <typename T>
__global__ void __launch_bounds__(256) sumsq_multi_kernel(const int64_t* __restrict__ meta, int nt, int64_t chunk,
                                                          float* __restrict__ partial) {
  __shared__ float red[32];
  const int64_t* pref = meta + 2 * nt;
  const int64_t c = blockIdx.x;
  int lo = 0, hi = nt - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (pref[mid] <= c) lo = mid; else hi = mid - 1;
  }
  const T* x = reinterpret_cast<const T*>(meta[lo]);
  const int64_t n = meta[nt + lo];
  const int64_t start = (c - pref[lo]) * chunk;
  const int64_t end = start + chunk < n ? start + chunk : n;
  float acc = 0.f;
  constexpr int N = Vec16<T>::N;
  int64_t e0 = start;
  if ((reinterpret_cast<uintptr_t>(x + start) & 15) == 0) {
    const int64_t vend = start + ((end - start) / N) * N;
    for (int64_t e = start + (int64_t)N * threadIdx.x; e < vend; e += (int64_t)N * blockDim.x) {
      float f[N];
      Vec16<T>::load(x + e, f);
#pragma unroll
      for (int k = 0; k < N; ++k) acc = fmaf(f[k], f[k], acc);
    }
    e0 = vend;
  }
  for (int64_t e = e0 + threadIdx.x; e < end; e += blockDim.x) {
    const float f = Conv<T>::load(x, e);
    acc = fmaf(f, f, acc);
  }
  acc = block_sum(acc, red);
  if (threadIdx.x == 0) partial[c] = acc;
}

void launch_sumsq_multi(const int64_t* meta, int nt, int64_t total_chunks, int64_t chunk, int xt, float* partial,
                        float* out, hipStream_t s) {
  if (total_chunks <= 0) return;
  DSA_DISPATCH_T(xt, T,
    hipLaunchKernelGGL((sumsq_multi_kernel<T>), dim3((unsigned)total_chunks), dim3(256), 0, s, meta, nt, chunk,
                       partial));
  hipLaunchKernelGGL(sum_finish_kernel, dim3(1), dim3(256), 0, s, partial, (int)total_chunks, out);
}

// Byte copy on a few workgroups, for HBM -> pinned host memory: ROCclr runs such copies as a blit
// kernel with a workgroup on EVERY CU (profiles/r4p_*), whichever hipMemcpyKind is given, and the
// PCIe link (~50 GB/s) is the bound either way.  Each thread keeps 4 16-byte loads in flight before
// its stores so 16-32 workgroups reach the link rate; the rest of the chip stays with the compute.
__global__ void __launch_bounds__(256) copy_narrow_kernel(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                                          int64_t n16) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + 3 * stride < n16; i += 4 * stride) {
    const uint4 a = src[i], b = src[i + stride], c = src[i + 2 * stride], d = src[i + 3 * stride];
    dst[i] = a;
    dst[i + stride] = b;
    dst[i + 2 * stride] = c;
    dst[i + 3 * stride] = d;
  }
  for (; i < n16; i += stride) dst[i] = src[i];
}

__global__ void copy_tail_kernel(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = src[i];
}

void launch_copy_narrow(const void* src, void* dst, int64_t bytes, int wgs, hipStream_t s) {
  if (bytes <= 0) return;
  const int64_t n16 = bytes / 16;
  if (n16 > 0)
    hipLaunchKernelGGL(copy_narrow_kernel, dim3(wgs), dim3(256), 0, s, (const uint4*)src, (uint4*)dst, n16);
  const int64_t tail = bytes - n16 * 16;
  if (tail > 0)
    hipLaunchKernelGGL(copy_tail_kernel, dim3(1), dim3(64), 0, s, (const uint8_t*)src + n16 * 16,
                       (uint8_t*)dst + n16 * 16, tail);
}

// y = x * scale, or y += x * scale (ACC: e.g. a bf16 micro-batch gradient accumulated into an
// fp32 shard in one pass instead of a cast kernel plus an add kernel); mixed dtypes
template <typename TI, typename TO, bool ACC>
__global__ void __launch_bounds__(256) scale_copy_kernel(const TI* __restrict__ x, TO* __restrict__ y,
                                                         int64_t n, const float* __restrict__ scale_ptr,
                                                         float scale) {
  const float s = scale_ptr ? scale * scale_ptr[0] : scale;
  const int64_t nvec = n / 4;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nvec; i += stride) {
    float f[4];
    load_n<TI, 4>(x + i * 4, f);
    if constexpr (ACC) {
      float o[4];
      load_n<TO, 4>(y + i * 4, o);
#pragma unroll
      for (int k = 0; k < 4; ++k) f[k] = o[k] + f[k] * s;
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) f[k] *= s;
    }
    store_n<TO, 4>(y + i * 4, f);
  }
  if (blockIdx.x == 0)
    for (int64_t e = nvec * 4 + threadIdx.x; e < n; e += blockDim.x)
      Conv<TO>::store(y, e, (ACC ? Conv<TO>::load(y, e) : 0.f) + Conv<TI>::load(x, e) * s);
}

// ---------------------------------------------------------------------------
// LAMB (per-tensor trust ratio). Stage 1: moments + update direction u written
// into `upd` (fp32) and per-block partial ||w||^2, ||u||^2. Stage 2 (finish): one
// block reduces partials and computes the clamped trust ratio. Stage 3: apply.
// Mirrors the 3-kernel structure of csrc/lamb/fused_lamb_cuda_kernel.cu:185-310 but
// with wave64 reductions and a device-resident coefficient (no host sync).
// ---------------------------------------------------------------------------
// LambArgs (launchers.h): adamw = 1 puts eps outside the sqrt (reference eps_mode 1), lr is the
// bias-corrected step size lr*sqrt(bc2)/bc1 and grad_scale the inverse loss scale.

template <typename TW, typename TG>
__global__ void __launch_bounds__(256) lamb_stage1_kernel(const TW* __restrict__ w, const TG* __restrict__ g,
                                                          float* __restrict__ m, float* __restrict__ v,
                                                          float* __restrict__ upd, int64_t n, LambArgs a,
                                                          float* __restrict__ partial /*2*gridDim*/) {
  __shared__ float red[32];
  float sw = 0.f, su = 0.f;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += stride) {
    float wf = Conv<TW>::load(w, e);
    float gf = Conv<TG>::load(g, e) * a.grad_scale;
    float mf = fmaf(a.beta1, m[e], (1.f - a.beta1) * gf);
    float vf = fmaf(a.beta2, v[e], (1.f - a.beta2) * gf * gf);
    m[e] = mf; v[e] = vf;
    // LAMB update direction (reference fused_lamb_cuda_kernel.cu:185-230): no bias correction
    // inside u (it is folded into the step size), eps outside (adamw=1) or inside the sqrt
    const float denom = a.adamw ? sqrtf(vf) + a.eps : sqrtf(vf + a.eps);
    const float u = mf / denom + a.weight_decay * wf;
    upd[e] = u;
    sw = fmaf(wf, wf, sw);
    su = fmaf(u, u, su);
  }
  block_sum2(sw, su, red);
  if (threadIdx.x == 0) { partial[2 * blockIdx.x] = sw; partial[2 * blockIdx.x + 1] = su; }
}

__global__ void __launch_bounds__(256) lamb_finish_kernel(const float* __restrict__ partial, int nb,
                                                          LambArgs a, float* __restrict__ coeff_out) {
  __shared__ float red[32];
  float sw = 0.f, su = 0.f;
  for (int i = threadIdx.x; i < nb; i += blockDim.x) { sw += partial[2 * i]; su += partial[2 * i + 1]; }
  block_sum2(sw, su, red);
  if (threadIdx.x == 0) {
    const float wn = sqrtf(sw), un = sqrtf(su);
    float c = 1.f;
    if (wn > 0.f && un > 0.f) c = fminf(fmaxf(wn / un, a.min_coeff), a.max_coeff);
    coeff_out[0] = c;
  }
}

template <typename TW, typename TO>
__global__ void __launch_bounds__(256) lamb_apply_kernel(TW* __restrict__ w, const float* __restrict__ upd,
                                                         int64_t n, float lr, const float* __restrict__ coeff,
                                                         TO* __restrict__ out) {
  const float s = lr * coeff[0];
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += stride) {
    float wf = Conv<TW>::load(w, e) - s * upd[e];
    Conv<TW>::store(w, e, wf);
    if (out) Conv<TO>::store(out, e, wf);
  }
}

// 4 consecutive elements as one vector access (16 bytes fp32, 8 bytes 16-bit)
template <typename T> struct V4;
template <> struct V4<float> {
  __device__ __forceinline__ static void load(const float* p, float* f) {
    const float4 x = *reinterpret_cast<const float4*>(p);
    f[0] = x.x; f[1] = x.y; f[2] = x.z; f[3] = x.w;
  }
  __device__ __forceinline__ static void store(float* p, const float* f) {
    *reinterpret_cast<float4*>(p) = make_float4(f[0], f[1], f[2], f[3]);
  }
};
template <typename T, float (*LD)(uint16_t), uint16_t (*ST)(float)>
struct V4Half {
  __device__ __forceinline__ static void load(const T* p, float* f) {
    const uint2 x = *reinterpret_cast<const uint2*>(p);
    f[0] = LD(x.x & 0xffff); f[1] = LD(x.x >> 16); f[2] = LD(x.y & 0xffff); f[3] = LD(x.y >> 16);
  }
  __device__ __forceinline__ static void store(T* p, const float* f) {
    *reinterpret_cast<uint2*>(p) = make_uint2((uint32_t)ST(f[0]) | ((uint32_t)ST(f[1]) << 16),
                                              (uint32_t)ST(f[2]) | ((uint32_t)ST(f[3]) << 16));
  }
};
template <> struct V4<bf16_t> : V4Half<bf16_t, bf16_to_f32, f32_to_bf16> {};
template <> struct V4<f16_t> : V4Half<f16_t, f16_to_f32, f32_to_f16> {};

template <typename... P>
__device__ __forceinline__ bool aligned16(const P*... p) {
  return ((reinterpret_cast<uintptr_t>(p) | ...) & 15) == 0;
}

// Multi-tensor LAMB: the whole parameter list in three launches (meta table as adam_multi:
// w, g, m, v, out pointers, numel, chunk prefix).  Stage 1 writes per-chunk partial ||w||^2,
// ||u||^2; finish reduces each tensor's chunks to its clamped trust ratio; apply recomputes
// u from the updated moments (no fp32 scratch for u) and steps w.
template <typename TW, typename TG>
__global__ void __launch_bounds__(256) lamb_multi_stage1_kernel(const int64_t* __restrict__ meta, int T,
                                                                int64_t chunk, LambArgs a,
                                                                float* __restrict__ partial) {
  __shared__ float red[32];
  const int64_t* pref = meta + 6 * T;
  const int64_t c = blockIdx.x;
  int lo = 0, hi = T - 1;
  while (lo < hi) {
    int mid = (lo + hi + 1) >> 1;
    if (pref[mid] <= c) lo = mid; else hi = mid - 1;
  }
  const int t = lo;
  const TW* w = reinterpret_cast<const TW*>(meta[t]);
  const TG* g = reinterpret_cast<const TG*>(meta[T + t]);
  float* m = reinterpret_cast<float*>(meta[2 * T + t]);
  float* v = reinterpret_cast<float*>(meta[3 * T + t]);
  const int64_t n = meta[5 * T + t];
  const int64_t start = (c - pref[t]) * chunk;
  const int64_t end = start + chunk < n ? start + chunk : n;
  float sw = 0.f, su = 0.f;
  float gscale = a.grad_scale;
  if (a.scale_ptr) {
    gscale *= *a.scale_ptr;
    if (!isfinite(gscale)) {  // skipped step: moments untouched
      if (threadIdx.x == 0) { partial[2 * c] = 0.f; partial[2 * c + 1] = 0.f; }
      return;
    }
  }
  auto elem = [&](float wf, float gf, float& mf, float& vf) {
    gf *= gscale;
    mf = fmaf(a.beta1, mf, (1.f - a.beta1) * gf);
    vf = fmaf(a.beta2, vf, (1.f - a.beta2) * gf * gf);
    const float denom = a.adamw ? sqrtf(vf) + a.eps : sqrtf(vf + a.eps);
    const float u = mf / denom + a.weight_decay * wf;
    sw = fmaf(wf, wf, sw);
    su = fmaf(u, u, su);
  };
  // 4-wide vector body when every stream is 16-byte aligned (always for whole allocations)
  int64_t e0 = start;
  if (aligned16(w, g, m, v)) {
    const int64_t vend = start + ((end - start) & ~(int64_t)3);
    for (int64_t e = start + 4 * threadIdx.x; e < vend; e += 4 * blockDim.x) {
      float wf[4], gf[4];
      V4<TW>::load(w + e, wf);
      V4<TG>::load(g + e, gf);
      float4 mm = *reinterpret_cast<const float4*>(m + e), vv = *reinterpret_cast<const float4*>(v + e);
      elem(wf[0], gf[0], mm.x, vv.x);
      elem(wf[1], gf[1], mm.y, vv.y);
      elem(wf[2], gf[2], mm.z, vv.z);
      elem(wf[3], gf[3], mm.w, vv.w);
      *reinterpret_cast<float4*>(m + e) = mm;
      *reinterpret_cast<float4*>(v + e) = vv;
    }
    e0 = vend;
  }
  for (int64_t e = e0 + threadIdx.x; e < end; e += blockDim.x) {
    float mf = m[e], vf = v[e];
    elem(Conv<TW>::load(w, e), Conv<TG>::load(g, e), mf, vf);
    m[e] = mf; v[e] = vf;
  }
  block_sum2(sw, su, red);
  if (threadIdx.x == 0) { partial[2 * c] = sw; partial[2 * c + 1] = su; }
}

__global__ void __launch_bounds__(256) lamb_multi_finish_kernel(const int64_t* __restrict__ meta, int T,
                                                                const float* __restrict__ partial, LambArgs a,
                                                                float* __restrict__ coeff) {
  __shared__ float red[32];
  const int64_t* pref = meta + 6 * T;
  const int t = blockIdx.x;
  float sw = 0.f, su = 0.f;
  for (int64_t c = pref[t] + threadIdx.x; c < pref[t + 1]; c += blockDim.x) {
    sw += partial[2 * c];
    su += partial[2 * c + 1];
  }
  block_sum2(sw, su, red);
  if (threadIdx.x == 0) {
    const float wn = sqrtf(sw), un = sqrtf(su);
    float cf = 1.f;
    if (wn > 0.f && un > 0.f) cf = fminf(fmaxf(wn / un, a.min_coeff), a.max_coeff);
    coeff[t] = cf;
  }
}

template <typename TW, typename TO>
__global__ void __launch_bounds__(256) lamb_multi_apply_kernel(const int64_t* __restrict__ meta, int T,
                                                               int64_t chunk, LambArgs a,
                                                               const float* __restrict__ coeff) {
  const int64_t* pref = meta + 6 * T;
  const int64_t c = blockIdx.x;
  int lo = 0, hi = T - 1;
  while (lo < hi) {
    int mid = (lo + hi + 1) >> 1;
    if (pref[mid] <= c) lo = mid; else hi = mid - 1;
  }
  const int t = lo;
  TW* w = reinterpret_cast<TW*>(meta[t]);
  const float* m = reinterpret_cast<const float*>(meta[2 * T + t]);
  const float* v = reinterpret_cast<const float*>(meta[3 * T + t]);
  TO* out = reinterpret_cast<TO*>(meta[4 * T + t]);
  const int64_t n = meta[5 * T + t];
  const int64_t start = (c - pref[t]) * chunk;
  const int64_t end = start + chunk < n ? start + chunk : n;
  if (a.scale_ptr && !isfinite(a.grad_scale * *a.scale_ptr)) return;  // skipped step
  const float s = (a.lr_ptr ? *a.lr_ptr : a.lr) * coeff[t];
  auto step = [&](float wf, float mf, float vf) {
    const float denom = a.adamw ? sqrtf(vf) + a.eps : sqrtf(vf + a.eps);
    return wf - s * (mf / denom + a.weight_decay * wf);
  };
  int64_t e0 = start;
  if (aligned16(w, m, v, out)) {
    const int64_t vend = start + ((end - start) & ~(int64_t)3);
    for (int64_t e = start + 4 * threadIdx.x; e < vend; e += 4 * blockDim.x) {
      float wf[4];
      V4<TW>::load(w + e, wf);
      const float4 mm = *reinterpret_cast<const float4*>(m + e), vv = *reinterpret_cast<const float4*>(v + e);
      wf[0] = step(wf[0], mm.x, vv.x);
      wf[1] = step(wf[1], mm.y, vv.y);
      wf[2] = step(wf[2], mm.z, vv.z);
      wf[3] = step(wf[3], mm.w, vv.w);
      V4<TW>::store(w + e, wf);
      if (out) V4<TO>::store(out + e, wf);
    }
    e0 = vend;
  }
  for (int64_t e = e0 + threadIdx.x; e < end; e += blockDim.x) {
    const float nw = step(Conv<TW>::load(w, e), m[e], v[e]);
    Conv<TW>::store(w, e, nw);
    if (out) Conv<TO>::store(out, e, nw);
  }
}

// ---------------------------------------------------------------------------
// Host launchers (called from bindings.cpp)
// ---------------------------------------------------------------------------
static inline int grid_for(int64_t work, int block = 256, int cap = 2048) {
  int64_t g = (work + block - 1) / block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (int)g;
}


void launch_adam_flat(void* w, int wt, const void* g, int gt, float* m, float* v, void* out, int ot,
                      int64_t n, AdamArgs a, hipStream_t s) {
  const int grid = grid_for(n / 4, 256, 4096);
  DSA_DISPATCH_T(wt, TW, DSA_DISPATCH_T(gt, TG, DSA_DISPATCH_T(ot, TO,
    hipLaunchKernelGGL((adam_flat_kernel<TW, TG, TO>), dim3(grid), dim3(256), 0, s,
                       (TW*)w, (const TG*)g, m, v, (TO*)out, n, a))));
}

void launch_adam_compact(void* hi, void* res, const void* g, int gt, float* m, float* v, int64_t n, AdamArgs a,
                         hipStream_t s) {
  const int grid = grid_for(n / 4, 256, 4096);
  DSA_DISPATCH_T(gt, TG,
    hipLaunchKernelGGL((adam_compact_kernel<TG>), dim3(grid), dim3(256), 0, s, (uint16_t*)hi, (int16_t*)res,
                       (const TG*)g, m, v, n, a));
}

void launch_adam_multi(const int64_t* meta, int T, int64_t total_chunks, int64_t chunk, int wt, int gt,
                       int ot, AdamArgs a, hipStream_t s) {
  if (total_chunks <= 0) return;
  DSA_DISPATCH_T(wt, TW, DSA_DISPATCH_T(gt, TG, DSA_DISPATCH_T(ot, TO,
    hipLaunchKernelGGL((adam_multi_kernel<TW, TG, TO>), dim3((unsigned)total_chunks), dim3(256), 0, s,
                       meta, T, chunk, a))));
}

// out[0] += sum(x^2); workspace must hold >= 1024 floats.
void launch_sumsq_accum(const void* x, int xt, int64_t n, float* workspace, float* out, hipStream_t s) {
  if (n <= 0) return;
  const int grid = grid_for(n / 8, 256, 1024);
  DSA_DISPATCH_T(xt, T,
    hipLaunchKernelGGL((sumsq_partial_kernel<T>), dim3(grid), dim3(256), 0, s, (const T*)x, n, workspace));
  hipLaunchKernelGGL(sum_finish_kernel, dim3(1), dim3(256), 0, s, workspace, grid, out);
}

void launch_scale_copy(const void* x, int xt, void* y, int yt, int64_t n, const float* scale_ptr,
                       float scale, hipStream_t s, int accumulate) {
  if (n <= 0) return;
  const int grid = grid_for(n / 4, 256, 4096);
  DSA_DISPATCH_T(xt, TI, DSA_DISPATCH_T(yt, TO,
    if (accumulate)
      hipLaunchKernelGGL((scale_copy_kernel<TI, TO, true>), dim3(grid), dim3(256), 0, s,
                         (const TI*)x, (TO*)y, n, scale_ptr, scale);
    else
      hipLaunchKernelGGL((scale_copy_kernel<TI, TO, false>), dim3(grid), dim3(256), 0, s,
                         (const TI*)x, (TO*)y, n, scale_ptr, scale)));
}

// workspace: >= 2*1024 + 1 floats; upd: n floats
void launch_lamb(void* w, int wt, const void* g, int gt, float* m, float* v, float* upd, void* out, int ot,
                 int64_t n, LambArgs a, float* workspace, float* coeff_out, hipStream_t s) {
  if (n <= 0) return;
  const int grid = grid_for(n, 256, 1024);
  DSA_DISPATCH_T(wt, TW, DSA_DISPATCH_T(gt, TG,
    hipLaunchKernelGGL((lamb_stage1_kernel<TW, TG>), dim3(grid), dim3(256), 0, s,
                       (const TW*)w, (const TG*)g, m, v, upd, n, a, workspace)));
  hipLaunchKernelGGL(lamb_finish_kernel, dim3(1), dim3(256), 0, s, workspace, grid, a, coeff_out);
  DSA_DISPATCH_T(wt, TW, DSA_DISPATCH_T(ot, TO,
    hipLaunchKernelGGL((lamb_apply_kernel<TW, TO>), dim3(grid_for(n, 256, 4096)), dim3(256), 0, s,
                       (TW*)w, upd, n, a.lr, coeff_out, (TO*)out)));
}

// partial: 2 * total_chunks floats; coeff: T floats (device-resident trust ratios)
void launch_lamb_multi(const int64_t* meta, int T, int64_t total_chunks, int64_t chunk, int wt, int gt, int ot,
                       LambArgs a, float* partial, float* coeff, hipStream_t s) {
  if (total_chunks <= 0 || T <= 0) return;
  DSA_DISPATCH_T(wt, TW, DSA_DISPATCH_T(gt, TG,
    hipLaunchKernelGGL((lamb_multi_stage1_kernel<TW, TG>), dim3((unsigned)total_chunks), dim3(256), 0, s,
                       meta, T, chunk, a, partial)));
  hipLaunchKernelGGL(lamb_multi_finish_kernel, dim3((unsigned)T), dim3(256), 0, s, meta, T, partial, a, coeff);
  DSA_DISPATCH_T(wt, TW, DSA_DISPATCH_T(ot, TO,
    hipLaunchKernelGGL((lamb_multi_apply_kernel<TW, TO>), dim3((unsigned)total_chunks), dim3(256), 0, s,
                       meta, T, chunk, a, coeff)));
}

}  // namespace dsa
