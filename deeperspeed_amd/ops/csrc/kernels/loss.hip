// Fused softmax cross-entropy on 16-bit logits (the LM head loss).
//
// The reference computes the loss in fp32 through framework ops (logits.float() ->
// log_softmax -> nll), keeping two fp32 copies of a [tokens, vocab] tensor alive; here
// forward reads the bf16 logits once (online max/sum per thread, one block per row) and
// saves only the per-row logsumexp, and backward writes the 16-bit logit gradient directly:
//   dlogit_j = (exp(x_j - lse) - [j == target]) * dloss_row.
// Rows whose label is negative (ignore_index) get zero loss and zero gradient.
#include "../include/dsa_common.h"
#include "../include/launchers.h"

namespace dsa {

template <typename T>
__global__ void __launch_bounds__(256) xent_fwd_kernel(const T* __restrict__ x, const int64_t* __restrict__ labels,
                                                       float* __restrict__ loss, float* __restrict__ lse_out, int V) {
  const int64_t row = blockIdx.x;
  const T* xr = x + row * (int64_t)V;
  float m = -INFINITY, s = 0.f;
  const int nvec = V / 8;
  for (int c = threadIdx.x; c < nvec; c += blockDim.x) {
    float f[8];
    Vec16<T>::load(xr + c * 8, f);
    float mm = f[0];
#pragma unroll
    for (int j = 1; j < 8; ++j) mm = fmaxf(mm, f[j]);
    const float mn = fmaxf(m, mm);
    s = s * __expf(m - mn);
#pragma unroll
    for (int j = 0; j < 8; ++j) s += __expf(f[j] - mn);
    m = mn;
  }
  for (int j = nvec * 8 + threadIdx.x; j < V; j += blockDim.x) {
    const float f = Conv<T>::load(xr, j);
    const float mn = fmaxf(m, f);
    s = s * __expf(m - mn) + __expf(f - mn);
    m = mn;
  }
  // block combine of (m, s)
  __shared__ float sm[8], ss[8];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  float wm = wave_max(m);
  s = (m == -INFINITY) ? 0.f : s * __expf(m - wm);
  s = wave_sum(s);
  if (lane == 0) { sm[w] = wm; ss[w] = s; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float M = sm[0];
    for (int i = 1; i < (int)(blockDim.x >> 6); ++i) M = fmaxf(M, sm[i]);
    float S = 0.f;
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) S += ss[i] * __expf(sm[i] - M);
    const float l = M + __logf(S);
    lse_out[row] = l;
    const int64_t t = labels[row];
    loss[row] = (t >= 0 && t < V) ? l - Conv<T>::load(xr, t) : 0.f;
  }
}

// x and dx may alias (in-place backward): every element is loaded and stored by the same thread
template <typename T>
__global__ void __launch_bounds__(256) xent_bwd_kernel(const T* x, const int64_t* __restrict__ labels,
                                                       const float* __restrict__ lse, const float* __restrict__ dloss,
                                                       int64_t dloss_stride, T* dx, int V) {
  const int64_t row = blockIdx.x;
  const T* xr = x + row * (int64_t)V;
  T* dr = dx + row * (int64_t)V;
  const int64_t t = labels[row];
  const float g = (t >= 0) ? dloss[dloss_stride ? row : 0] : 0.f;
  const float l = lse[row];
  const int nvec = V / 8;
  for (int c = threadIdx.x; c < nvec; c += blockDim.x) {
    float f[8];
    Vec16<T>::load(xr + c * 8, f);
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = (__expf(f[j] - l) - (c * 8 + j == t ? 1.f : 0.f)) * g;
    Vec16<T>::store(dr + c * 8, f);
  }
  for (int j = nvec * 8 + threadIdx.x; j < V; j += blockDim.x)
    Conv<T>::store(dr, j, (__expf(Conv<T>::load(xr, j) - l) - (j == t ? 1.f : 0.f)) * g);
}

void launch_xent_fwd(const void* x, const int64_t* labels, float* loss, float* lse, int64_t rows, int V, int dt,
                     hipStream_t s) {
  if (rows <= 0) return;
  DSA_DISPATCH_16(dt, T,
    hipLaunchKernelGGL((xent_fwd_kernel<T>), dim3((unsigned)rows), dim3(256), 0, s, (const T*)x, labels, loss, lse,
                       V));
}

void launch_xent_bwd(const void* x, const int64_t* labels, const float* lse, const float* dloss, int64_t dloss_stride,
                     void* dx, int64_t rows, int V, int dt, hipStream_t s) {
  if (rows <= 0) return;
  DSA_DISPATCH_16(dt, T,
    hipLaunchKernelGGL((xent_bwd_kernel<T>), dim3((unsigned)rows), dim3(256), 0, s, (const T*)x, labels, lse, dloss,
                       dloss_stride, (T*)dx, V));
}

}  // namespace dsa
