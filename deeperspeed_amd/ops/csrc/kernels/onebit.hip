// 1-bit error-compensated compression for 1-bit Adam / 1-bit LAMB.
//
// Reference: deepspeed/runtime/comm/nccl.py:47-186 (compressed_allreduce, CuPy packbits /
// unpackbits, torch sign/norm ops).  Here each phase is one or two HIP launches:
//   worker:  c = m + e; s = |c|/sqrt(n); bits = (c >= 0); e = c - s*(+-1)       (2 launches)
//   server:  c = e + (1/P) sum_p s_p*(+-1)_p over the P received sign chunks;
//            then the same pack/error update as the worker                      (2 launches)
//   unpack:  out[p][i] = s_p * (+-1)                                             (1 launch)
// Bits are packed MSB-first (numpy/cupy packbits order), 8 elements per byte; every
// length is a multiple of 8 (the optimizers pad to world*8*k).
#include "../include/dsa_common.h"
#include "../include/launchers.h"

namespace dsa {

static inline int ob_grid(int64_t work, int cap) {
  int64_t g = (work + 255) / 256;
  return (int)(g < 1 ? 1 : (g > cap ? cap : g));
}

__global__ void __launch_bounds__(256) ob_compensate_kernel(const float* __restrict__ m, float* __restrict__ e,
                                                            int64_t n, float* __restrict__ partial) {
  __shared__ float red[32];
  float s = 0.f;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const float c = m[i] + e[i];
    e[i] = c;
    s = fmaf(c, c, s);
  }
  s = block_sum(s, red);
  if (threadIdx.x == 0) partial[blockIdx.x] = s;
}

// server side: c = e + inv_p * sum_p scale_p * sign_p   (signs: [P][nbytes])
__global__ void __launch_bounds__(256) ob_server_avg_kernel(const uint8_t* __restrict__ signs,
                                                            const float* __restrict__ scales, int P, int64_t nbytes,
                                                            float inv_p, float* __restrict__ e,
                                                            float* __restrict__ partial) {
  __shared__ float red[32];
  float s = 0.f;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < nbytes; j += stride) {
    float acc[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] = 0.f;
    for (int p = 0; p < P; ++p) {
      const uint32_t b = signs[(int64_t)p * nbytes + j];
      const float sc = scales[p];
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] += ((b >> (7 - k)) & 1u) ? sc : -sc;
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float c = e[8 * j + k] + acc[k] * inv_p;
      e[8 * j + k] = c;
      s = fmaf(c, c, s);
    }
  }
  s = block_sum(s, red);
  if (threadIdx.x == 0) partial[blockIdx.x] = s;
}

// e holds the compensated values c; writes packed sign bytes, the new error and the scale
__global__ void __launch_bounds__(256) ob_pack_kernel(float* __restrict__ e, int64_t nbytes,
                                                      const float* __restrict__ partial, int nparts, float inv_n,
                                                      uint8_t* __restrict__ packed, float* __restrict__ scale_out) {
  __shared__ float sc_sh;
  if (threadIdx.x < 64) {
    float t = 0.f;
    for (int i = threadIdx.x; i < nparts; i += 64) t += partial[i];
    t = wave_sum(t);
    if (threadIdx.x == 0) sc_sh = sqrtf(t * inv_n);
  }
  __syncthreads();
  const float sc = sc_sh;
  if (blockIdx.x == 0 && threadIdx.x == 0) scale_out[0] = sc;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < nbytes; j += stride) {
    uint32_t b = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float c = e[8 * j + k];
      const bool pos = c >= 0.f;
      b |= (pos ? 1u : 0u) << (7 - k);
      e[8 * j + k] = c - (pos ? sc : -sc);
    }
    packed[j] = (uint8_t)b;
  }
}

__global__ void __launch_bounds__(256) ob_unpack_kernel(const uint8_t* __restrict__ signs,
                                                        const float* __restrict__ scales, int64_t nbytes_per,
                                                        int64_t total_bytes, float* __restrict__ out) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < total_bytes; j += stride) {
    const uint32_t b = signs[j];
    const float sc = scales[j / nbytes_per];
    float4 lo, hi;
    lo.x = (b & 0x80u) ? sc : -sc; lo.y = (b & 0x40u) ? sc : -sc;
    lo.z = (b & 0x20u) ? sc : -sc; lo.w = (b & 0x10u) ? sc : -sc;
    hi.x = (b & 0x08u) ? sc : -sc; hi.y = (b & 0x04u) ? sc : -sc;
    hi.z = (b & 0x02u) ? sc : -sc; hi.w = (b & 0x01u) ? sc : -sc;
    reinterpret_cast<float4*>(out)[2 * j] = lo;
    reinterpret_cast<float4*>(out)[2 * j + 1] = hi;
  }
}

// workspace: >= 1024 floats
void launch_onebit_worker(const float* m, float* err, int64_t n, uint8_t* packed, float* scale_out, float* ws,
                          hipStream_t s) {
  const int g1 = ob_grid(n, 1024);
  hipLaunchKernelGGL(ob_compensate_kernel, dim3(g1), dim3(256), 0, s, m, err, n, ws);
  hipLaunchKernelGGL(ob_pack_kernel, dim3(ob_grid(n / 8, 2048)), dim3(256), 0, s, err, n / 8, ws, g1,
                     1.0f / (float)n, packed, scale_out);
}

void launch_onebit_server(const uint8_t* signs, const float* scales, int P, int64_t nbytes, float* server_err,
                          uint8_t* packed, float* scale_out, float* ws, hipStream_t s) {
  const int g1 = ob_grid(nbytes, 1024);
  hipLaunchKernelGGL(ob_server_avg_kernel, dim3(g1), dim3(256), 0, s, signs, scales, P, nbytes, 1.0f / (float)P,
                     server_err, ws);
  hipLaunchKernelGGL(ob_pack_kernel, dim3(ob_grid(nbytes, 2048)), dim3(256), 0, s, server_err, nbytes, ws, g1,
                     1.0f / (float)(nbytes * 8), packed, scale_out);
}

void launch_onebit_unpack(const uint8_t* signs, const float* scales, int P, int64_t nbytes_per, float* out,
                          hipStream_t s) {
  const int64_t total = (int64_t)P * nbytes_per;
  hipLaunchKernelGGL(ob_unpack_kernel, dim3(ob_grid(total, 4096)), dim3(256), 0, s, signs, scales, nbytes_per,
                     total, out);
}

}  // namespace dsa
