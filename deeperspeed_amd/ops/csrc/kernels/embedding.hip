// Embedding backward without a host round trip.
//
// PyTorch's dense embedding backward on the GPU sorts the token ids, counts the runs of equal
// ids and reads that count back to size its launches: a device -> host sync at the end of every
// backward, which drains the queue and leaves the GPU idle while the host catches up (~1 ms per
// BERT-Large step in profiles/r3o_bert_large_seq128_timed_kernel_stats.md's trace).  Here every
// launch is sized by the number of TOKENS, which the host knows, and the result is deterministic
// (fp32 sums in sorted order):
//   pass 1: block c owns sorted positions [R c, R c + R).  A run of equal ids that starts and
//           ends inside the chunk is summed and written to its weight-gradient row directly; the
//           piece of a run continued from the previous chunk goes to cont[c], the piece of a run
//           that starts here and continues past the chunk goes to head[c] (fp32 partial rows);
//   pass 2: block c whose last run continues past the chunk adds head[c] and the cont[] pieces
//           of the following chunks until the run ends, and writes the row.
// Long runs (padding tokens, frequent words) therefore cost R rows per block plus one partial
// row per chunk they span, never a serial walk over the run.
//
// Reference counterpart: none in DeeperSpeed (its models use torch.nn.Embedding); the gradient is
// the one PyTorch's embedding_dense_backward produces.
#include "../include/dsa_common.h"
#include "../include/launchers.h"

namespace dsa {
namespace {

constexpr int EMB_R = 32;  // sorted positions per pass-1 block

template <typename T>
__device__ __forceinline__ void emb_store(T* __restrict__ dw, int64_t id, int H, int v, const float (&acc)[8],
                                          int accumulate) {
  T* out = dw + id * (int64_t)H + v * 8;
  if (accumulate) {
    float o[8];
    Vec16<T>::load(out, o);
    float s[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) s[j] = acc[j] + o[j];
    Vec16<T>::store(out, s);
  } else {
    Vec16<T>::store(out, acc);
  }
}

template <typename T>
__global__ void __launch_bounds__(256) embedding_bwd_pass1(const int64_t* __restrict__ ids,
                                                           const int64_t* __restrict__ perm,
                                                           const T* __restrict__ dy, T* __restrict__ dw,
                                                           float* __restrict__ head, float* __restrict__ cont,
                                                           int64_t n, int H, int64_t padding_idx, int accumulate) {
  const int64_t c = blockIdx.x;
  const int64_t c0 = c * EMB_R, c1 = c0 + EMB_R < n ? c0 + EMB_R : n;
  const int nvec = H / 8;
  int64_t ps = c0;
  while (ps < c1) {  // block-uniform walk over the runs of this chunk
    const int64_t id = ids[ps];
    int64_t pe = ps + 1;
    while (pe < c1 && ids[pe] == id) ++pe;
    const bool starts = ps > 0 ? ids[ps - 1] != id : true;
    const bool ends = pe < n ? ids[pe] != id : true;
    for (int v = threadIdx.x; v < nvec; v += blockDim.x) {
      float acc[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] = 0.f;
      for (int64_t r = ps; r < pe; ++r) {
        float x[8];
        Vec16<T>::load(dy + perm[r] * (int64_t)H + v * 8, x);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += x[j];
      }
      if (starts && ends) {
        if (id != padding_idx) emb_store<T>(dw, id, H, v, acc, accumulate);
      } else {
        float* p = (starts ? head : cont) + c * (int64_t)H + v * 8;
        *reinterpret_cast<float4*>(p) = make_float4(acc[0], acc[1], acc[2], acc[3]);
        *reinterpret_cast<float4*>(p + 4) = make_float4(acc[4], acc[5], acc[6], acc[7]);
      }
    }
    ps = pe;
  }
}

template <typename T>
__global__ void __launch_bounds__(256) embedding_bwd_pass2(const int64_t* __restrict__ ids,
                                                           const float* __restrict__ head,
                                                           const float* __restrict__ cont, T* __restrict__ dw,
                                                           int64_t n, int H, int64_t padding_idx, int accumulate) {
  const int64_t c = blockIdx.x;
  const int64_t last = (c * EMB_R + EMB_R < n ? c * EMB_R + EMB_R : n) - 1;
  const int64_t id = ids[last];
  if (last + 1 >= n || ids[last + 1] != id) return;  // the chunk's last run ends inside it
  // does that run start inside this chunk (else an earlier chunk owns it)?
  int64_t ps = last;
  while (ps > c * EMB_R && ids[ps - 1] == id) --ps;
  if (ps == c * EMB_R && ps > 0 && ids[ps - 1] == id) return;
  if (id == padding_idx) return;
  const int nchunks = (int)((n + EMB_R - 1) / EMB_R);
  const int nvec = H / 8;
  for (int v = threadIdx.x; v < nvec; v += blockDim.x) {
    float acc[8];
    const float* hp = head + c * (int64_t)H + v * 8;
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = hp[j];
    for (int64_t c2 = c + 1; c2 < nchunks; ++c2) {
      const float* cp = cont + c2 * (int64_t)H + v * 8;
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += cp[j];
      const int64_t l2 = (c2 * EMB_R + EMB_R < n ? c2 * EMB_R + EMB_R : n) - 1;
      if (ids[l2] != id || l2 + 1 >= n || ids[l2 + 1] != id) break;  // the run ends in chunk c2
    }
    emb_store<T>(dw, id, H, v, acc, accumulate);
  }
}

}  // namespace

int64_t embedding_bwd_chunks(int64_t n) { return (n + EMB_R - 1) / EMB_R; }

// head / cont: fp32 workspaces of embedding_bwd_chunks(n) * H each
void launch_embedding_bwd_sorted(const int64_t* sorted_ids, const int64_t* perm, const void* dy, void* dw,
                                 float* head, float* cont, int64_t n, int H, int64_t padding_idx, int accumulate,
                                 int dt, hipStream_t s) {
  if (n <= 0) return;
  const unsigned nc = (unsigned)embedding_bwd_chunks(n);
  DSA_DISPATCH_16(dt, T,
    hipLaunchKernelGGL((embedding_bwd_pass1<T>), dim3(nc), dim3(256), 0, s, sorted_ids, perm, (const T*)dy, (T*)dw,
                       head, cont, n, H, padding_idx, accumulate);
    hipLaunchKernelGGL((embedding_bwd_pass2<T>), dim3(nc), dim3(256), 0, s, sorted_ids, (const float*)head,
                       (const float*)cont, (T*)dw, n, H, padding_idx, accumulate));
}

}  // namespace dsa
