// Exhaustive hipBLASLt algorithm sweep for the GEMM layouts of a transformer linear's backward.
//
// The heuristic top-16 (ops/csrc/gemm_lt.cpp) never offered a fast kernel for the token-major
// weight-gradient (NT) and the untransposed input-gradient (NN) layouts on gfx950, which is why
// the backward transposes its operands first (ops/linear.py).  This tool times EVERY algorithm
// hipblaslt_ext::getAllAlgos returns for a row-major problem and prints the fastest few, so a
// layout that hipBLASLt can run at the TN rate would let the transposes go.
//
//   layouts (row-major meaning):
//     fwd    Y[M,N]  = X[M,K] . W[N,K]^T        (col-major TN)
//     dgrad  dX[M,K] = dY[M,N] . W[N,K]         (col-major NN)
//     wgrad  dW[N,K] += dY[M,N]^T . X[M,K]      (col-major NT, beta = 1)
//     wgradT dW[N,K] += dYt[N,M] . Xt[K,M]^T    (col-major TN after the two transposes, beta = 1)
//
//     fwdb   fwd with the BIAS epilogue (what F.linear(x, W, b) asks for)
//
// Build: hipcc -O2 --offload-arch=gfx950 scripts/lt_sweep.cpp -lhipblaslt -o lt_sweep
// Run:   ./lt_sweep <layout>:M:N:K [<layout>:M:N:K ...]   (one JSON line per problem)
// Only macro tiles of at least 128 x 128 are timed when both output dims are >= 2048 (the small
// tiles cannot fill the chip there, and each kernel's first launch loads its code object).
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt-ext.hpp>
#include <hipblaslt/hipblaslt.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#define CK(x)                                                                      \
  do {                                                                             \
    auto _s = (x);                                                                 \
    if ((int)_s != 0) {                                                            \
      fprintf(stderr, "error %d at %s:%d: %s\n", (int)_s, __FILE__, __LINE__, #x); \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

__global__ void fill_rand(uint16_t* p, size_t n, uint32_t seed) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  for (; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 13;
    h *= 0x5bd1e995u;
    h ^= h >> 15;
    float f = ((h & 0xffff) / 32768.0f - 1.0f);  // uniform [-1, 1)
    uint32_t b;
    memcpy(&b, &f, 4);
    p[i] = (uint16_t)(b >> 16);
  }
}

static bool small_tile(const std::string& name) {
  const size_t p = name.find("_MT");
  if (p == std::string::npos) return false;
  const int a = atoi(name.c_str() + p + 3);
  const size_t x = name.find('x', p + 3);
  const int b = x == std::string::npos ? 0 : atoi(name.c_str() + x + 1);
  return a < 128 || b < 128;
}

static int sweep(hipblasLtHandle_t h, const std::string& spec, void* ws, size_t wsz);

int main(int argc, char** argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: %s layout:M:N:K ...\n", argv[0]);
    return 2;
  }
  hipblasLtHandle_t h;
  CK(hipblasLtCreate(&h));
  void* ws;
  const size_t wsz = 64ull << 20;
  CK(hipMalloc(&ws, wsz));
  for (int i = 1; i < argc; ++i)
    if (sweep(h, argv[i], ws, wsz)) return 1;
  return 0;
}

static int sweep(hipblasLtHandle_t h, const std::string& spec, void* ws, size_t wsz) {
  char lbuf[16];
  long M_, N_, K_;
  if (sscanf(spec.c_str(), "%15[a-zA-Z]:%ld:%ld:%ld", lbuf, &M_, &N_, &K_) != 4) {
    fprintf(stderr, "bad problem %s\n", spec.c_str());
    return 1;
  }
  std::string lay = lbuf;
  const int64_t M = M_, N = N_, K = K_;
  const int top = 6;
  const bool bias = lay == "fwdb";
  if (bias) lay = "fwd";
  // column-major problem D[m,n] = op(A)[m,k] op(B)[k,n]
  hipblasOperation_t ta, tb;
  int64_t m, n, k, lda, ldb, ldd, ar, ac, br, bc;
  float beta = 0.f;
  if (lay == "fwd") {  // Y^T[N,M] = W(col [K,N])^T . X(col [K,M])
    ta = HIPBLAS_OP_T, tb = HIPBLAS_OP_N, m = N, n = M, k = K;
    ar = K, ac = N, lda = K, br = K, bc = M, ldb = K, ldd = N;
  } else if (lay == "dgrad") {  // dX^T[K,M] = W(col [K,N]) . dY(col [N,M])
    ta = HIPBLAS_OP_N, tb = HIPBLAS_OP_N, m = K, n = M, k = N;
    ar = K, ac = N, lda = K, br = N, bc = M, ldb = N, ldd = K;
  } else if (lay == "wgrad") {  // dW^T[K,N] = X(col [K,M]) . dY(col [N,M])^T
    ta = HIPBLAS_OP_N, tb = HIPBLAS_OP_T, m = K, n = N, k = M, beta = 1.f;
    ar = K, ac = M, lda = K, br = N, bc = M, ldb = N, ldd = K;
  } else if (lay == "wgradT") {  // dW^T[K,N] = Xt(col [M,K])^T . dYt(col [M,N])
    ta = HIPBLAS_OP_T, tb = HIPBLAS_OP_N, m = K, n = N, k = M, beta = 1.f;
    ar = M, ac = K, lda = M, br = M, bc = N, ldb = M, ldd = K;
  } else {
    fprintf(stderr, "unknown layout %s\n", lay.c_str());
    return 1;
  }
  uint16_t *A, *B, *D, *bvec = nullptr;
  CK(hipMalloc(&A, ar * ac * 2));
  CK(hipMalloc(&B, br * bc * 2));
  CK(hipMalloc(&D, m * n * 2));
  if (bias) {
    CK(hipMalloc(&bvec, m * 2));
    fill_rand<<<64, 256>>>(bvec, m, 4);
  }
  fill_rand<<<2048, 256>>>(A, ar * ac, 1);
  fill_rand<<<2048, 256>>>(B, br * bc, 2);
  fill_rand<<<2048, 256>>>(D, m * n, 3);
  CK(hipDeviceSynchronize());

  hipblasLtMatmulDesc_t op;
  CK(hipblasLtMatmulDescCreate(&op, HIPBLAS_COMPUTE_32F, HIP_R_32F));
  CK(hipblasLtMatmulDescSetAttribute(op, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta)));
  CK(hipblasLtMatmulDescSetAttribute(op, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb)));
  if (bias) {
    const hipblasLtEpilogue_t e = HIPBLASLT_EPILOGUE_BIAS;
    const hipDataType bt = HIP_R_16BF;
    CK(hipblasLtMatmulDescSetAttribute(op, HIPBLASLT_MATMUL_DESC_EPILOGUE, &e, sizeof(e)));
    CK(hipblasLtMatmulDescSetAttribute(op, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bvec, sizeof(void*)));
    CK(hipblasLtMatmulDescSetAttribute(op, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof(bt)));
  }
  hipblasLtMatrixLayout_t la, lb, ld;
  CK(hipblasLtMatrixLayoutCreate(&la, HIP_R_16BF, ar, ac, lda));
  CK(hipblasLtMatrixLayoutCreate(&lb, HIP_R_16BF, br, bc, ldb));
  CK(hipblasLtMatrixLayoutCreate(&ld, HIP_R_16BF, m, n, ldd));
  const float alpha = 1.f;

  std::vector<hipblasLtMatmulHeuristicResult_t> all;
  CK(hipblaslt_ext::getAllAlgos(h, hipblaslt_ext::GemmType::HIPBLASLT_GEMM, ta, tb, HIP_R_16BF, HIP_R_16BF,
                                HIP_R_16BF, HIP_R_16BF, HIPBLAS_COMPUTE_32F, all));
  // the heuristic's first choice, for comparison
  hipblasLtMatmulPreference_t pref;
  CK(hipblasLtMatmulPreferenceCreate(&pref));
  uint64_t w64 = wsz;
  CK(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &w64, sizeof(w64)));
  hipblasLtMatmulHeuristicResult_t heur[1];
  int nh = 0;
  hipblasLtMatmulAlgoGetHeuristic(h, op, la, lb, ld, ld, pref, 1, heur, &nh);
  const int heur_idx = nh > 0 ? hipblaslt_ext::getIndexFromAlgo(heur[0].algo) : -1;

  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  struct R {
    float ms;
    int idx;
    std::string name;
    std::string sol;
  };
  std::vector<R> res;
  const double flops = 2.0 * M * N * K;
  int tried = 0;
  const bool big = m >= 2048 && n >= 2048;
  for (auto& r : all) {
    if (big && small_tile(hipblaslt_ext::getKernelNameFromAlgo(h, r.algo))) continue;
    size_t need = 0;
    if (hipblaslt_ext::matmulIsAlgoSupported(h, op, &alpha, la, lb, &beta, ld, ld, r.algo, need) !=
            HIPBLAS_STATUS_SUCCESS ||
        need > wsz)
      continue;
    ++tried;
    bool ok = true;
    for (int i = 0; i < 1 && ok; ++i)
      ok = hipblasLtMatmul(h, op, &alpha, A, la, B, lb, &beta, D, ld, D, ld, &r.algo, ws, wsz, 0) ==
           HIPBLAS_STATUS_SUCCESS;
    if (!ok) continue;
    const int reps = 3;
    hipEventRecord(e0, 0);
    for (int i = 0; i < reps; ++i) hipblasLtMatmul(h, op, &alpha, A, la, B, lb, &beta, D, ld, D, ld, &r.algo, ws, wsz, 0);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    res.push_back({ms / reps, hipblaslt_ext::getIndexFromAlgo(r.algo), hipblaslt_ext::getKernelNameFromAlgo(h, r.algo),
                   hipblaslt_ext::getSolutionNameFromAlgo(h, r.algo)});
  }
  std::sort(res.begin(), res.end(), [](const R& a, const R& b) { return a.ms < b.ms; });
  float heur_ms = -1;
  for (auto& r : res)
    if (r.idx == heur_idx) heur_ms = r.ms;
  printf("{\"layout\": \"%s%s\", \"M\": %ld, \"N\": %ld, \"K\": %ld, \"algos\": %zu, \"supported\": %d, "
         "\"heuristic_idx\": %d, \"heuristic_tflops\": %.1f, "
         "\"col\": {\"ta\": %d, \"tb\": %d, \"m\": %ld, \"n\": %ld, \"k\": %ld, \"epi\": %d, \"beta\": %d}, \"top\": [",
         lay.c_str(), bias ? "+bias" : "", (long)M, (long)N, (long)K, all.size(), tried, heur_idx,
         heur_ms > 0 ? flops / heur_ms / 1e9 : -1.0, ta == HIPBLAS_OP_T, tb == HIPBLAS_OP_T, (long)m, (long)n, (long)k,
         bias ? (int)HIPBLASLT_EPILOGUE_BIAS : (int)HIPBLASLT_EPILOGUE_DEFAULT, beta != 0.f);
  for (int i = 0; i < top && i < (int)res.size(); ++i)
    printf("%s{\"idx\": %d, \"tflops\": %.1f, \"kernel\": \"%s\", \"sol\": \"%s\"}", i ? ", " : "", res[i].idx,
           flops / res[i].ms / 1e9, res[i].name.substr(0, 120).c_str(), res[i].sol.c_str());
  printf("]}\n");
  fflush(stdout);
  hipFree(A);
  hipFree(B);
  hipFree(D);
  if (bvec) hipFree(bvec);
  hipblasLtMatrixLayoutDestroy(la);
  hipblasLtMatrixLayoutDestroy(lb);
  hipblasLtMatrixLayoutDestroy(ld);
  hipblasLtMatmulDescDestroy(op);
  hipblasLtMatmulPreferenceDestroy(pref);
  return 0;
}
