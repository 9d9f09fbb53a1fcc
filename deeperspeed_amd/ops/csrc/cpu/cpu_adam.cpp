// Host-side Adam/AdamW for ZeRO-Offload (module `_cpu_ops`).
//
// Reference parity: csrc/adam/cpu_adam.cpp (Step/Step_4/Step_8 AVX512/AVX2 unrolls over
// 128M-element tiles with OpenMP, optional low-precision copy of the updated weights).
// MI355X-host design: the update kernel is compiled three times (AVX-512, AVX2+FMA,
// scalar) and selected at run time from CPUID, so one build runs on any EPYC; the
// low-precision output is templated (bf16 or fp16) and written straight into a pinned
// buffer that the caller streams to HBM with hipMemcpyAsync (no fp16-only device kernel
// as in the reference, whose bf16 path is missing).
#include <torch/extension.h>
#include <immintrin.h>
#include <omp.h>

#include <cmath>
#include <cstdint>
#include <cstring>

namespace {

struct AdamHP {
  float lr, b1, b2, eps, wd, bc1, bc2, gscale;
  bool adamw;
};

enum OutKind { kNone = 0, kBF16 = 1, kF16 = 2 };

inline uint16_t f32_to_bf16_rne(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);  // quiet NaN stays NaN
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

inline uint16_t f32_to_f16(float f) {
  return (uint16_t)_cvtss_sh(f, _MM_FROUND_TO_NEAREST_INT);
}

// ---------------------------------------------------------------- scalar tail / fallback
inline float bf16_to_f32(uint16_t b) {
  uint32_t u = (uint32_t)b << 16;
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}

inline float load_g(const float* g, int64_t i) { return g[i]; }
inline float load_g(const uint16_t* g, int64_t i) { return bf16_to_f32(g[i]); }

// Gradients arrive as fp32 or as bf16 (the reduced HBM shard copied to host as is: half the
// PCIe bytes of an fp32 copy; widened here, in registers).
template <typename GT>
inline void adam_scalar(float* p, const GT* g, float* m, float* v, uint16_t* out, OutKind ok, int64_t i0,
                        int64_t i1, const AdamHP& h) {
  for (int64_t i = i0; i < i1; ++i) {
    float gr = load_g(g, i) * h.gscale;
    float w = p[i];
    if (!h.adamw && h.wd != 0.f) gr += h.wd * w;
    float mm = h.b1 * m[i] + (1.f - h.b1) * gr;
    float vv = h.b2 * v[i] + (1.f - h.b2) * gr * gr;
    float upd = (mm / h.bc1) / (std::sqrt(vv / h.bc2) + h.eps);
    if (h.adamw && h.wd != 0.f) upd += h.wd * w;
    w -= h.lr * upd;
    p[i] = w;
    m[i] = mm;
    v[i] = vv;
    if (ok == kBF16) out[i] = f32_to_bf16_rne(w);
    else if (ok == kF16) out[i] = f32_to_f16(w);
  }
}

// ---------------------------------------------------------------- AVX2 + FMA (8 lanes)
__attribute__((target("avx2,fma,f16c"))) inline __m256 load8(const float* g, int64_t i) {
  return _mm256_loadu_ps(g + i);
}
__attribute__((target("avx2,fma,f16c"))) inline __m256 load8(const uint16_t* g, int64_t i) {
  __m256i w = _mm256_cvtepu16_epi32(_mm_loadu_si128(reinterpret_cast<const __m128i*>(g + i)));
  return _mm256_castsi256_ps(_mm256_slli_epi32(w, 16));
}

template <typename GT>
__attribute__((target("avx2,fma,f16c"))) void adam_avx2(float* p, const GT* g, float* m, float* v,
                                                        uint16_t* out, OutKind ok, int64_t i0, int64_t i1,
                                                        const AdamHP& h) {
  const __m256 b1 = _mm256_set1_ps(h.b1), b2 = _mm256_set1_ps(h.b2);
  const __m256 ob1 = _mm256_set1_ps(1.f - h.b1), ob2 = _mm256_set1_ps(1.f - h.b2);
  const __m256 ibc1 = _mm256_set1_ps(1.f / h.bc1), ibc2 = _mm256_set1_ps(1.f / h.bc2);
  const __m256 eps = _mm256_set1_ps(h.eps), wd = _mm256_set1_ps(h.wd), nlr = _mm256_set1_ps(-h.lr);
  const __m256 gs = _mm256_set1_ps(h.gscale);
  const bool l2 = !h.adamw && h.wd != 0.f, dec = h.adamw && h.wd != 0.f;
  int64_t i = i0;
  for (; i + 8 <= i1; i += 8) {
    __m256 w = _mm256_loadu_ps(p + i);
    __m256 gr = _mm256_mul_ps(load8(g, i), gs);
    if (l2) gr = _mm256_fmadd_ps(wd, w, gr);
    __m256 mm = _mm256_fmadd_ps(b1, _mm256_loadu_ps(m + i), _mm256_mul_ps(ob1, gr));
    __m256 vv = _mm256_fmadd_ps(b2, _mm256_loadu_ps(v + i), _mm256_mul_ps(ob2, _mm256_mul_ps(gr, gr)));
    __m256 den = _mm256_add_ps(_mm256_sqrt_ps(_mm256_mul_ps(vv, ibc2)), eps);
    __m256 upd = _mm256_div_ps(_mm256_mul_ps(mm, ibc1), den);
    if (dec) upd = _mm256_fmadd_ps(wd, w, upd);
    w = _mm256_fmadd_ps(nlr, upd, w);
    _mm256_storeu_ps(p + i, w);
    _mm256_storeu_ps(m + i, mm);
    _mm256_storeu_ps(v + i, vv);
    if (ok == kF16) {
      _mm_storeu_si128(reinterpret_cast<__m128i*>(out + i), _mm256_cvtps_ph(w, _MM_FROUND_TO_NEAREST_INT));
    } else if (ok == kBF16) {
      __m256i u = _mm256_castps_si256(w);
      __m256i lsb = _mm256_and_si256(_mm256_srli_epi32(u, 16), _mm256_set1_epi32(1));
      __m256i r = _mm256_srli_epi32(_mm256_add_epi32(_mm256_add_epi32(u, _mm256_set1_epi32(0x7fff)), lsb), 16);
      __m128i lo = _mm256_castsi256_si128(r), hi = _mm256_extracti128_si256(r, 1);
      _mm_storeu_si128(reinterpret_cast<__m128i*>(out + i), _mm_packus_epi32(lo, hi));
    }
  }
  adam_scalar(p, g, m, v, out, ok, i, i1, h);
}

// ---------------------------------------------------------------- AVX-512 (16 lanes)
__attribute__((target("avx512f,avx512bw,avx512vl,fma,f16c"))) inline __m512 load16(const float* g, int64_t i) {
  return _mm512_loadu_ps(g + i);
}
__attribute__((target("avx512f,avx512bw,avx512vl,fma,f16c"))) inline __m512 load16(const uint16_t* g, int64_t i) {
  __m512i w = _mm512_cvtepu16_epi32(_mm256_loadu_si256(reinterpret_cast<const __m256i*>(g + i)));
  return _mm512_castsi512_ps(_mm512_slli_epi32(w, 16));
}

template <typename GT>
__attribute__((target("avx512f,avx512bw,avx512vl,fma,f16c"))) void adam_avx512(float* p, const GT* g, float* m,
                                                                               float* v, uint16_t* out, OutKind ok,
                                                                               int64_t i0, int64_t i1,
                                                                               const AdamHP& h) {
  const __m512 b1 = _mm512_set1_ps(h.b1), b2 = _mm512_set1_ps(h.b2);
  const __m512 ob1 = _mm512_set1_ps(1.f - h.b1), ob2 = _mm512_set1_ps(1.f - h.b2);
  const __m512 ibc1 = _mm512_set1_ps(1.f / h.bc1), ibc2 = _mm512_set1_ps(1.f / h.bc2);
  const __m512 eps = _mm512_set1_ps(h.eps), wd = _mm512_set1_ps(h.wd), nlr = _mm512_set1_ps(-h.lr);
  const __m512 gs = _mm512_set1_ps(h.gscale);
  const bool l2 = !h.adamw && h.wd != 0.f, dec = h.adamw && h.wd != 0.f;
  int64_t i = i0;
  for (; i + 16 <= i1; i += 16) {
    __m512 w = _mm512_loadu_ps(p + i);
    __m512 gr = _mm512_mul_ps(load16(g, i), gs);
    if (l2) gr = _mm512_fmadd_ps(wd, w, gr);
    __m512 mm = _mm512_fmadd_ps(b1, _mm512_loadu_ps(m + i), _mm512_mul_ps(ob1, gr));
    __m512 vv = _mm512_fmadd_ps(b2, _mm512_loadu_ps(v + i), _mm512_mul_ps(ob2, _mm512_mul_ps(gr, gr)));
    __m512 den = _mm512_add_ps(_mm512_sqrt_ps(_mm512_mul_ps(vv, ibc2)), eps);
    __m512 upd = _mm512_div_ps(_mm512_mul_ps(mm, ibc1), den);
    if (dec) upd = _mm512_fmadd_ps(wd, w, upd);
    w = _mm512_fmadd_ps(nlr, upd, w);
    _mm512_storeu_ps(p + i, w);
    _mm512_storeu_ps(m + i, mm);
    _mm512_storeu_ps(v + i, vv);
    if (ok == kF16) {
      _mm256_storeu_si256(reinterpret_cast<__m256i*>(out + i), _mm512_cvtps_ph(w, _MM_FROUND_TO_NEAREST_INT));
    } else if (ok == kBF16) {
      __m512i u = _mm512_castps_si512(w);
      __m512i lsb = _mm512_and_si512(_mm512_srli_epi32(u, 16), _mm512_set1_epi32(1));
      __m512i r = _mm512_srli_epi32(_mm512_add_epi32(_mm512_add_epi32(u, _mm512_set1_epi32(0x7fff)), lsb), 16);
      _mm256_storeu_si256(reinterpret_cast<__m256i*>(out + i), _mm512_cvtepi32_epi16(r));
    }
  }
  adam_scalar(p, g, m, v, out, ok, i, i1, h);
}

enum Isa { kScalar = 0, kAvx2 = 1, kAvx512 = 2 };

Isa detect_isa() {
  static int isa = -1;
  if (isa < 0) {
    __builtin_cpu_init();
    if (__builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512bw") && __builtin_cpu_supports("avx512vl"))
      isa = kAvx512;
    else if (__builtin_cpu_supports("avx2") && __builtin_cpu_supports("fma"))
      isa = kAvx2;
    else
      isa = kScalar;
    if (const char* e = std::getenv("DSA_CPU_ADAM_ISA")) isa = std::atoi(e);
  }
  return (Isa)isa;
}

constexpr int64_t kTile = 1 << 16;  // elements per OpenMP work item (256 KB of fp32)

template <typename GT>
void adam_run(float* p, const GT* g, float* m, float* v, uint16_t* out, OutKind ok, int64_t n, const AdamHP& h) {
  const Isa isa = detect_isa();
  const int64_t tiles = (n + kTile - 1) / kTile;
#pragma omp parallel for schedule(static)
  for (int64_t t = 0; t < tiles; ++t) {
    const int64_t i0 = t * kTile, i1 = std::min(n, i0 + kTile);
    if (isa == kAvx512) adam_avx512(p, g, m, v, out, ok, i0, i1, h);
    else if (isa == kAvx2) adam_avx2(p, g, m, v, out, ok, i0, i1, h);
    else adam_scalar(p, g, m, v, out, ok, i0, i1, h);
  }
}

}  // namespace

// Python: adam_update(p, g, m, v, lr, b1, b2, eps, wd, step, bias_correction, grad_scale, adamw, out)
void cpu_adam_update(at::Tensor p, at::Tensor g, at::Tensor m, at::Tensor v, double lr, double b1, double b2,
                     double eps, double wd, int64_t step, bool bias_correction, double grad_scale, bool adamw,
                     c10::optional<at::Tensor> out) {
  TORCH_CHECK(!p.is_cuda() && !g.is_cuda() && !m.is_cuda() && !v.is_cuda(), "cpu_adam: host tensors required");
  TORCH_CHECK(p.scalar_type() == at::kFloat && m.scalar_type() == at::kFloat && v.scalar_type() == at::kFloat,
              "cpu_adam: fp32 master / moments required");
  TORCH_CHECK(g.scalar_type() == at::kFloat || g.scalar_type() == at::kBFloat16, "cpu_adam: fp32 or bf16 gradients");
  TORCH_CHECK(p.is_contiguous() && g.is_contiguous() && m.is_contiguous() && v.is_contiguous(), "cpu_adam: contiguous");
  const int64_t n = p.numel();
  TORCH_CHECK(g.numel() == n && m.numel() == n && v.numel() == n, "cpu_adam: size mismatch");
  OutKind ok = kNone;
  uint16_t* optr = nullptr;
  if (out.has_value()) {
    TORCH_CHECK(!out->is_cuda() && out->numel() == n && out->is_contiguous(), "cpu_adam: out must be host, same size");
    TORCH_CHECK(out->scalar_type() == at::kBFloat16 || out->scalar_type() == at::kHalf, "cpu_adam: out bf16/fp16");
    ok = out->scalar_type() == at::kBFloat16 ? kBF16 : kF16;
    optr = reinterpret_cast<uint16_t*>(out->data_ptr());
  }
  AdamHP h{(float)lr, (float)b1, (float)b2, (float)eps, (float)wd,
           bias_correction ? (float)(1.0 - std::pow(b1, (double)step)) : 1.f,
           bias_correction ? (float)(1.0 - std::pow(b2, (double)step)) : 1.f, (float)grad_scale, adamw};
  {
    pybind11::gil_scoped_release nogil;
    if (g.scalar_type() == at::kBFloat16)
      adam_run(p.data_ptr<float>(), reinterpret_cast<const uint16_t*>(g.data_ptr()), m.data_ptr<float>(),
               v.data_ptr<float>(), optr, ok, n, h);
    else
      adam_run(p.data_ptr<float>(), g.data_ptr<float>(), m.data_ptr<float>(), v.data_ptr<float>(), optr, ok, n, h);
  }
}

int64_t cpu_adam_isa() { return (int64_t)detect_isa(); }
