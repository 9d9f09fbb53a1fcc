// Fused (flash-style) attention forward + backward for CDNA4 (gfx950) on bf16/fp16 MFMA.
//
// Replaces the reference's materialised attention path (QK^T strided-batched GEMM ->
// attn_softmax -> PV GEMM, csrc/transformer/softmax_kernels.cu, strided_batch_gemm.h) and
// its S<8192 limit: scores never leave the CU.  Layout: q,k,v,o [B*H, S, D] row-major,
// lse [B*H, S] fp32 (natural log of the scaled row sum), D in {64, 96, 128}.
//
// Every kernel here runs v_mfma_f32_32x32x16 (bf16 / fp16) on wave64 with 4-wave workgroups of
// 128 rows (BM2: queries for the forward and dQ, keys for dK/dV), K / V (or Q / dO) tiles of 64
// rows (BN2) double-buffered in LDS and read "down a column" with ds_read_b64_tr_b16 (hardware
// transpose), softmax in registers in the C layout (see "forward v2" below).  Backward is
// FA2-style without atomics: dQ (+ Delta) first, then dK/dV per key block, both recomputing P
// from the saved LSE.  Block-sparse variants walk a LUT of active 64 x 64 tiles (bottom).
#include <algorithm>
#include <cstdlib>
#include <stdexcept>
#include <type_traits>

#include "../include/dsa_common.h"
#include "../include/launchers.h"

namespace dsa {
namespace fa {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

// LDS row stride (elements) of the [rows][D] Q / K / V / dO tiles.  D + 8 keeps the ds_read_b128 row
// reads conflict-free for every D; the 32x32x16 transposed reads (ds_read_b64_tr_b16, 4 rows x 4
// lanes x 2 column halves per 32-lane half) are 2-way at D = 64 / 96 with +8 but 4-way at D = 128
// (stride 272 B puts rows 4 banks apart); +24 (304 B) brings D = 128 to 2-way with the row reads
// still conflict-free (rocprofv3 SQ_LDS_BANK_CONFLICT: 3.2-3.4 cycles per LDS instruction at D = 128
// vs 1.2 at D = 96 before, profiles/r4z_notes.md).
template <int D> constexpr int LDP = D + (D == 128 ? 24 : 8);

template <typename T> __device__ __forceinline__ uint16_t to16(float f);
template <> __device__ __forceinline__ uint16_t to16<bf16_t>(float f) { return f32_to_bf16(f); }
template <> __device__ __forceinline__ uint16_t to16<f16_t>(float f) { return f32_to_f16(f); }

// 8 consecutive 16-bit elements of an LDS row (A fragment / B-from-transposed-storage)
__device__ __forceinline__ s16x8 lds_row8(const uint16_t* p) { return *reinterpret_cast<const s16x8*>(p); }

// O / dO addressing: onh == 0 -> [B*H, S, D] (head-major, like q/k/v); onh == H -> [B, S, H, D]
// (token-major: the attention output is consumed as [B, S, H*D] by the output projection with
// no transpose copy, and its gradient arrives in that layout).
template <int D>
__device__ __forceinline__ int64_t o_base(int64_t bh, int S, int onh) {
  return onh ? ((bh / onh) * (int64_t)S * onh + bh % onh) * D : bh * (int64_t)S * D;
}
template <int D>
__device__ __forceinline__ int o_ld(int onh) { return onh ? onh * D : D; }

// ======================================================================== backward: delta
template <typename T, int D>
__global__ void __launch_bounds__(256) delta_kernel(const uint16_t* __restrict__ dO, const uint16_t* __restrict__ O,
                                                    float* __restrict__ delta, int64_t rows, int S, int onh) {
  // 8 lanes per row, 16-byte loads; row = bh * S + s (delta is head-major like LSE)
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t row = t >> 3;
  const int sub = t & 7;
  float acc = 0.f;
  if (row < rows) {
    const int64_t off = o_base<D>(row / S, S, onh) + (row % S) * o_ld<D>(onh);
    for (int c = sub; c < D / 8; c += 8) {
      float a[8], b[8];
      Vec16<T>::load(reinterpret_cast<const T*>(dO) + off + c * 8, a);
      Vec16<T>::load(reinterpret_cast<const T*>(O) + off + c * 8, b);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc = fmaf(a[j], b[j], acc);
    }
  }
  acc += __shfl_xor(acc, 1, 64);
  acc += __shfl_xor(acc, 2, 64);
  acc += __shfl_xor(acc, 4, 64);
  if (row < rows && sub == 0) delta[row] = acc;
}

// ======================================================================== forward v2
// 32x32x16 MFMA, S^T = K Q^T formulation (one wave = 32 queries, WG = 128 queries):
//  * Q^T is the B operand and stays in registers for the whole key loop;
//  * S^T's C layout gives every lane one query (col) and 16 keys per tile, so the softmax
//    max / sum are in-lane plus one xor-32 shuffle, and the rescale of O^T is per lane;
//  * P^T is used as the B operand of O^T = V^T P^T straight from registers: the k (key)
//    index of both operands follows the C-layout permutation {4h..4h+3, 8+4h..8+4h+3};
//  * V^T fragments come from ds_read_b64_tr_b16 on the natural [key][d] V tile;
//  * K/V tiles are double-buffered in LDS; the next tile's global loads are issued before
//    the current tile's MFMAs and written to the other buffer afterwards (1 barrier/tile).
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <typename T> struct Mfma32;
template <> struct Mfma32<bf16_t> {
  __device__ __forceinline__ static f32x16 run(s16x8 a, s16x8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c,
                                                   0, 0, 0);
  }
};
template <> struct Mfma32<f16_t> {
  __device__ __forceinline__ static f32x16 run(s16x8 a, s16x8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0,
                                                  0, 0);
  }
};

constexpr int BM2 = 128;
constexpr int BN2 = 64;

// reductions across the two 32-lane halves of a wave (the two halves of a query row's keys):
// v_permlane32_swap of x with itself leaves {lower half, upper half} values of the lane pair in
// the two results on EVERY lane, so max / sum need no ds_bpermute round trip through the LDS
// crossbar and no select; both halves add in the same order (bit-identical row statistics)
__device__ __forceinline__ float xhalf_max(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float xhalf_sum(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// raw v_exp_f32 (no denormal range fix-up: softmax weights below 2^-126 are zero anyway)
__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

// 1-D grid -> task id such that consecutive tasks (the row blocks of one head, which share its
// K/V) run on the same XCD and hit that XCD's L2: the hardware deals workgroups round-robin to
// the 8 XCDs, so XCD x = lin % 8 receives the contiguous task range [base_x, base_x + count_x).
// Bijective for any n (also n % 8 != 0).  Placement only affects speed, never correctness.
__device__ __forceinline__ int xcd_task(int lin, int n) {
  const int xcd = lin & 7, slot = lin >> 3, q = n >> 3, r = n & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + slot;
}

// Buffer-load form of tile_load for a loop that walks tiles of one head: the head's rows sit
// behind one buffer resource (scalar registers) sized to its S rows, so a row past the end
// reads 0 in hardware and each lane keeps only a 32-bit offset -- the pointer form holds a
// 64-bit address per chunk plus a bounds branch, which spilled registers in the dK/dV kernel.
typedef unsigned int fa_u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t head_rsrc(const uint16_t* g, int S, int ld) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)g, (short)0, S * ld * 2, 0x00020000);
}

template <int D>
__device__ __forceinline__ void tile_load_buf(uint4 (&r)[D / 32], __amdgpu_buffer_rsrc_t rs, int r0, int ld) {
  constexpr int CH = D / 8;
#pragma unroll
  for (int k = 0; k < D / 32; ++k) {
    const int c = threadIdx.x + 256 * k;
    const int row = c / CH, ch = c - row * CH;
    const fa_u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, ((r0 + row) * ld + ch * 8) * 2, 0, 0);
    r[k] = make_uint4(v.x, v.y, v.z, v.w);
  }
}

template <int D>
__device__ __forceinline__ void tile_load(uint4 (&r)[D / 32], const uint16_t* __restrict__ g, int r0, int S,
                                          int ld = D) {
  constexpr int CH = D / 8;
#pragma unroll
  for (int k = 0; k < D / 32; ++k) {
    const int c = threadIdx.x + 256 * k;
    const int row = c / CH, ch = c - row * CH;
    r[k] = (r0 + row < S) ? *reinterpret_cast<const uint4*>(g + (int64_t)(r0 + row) * ld + ch * 8)
                          : make_uint4(0, 0, 0, 0);
  }
}

template <int D, int LD = LDP<D>>
__device__ __forceinline__ void tile_store(uint16_t* lds, const uint4 (&r)[D / 32]) {
  constexpr int CH = D / 8;
#pragma unroll
  for (int k = 0; k < D / 32; ++k) {
    const int c = threadIdx.x + 256 * k;
    const int row = c / CH, ch = c - row * CH;
    *reinterpret_cast<uint4*>(lds + row * LD + ch * 8) = r[k];
  }
}

// Row stride of a tile that is ONLY read transposed (ds_read_b64_tr_b16, 32 lanes = 4 rows x 64 B):
// the 4 rows must start 16 banks apart.  At D = 96 the unpadded 192-byte row (48 banks) does that;
// the padded 208-byte row (52 banks) puts rows 0 and 1 of the two column halves on banks 0-3 (2-way).
// Tiles also read row-wise keep LDP (whose padding makes the ds_read_b128 row reads conflict-free).
template <int D> constexpr int LDPT = D == 96 ? 96 : LDP<D>;

// Dual-use LDS image for a [64][D] tile read BOTH row-wise (ds_read_b128 A fragments) and
// transposed (ds_read_b64_tr_b16): 8-row x 32-column subtiles of 512 B with the 16-byte chunks of
// each row XOR-permuted by bits 2-3 of the row (cdna_hip_programming.md T10, image (a)).  Both
// read kinds are conflict-free; on the padded 208-byte rows (D = 96) the transposed reads are 2-way
// for half the lanes.  Element offset of 16-byte chunk `ch` of row `r`:
template <int D>
__device__ __forceinline__ int swz_el(int r, int ch) {
  return (D * 8) * (r >> 3) + 256 * (ch >> 2) + 32 * (r & 7) + 8 * ((ch & 3) ^ ((r >> 2) & 3));
}
template <int D>
__device__ __forceinline__ void tile_store_sw(uint16_t* lds, const uint4 (&r)[D / 32]) {
  constexpr int CH = D / 8;
#pragma unroll
  for (int k = 0; k < D / 32; ++k) {
    const int c = threadIdx.x + 256 * k;
    const int row = c / CH, ch = c - row * CH;
    *reinterpret_cast<uint4*>(lds + swz_el<D>(row, ch)) = r[k];
  }
}
// The kernels' two read patterns on a swizzled image, split into a lane constant (two per pattern,
// computed once) and a compile-time offset per unrolled step, so every read is one base VGPR plus
// an immediate offset, as on the padded image:
//   row read of the 32x32x16 A fragment: row 32t + c32, chunk 2ks + h
//     = swz_row_lane(ks & 1) + 32*D*t + 256*(ks >> 1)
//   transposed read: rows 16kb + 4(g16 >> 1) + qd (+ 8 e8), chunk 4dt + 2(g16 & 1) + (pc >> 1)
//     = swz_tr_lane(e8) + 16*D*kb + 256*dt
template <int D>
__device__ __forceinline__ int swz_row_lane(int lane, int odd) {
  const int c32 = lane & 31, h = lane >> 5;
  return D * 8 * (c32 >> 3) + 32 * (c32 & 7) + 8 * ((2 * odd + h) ^ ((c32 >> 2) & 3));
}
template <int D>
__device__ __forceinline__ int swz_tr_lane(int lane, int e8) {
  const int g16 = lane >> 4, qd = (lane & 15) >> 2, pc = lane & 3;
  return D * 8 * e8 + 32 * (4 * (g16 >> 1) + qd) + 8 * ((2 * (g16 & 1) + (pc >> 1)) ^ ((g16 >> 1) + 2 * e8)) +
         4 * (pc & 1);
}
template <int D>
struct SwzLanes {
  int r0, r1, t0, t1;
  __device__ __forceinline__ explicit SwzLanes(int lane)
      : r0(swz_row_lane<D>(lane, 0)), r1(swz_row_lane<D>(lane, 1)), t0(swz_tr_lane<D>(lane, 0)),
        t1(swz_tr_lane<D>(lane, 1)) {}
  __device__ __forceinline__ int row(int t, int ks) const { return ((ks & 1) ? r1 : r0) + 32 * D * t + 256 * (ks >> 1); }
  __device__ __forceinline__ int tr(int kb, int e8, int dt) const { return (e8 ? t1 : t0) + 16 * D * kb + 256 * dt; }
};
template <int D, bool SW>
__device__ __forceinline__ void tile_put(uint16_t* lds, const uint4 (&r)[D / 32]) {
  if constexpr (SW) tile_store_sw<D>(lds, r);
  else tile_store<D>(lds, r);
}

__device__ __forceinline__ s16x8 pack8(const float* v, int base) {
  s16x8 out;
#pragma unroll
  for (int j = 0; j < 8; ++j) out[j] = (short)f32_to_bf16(v[base + j]);
  return out;
}
__device__ __forceinline__ s16x8 pack8_h(const float* v, int base) {
  s16x8 out;
#pragma unroll
  for (int j = 0; j < 8; ++j) out[j] = (short)f32_to_f16(v[base + j]);
  return out;
}

// LAZY: the running max m is raised only when a tile's max exceeds it by more than
// LAZY_TH (log2 units, i.e. P <= 2^8 in between), decided per wave: most tiles then skip the
// O / l rescale (D/32*16 + 1 multiplies per lane) and alpha's exp.  Exact up to rounding.
constexpr float LAZY_TH = 8.0f;

// ---- encoder (BERT) extras, compiled in by the EX template bits of the v2 kernels
//   EX_BIAS: additive per-key bias kbias[b][key] (the [B,1,1,S] padding mask), b = bh / hdiv
//   EX_DROP: dropout on the probabilities (reference attn_dropout after the softmax).  The
//            keep mask is a counter-based hash of (seed, bh, query, key), so the backward
//            kernels regenerate it in their own register layouts and nothing S x S is stored:
//            one 32-bit hash yields the 16-bit draws of keys 2j and 2j+1 of a query row.
//            The normaliser l / LSE stays the undropped one; O = (P * Z) V / (1 - p).
constexpr int EX_BIAS = 1, EX_DROP = 2, EX_QKV = 4;  // EX_QKV: token-major q/k/v (Extra::inh/ild)
struct Extra {
  const float* kbias = nullptr;
  int hdiv = 1;
  uint32_t seed = 0;
  uint32_t thresh = 0;  // a draw below thresh (of 65536) drops the element
  float rscale = 1.f;   // 1 / (1 - p)
  // token-major q/k/v (and dq/dk/dv) with row stride ild elements, head h at column h*D, batch
  // b = bh / inh (e.g. straight out of the fused QKV projection [B, S, 3, H, D]); inh == 0:
  // the [B*H, S, D] layout
  int inh = 0;
  int64_t ild = 0;
  // optional device int64 [seed, step] mixed into `seed` on the GPU (graph-replayable dropout)
  const int64_t* rng = nullptr;
};

// compile-time layout switch: the head-major kernels keep constant row strides (immediate load
// offsets); only EX_QKV instantiations pay for the runtime stride
template <int D, int EX>
__device__ __forceinline__ int64_t in_base(const Extra& ex, int64_t bh, int S) {
  if constexpr ((EX & EX_QKV) != 0) return (bh / ex.inh) * (int64_t)S * ex.ild + (bh % ex.inh) * D;
  return bh * (int64_t)S * D;
}
template <int D, int EX>
__device__ __forceinline__ int64_t in_ld(const Extra& ex) {
  if constexpr ((EX & EX_QKV) != 0) return ex.ild;
  return D;
}
constexpr float LOG2E = 1.4426950408889634f;
__device__ __forceinline__ uint32_t drop_mix(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}
__device__ __forceinline__ uint32_t drop_head(uint32_t seed, int64_t bh) {
  return drop_mix(seed ^ drop_mix((uint32_t)bh * 0x9e3779b1u + 0x632be5abu));
}
// the kernel's dropout seed: the host value, mixed with the device [seed, step] when present
__device__ __forceinline__ uint32_t ex_seed(const Extra& ex) {
  if (!ex.rng) return ex.seed;
  return ex.seed ^ drop_mix((uint32_t)ex.rng[0] ^ drop_mix((uint32_t)ex.rng[1] * 0x85ebca6bu + 0x27d4eb2fu));
}
// draws of (q, 2j) in the low and (q, 2j+1) in the high 16 bits
__device__ __forceinline__ uint32_t drop_pair(uint32_t hb, int q, int half_s, int j) {
  return drop_mix(((uint32_t)q * (uint32_t)half_s + (uint32_t)j) * 0x85ebca6bu ^ hb);
}

// EX_BIAS: the head's key-bias row (S fp32) is staged once in LDS behind the K/V double buffer
// and read per tile with broadcast LDS loads: per-tile global float4 loads of it tripled the
// vector-memory instructions of the encoder kernels (fwd 31 -> 51 us at B16 H16 S512 D64)
template <int D>
__device__ __forceinline__ float* stage_kbias(uint16_t* smem, const float* __restrict__ kbrow, int S) {
  float* kbs = reinterpret_cast<float*>(smem + 4 * BN2 * LDP<D>);
  for (int i = threadIdx.x; i < S / 4; i += blockDim.x)
    reinterpret_cast<float4*>(kbs)[i] = reinterpret_cast<const float4*>(kbrow)[i];
  return kbs;  // visible after the caller's first __syncthreads()
}

template <typename T, int D, bool CAUSAL, bool LAZY = true, int EX = 0, bool BUF = true, bool NL = true>
__global__ void __launch_bounds__(256, (D >= 128 ? 2 : 3)) fwd_v2_kernel(const uint16_t* __restrict__ Q, const uint16_t* __restrict__ K,
                                                        const uint16_t* __restrict__ V, uint16_t* __restrict__ O,
                                                        float* __restrict__ LSE, int S, float scale, int onh,
                                                        Extra ex = Extra()) {
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  constexpr int TS = BN2 * LDP<D>;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int h = lane >> 5, c32 = lane & 31;
  const int g16 = lane >> 4, qd = (lane & 15) >> 2, pc = lane & 3;
  // heaviest (last) causal row block of each head first, heads grouped per XCD
  const int nqb = (S + BM2 - 1) / BM2;
  const int task = xcd_task(blockIdx.x, gridDim.x);
  const int64_t bh = task / nqb;
  const int qb = (CAUSAL ? nqb - 1 - (task - (int)bh * nqb) : task - (int)bh * nqb) * BM2;
  const int myq = qb + 32 * w + c32;
  const int64_t ib = in_base<D, EX>(ex, bh, S), ldi = in_ld<D, EX>(ex);
  const uint16_t* Qb = Q + ib;
  const uint16_t* Kb = K + ib;
  const uint16_t* Vb = V + ib;
  constexpr bool BIAS = (EX & EX_BIAS) != 0, DROP = (EX & EX_DROP) != 0;
  const float* kbrow = BIAS ? ex.kbias + (bh / ex.hdiv) * (int64_t)S : nullptr;
  const uint32_t hb = DROP ? drop_head(ex_seed(ex), bh) : 0u;
  const float* kbs = BIAS ? stage_kbias<D>(smem, kbrow, S) : nullptr;

  s16x8 qf[D / 16];
#pragma unroll
  for (int ks = 0; ks < D / 16; ++ks)
    qf[ks] = myq < S ? *reinterpret_cast<const s16x8*>(Qb + (int64_t)myq * ldi + 16 * ks + 8 * h) : s16x8{};
  f32x16 o[D / 32];
#pragma unroll
  for (int dt = 0; dt < D / 32; ++dt)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[dt][r] = 0.f;
  float m = -INFINITY, l = 0.f;
  const float sl2 = scale * 1.4426950408889634f;

  const int kend = CAUSAL ? min(S, qb + BM2) : S;
  const int ntiles = (kend + BN2 - 1) / BN2;
  uint4 kr[D / 32], vr[D / 32];
  const __amdgpu_buffer_rsrc_t k_rs = head_rsrc(Kb, S, (int)ldi), v_rs = head_rsrc(Vb, S, (int)ldi);
  if constexpr (BUF && EX == 0) {
    tile_load_buf<D>(kr, k_rs, 0, (int)ldi);
    tile_load_buf<D>(vr, v_rs, 0, (int)ldi);
  } else {
    tile_load<D>(kr, Kb, 0, S, ldi);
    tile_load<D>(vr, Vb, 0, S, ldi);
  }
  tile_store<D>(smem, kr);
  tile_store<D, (NL ? LDPT<D> : LDP<D>)>(smem + TS, vr);
  __syncthreads();
  for (int it = 0; it < ntiles; ++it) {
    const int j0 = it * BN2;
    const bool has_next = it + 1 < ntiles;
    if (has_next) {
      if constexpr (BUF && EX == 0) {
        tile_load_buf<D>(kr, k_rs, j0 + BN2, (int)ldi);
        tile_load_buf<D>(vr, v_rs, j0 + BN2, (int)ldi);
      } else {
        tile_load<D>(kr, Kb, j0 + BN2, S, ldi);
        tile_load<D>(vr, Vb, j0 + BN2, S, ldi);
      }
    }
    const uint16_t* Ks = smem + (it & 1) * 2 * TS;
    const uint16_t* Vs = Ks + TS;
    float4 kb4[BIAS ? 8 : 1];  // this tile's key biases from the LDS-staged row
    if constexpr (BIAS) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int key0 = j0 + 32 * (i >> 2) + 8 * (i & 3) + 4 * h;
        kb4[i] = key0 < S ? *reinterpret_cast<const float4*>(kbs + key0) : make_float4(0, 0, 0, 0);
      }
    }
    float sv[32];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      f32x16 acc;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
      for (int ks = 0; ks < D / 16; ++ks)
        acc = Mfma32<T>::run(lds_row8(Ks + (32 * t + c32) * LDP<D> + 16 * ks + 8 * h), qf[ks], acc);
#pragma unroll
      for (int r = 0; r < 16; ++r) sv[16 * t + r] = acc[r];
    }
    // keys of value index 16t+r: j0 + 32t + 8(r>>2) + 4h + (r&3); this lane's query is myq.
    // Masking is only needed on the diagonal / ragged tiles (wave-uniform branch).
    if ((j0 + BN2 > S) || (CAUSAL && j0 + BN2 - 1 > qb + 32 * w)) {
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int key = j0 + 32 * t + 8 * (r >> 2) + 4 * h + (r & 3);
          if (key >= S || (CAUSAL && key > myq)) sv[16 * t + r] = -INFINITY;
        }
    }
    if constexpr (BIAS) {  // scores to the log2 domain with the key bias folded in (S % 8 == 0)
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int rb = 0; rb < 4; ++rb) {
          const float4 b4 = kb4[4 * t + rb];
          float* s4 = sv + 16 * t + 4 * rb;
          s4[0] = fmaf(s4[0], sl2, b4.x * LOG2E);
          s4[1] = fmaf(s4[1], sl2, b4.y * LOG2E);
          s4[2] = fmaf(s4[2], sl2, b4.z * LOG2E);
          s4[3] = fmaf(s4[3], sl2, b4.w * LOG2E);
        }
    }
    const float a2 = BIAS ? 1.f : sl2;
    // running max on raw scores (scale > 0 preserves order), exponent in the log2 domain:
    // p = 2^(s * scale*log2e - m) as one packed FMA + one v_exp_f32 per element
    float mx = -INFINITY;
#pragma unroll
    for (int i = 0; i < 32; ++i) mx = fmaxf(mx, sv[i]);
    mx = xhalf_max(mx);
    const float mt = mx * a2;
    if (!LAZY || __any(mt > m + LAZY_TH)) {  // wave-uniform
      const float mn = fmaxf(m, mt);
      const float alpha = fast_exp2(m - ((mn == -INFINITY) ? 0.f : mn));
      l *= alpha;
      m = mn;
#pragma unroll
      for (int dt = 0; dt < D / 32; ++dt)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[dt][r] *= alpha;
    }
    const float mu = (m == -INFINITY) ? 0.f : m;
    // two partial sums keep the dependent add chain short
    float ps = 0.f, ps1 = 0.f;
#pragma unroll
    for (int i = 0; i < 32; i += 2) {
      sv[i] = fast_exp2(fmaf(sv[i], a2, -mu));
      sv[i + 1] = fast_exp2(fmaf(sv[i + 1], a2, -mu));
      ps += sv[i];
      ps1 += sv[i + 1];
    }
    ps += ps1;
    ps = xhalf_sum(ps);
    l += ps;
    if constexpr (DROP) {  // values 2i, 2i+1 of a lane are keys 2j, 2j+1 of its query row
#pragma unroll
      for (int i = 0; i < 32; i += 2) {
        const int key = j0 + 32 * (i >> 4) + 8 * ((i & 15) >> 2) + 4 * h + (i & 3);
        const uint32_t x = drop_pair(hb, myq, S >> 1, key >> 1);
        const bool k0 = (x & 0xffffu) >= ex.thresh, k1 = (x >> 16) >= ex.thresh;
        if (!k0) sv[i] = 0.f;
        if (!k1) sv[i + 1] = 0.f;
      }
    }
    // O^T += V^T P^T over the 64 keys (4 steps of 16)
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const s16x8 pf = (sizeof(T) == 2 && __is_same(T, bf16_t)) ? pack8(sv, 8 * ks) : pack8_h(sv, 8 * ks);
      const int row1 = 16 * ks + 4 * (g16 >> 1) + qd;
#pragma unroll
      for (int dt = 0; dt < D / 32; ++dt) {
        const uint16_t* a0 = Vs + row1 * (NL ? LDPT<D> : LDP<D>) + 32 * dt + 16 * (g16 & 1) + 4 * pc;
        const s16x4 x = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0));
        const s16x4 y = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0 + 8 * (NL ? LDPT<D> : LDP<D>)));
        o[dt] = Mfma32<T>::run(s16x8{x[0], x[1], x[2], x[3], y[0], y[1], y[2], y[3]}, pf, o[dt]);
      }
    }
    if (has_next) {
      uint16_t* nxt = smem + ((it + 1) & 1) * 2 * TS;
      tile_store<D>(nxt, kr);
      tile_store<D, (NL ? LDPT<D> : LDP<D>)>(nxt + TS, vr);
    }
    __syncthreads();
  }
  if (myq < S) {
    const float inv = l > 0.f ? (DROP ? ex.rscale : 1.f) / l : 0.f;
    uint16_t* orow = O + o_base<D>(bh, S, onh) + (int64_t)myq * o_ld<D>(onh);
    // widened store (cdna_hip_programming T21): lanes c32 and c32 + 32 hold the two 4-element
    // halves of each 8-element group of the row; one v_permlane32_swap per dword pair hands
    // the lower lane groups rb, rb+1 = elements 16j .. 16j+7 and the upper lane 16j+8 .. 16j+15
#pragma unroll
    for (int dt = 0; dt < D / 32; ++dt)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        uint32_t a[2], b[2];
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          a[e] = (uint32_t)to16<T>(o[dt][8 * j + 2 * e] * inv) |
                 ((uint32_t)to16<T>(o[dt][8 * j + 2 * e + 1] * inv) << 16);
          b[e] = (uint32_t)to16<T>(o[dt][8 * j + 4 + 2 * e] * inv) |
                 ((uint32_t)to16<T>(o[dt][8 * j + 4 + 2 * e + 1] * inv) << 16);
          const auto r = __builtin_amdgcn_permlane32_swap(a[e], b[e], false, false);
          a[e] = r[0];
          b[e] = r[1];
        }
        *reinterpret_cast<uint4*>(orow + 32 * dt + 16 * j + 8 * h) = make_uint4(a[0], a[1], b[0], b[1]);
      }
    if (h == 0)
      // a row with every key masked out stores +inf so the backward recomputes P = 0 for it
      LSE[bh * (int64_t)S + myq] = (m == -INFINITY) ? INFINITY : (m + log2f(l)) * 0.6931471805599453f;
  }
}

// ======================================================================== backward v2
// dK/dV: one wave = 32 keys (lane = key column of S = Q K^T); K, V are B operands held in
// registers; per 64-query tile: S, dP (A = Q / dO rows from LDS), P, dS in registers (query
// index per value from the C layout, LSE/Delta broadcast from LDS), then
//   dV^T += dO^T P   (A = dO^T via tr reads, B = P from registers)
//   dK^T += Q^T dS   (A = Q^T via tr reads,  B = dS from registers)
// V3 (no dropout): the row constants enter as the MFMAs' initial accumulators -- S starts at
// -LSE / scale and dP at -Delta (the "row constants as initial accumulator" idiom), read from
// LDS as one float4 per 4 C-layout rows instead of 16 scalar broadcasts per 32-query half --
// so P = exp2(S' * scale * log2e) and dS = P * dP' need no per-element subtraction.
template <typename T, int D, bool CAUSAL, int EX = 0, bool FQ = false, bool BUF = true, bool V3 = false>
__device__ __forceinline__ void dkdv_v2_body(int vblock, int nblock, const uint16_t* __restrict__ Q,
                                             const uint16_t* __restrict__ K, const uint16_t* __restrict__ V,
                                             const uint16_t* __restrict__ dO, const float* __restrict__ LSE,
                                             const float* __restrict__ DELTA, uint16_t* __restrict__ dK,
                                             uint16_t* __restrict__ dV, int S, float scale, int onh, const Extra& ex,
                                             uint16_t* __restrict__ dQ = nullptr, const uint16_t* __restrict__ Ofw = nullptr) {
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  constexpr int TS = BN2 * LDP<D>;
  float* stats = reinterpret_cast<float*>(smem + 4 * TS);  // [2 stages][LSE 64 | DELTA 64]
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int h = lane >> 5, c32 = lane & 31;
  const int g16 = lane >> 4, qd = (lane & 15) >> 2, pc = lane & 3;
  const int nkb = (S + BM2 - 1) / BM2;
  const int task = xcd_task(vblock, nblock);
  const int64_t bh = task / nkb;
  const int kb = (task - (int)bh * nkb) * BM2;
  const int mykey = kb + 32 * w + c32;
  const int64_t base = in_base<D, EX>(ex, bh, S), ldi = in_ld<D, EX>(ex);
  const int64_t obase = o_base<D>(bh, S, onh);
  const float sl2 = scale * 1.4426950408889634f;
  constexpr bool BIAS = (EX & EX_BIAS) != 0, DROP = (EX & EX_DROP) != 0;
  constexpr bool INIT = V3 && !DROP;
  // Q, dO: swizzled dual-use images -- off: at D = 96 this kernel is at 256 VGPRs and the image's
  // extra lane bases cost 48 spilled registers (kSwzDkdv = true builds it for A/B runs)
  constexpr int kSwzDkdv = 0;  // bit 0: Q image, bit 1: dO image
  constexpr bool SWQ = (kSwzDkdv & 1) && D == 96 && EX == 0 && !FQ;
  constexpr bool SWO = (kSwzDkdv & 2) && D == 96 && EX == 0 && !FQ;
  const SwzLanes<D> sz(lane);
  // this lane's key bias (log2 units) and which 16-bit half of a pair draw is its key's
  const float kb2 = (BIAS && mykey < S) ? ex.kbias[(bh / ex.hdiv) * (int64_t)S + mykey] * LOG2E : 0.f;
  const uint32_t hb = DROP ? drop_head(ex_seed(ex), bh) : 0u;
  const int dshift = (mykey & 1) * 16;
  // FQ (S <= BM2: this workgroup owns every key of the head): K [BM2][D+8] and the tile's dS
  // [BN2 queries][BM2 + 8 keys] also live in LDS, and dQ = dS K is formed per query tile here
  uint16_t* const Ks = smem + 4 * TS + 4 * BN2 * 2;
  uint16_t* const dSs = Ks + BM2 * LDP<D>;
  // FQ with the forward output O: Delta = rowsum(dO * O) of the head's S <= BM2 queries is formed
  // here into LDS (8 lanes per row, 16-byte loads) instead of by a separate pass over dO and O
  float* const dls = reinterpret_cast<float*>(dSs + BN2 * (BM2 + 8));
  if constexpr (FQ) {
    uint4 kr2[D / 32];
    tile_load<D>(kr2, K + base, 0, S, ldi);
    tile_store<D>(Ks, kr2);
    tile_load<D>(kr2, K + base, BN2, S, ldi);
    tile_store<D>(Ks + BN2 * LDP<D>, kr2);
    if (Ofw) {
      const int sub = threadIdx.x & 7;
      for (int q = threadIdx.x >> 3; q < BM2; q += 32) {  // uniform trip count: every lane shuffles
        float acc = 0.f;
        if (q < S) {
          const int64_t off = obase + (int64_t)q * o_ld<D>(onh);
          for (int c = sub; c < D / 8; c += 8) {
            float a[8], b[8];
            Vec16<T>::load(reinterpret_cast<const T*>(dO) + off + c * 8, a);
            Vec16<T>::load(reinterpret_cast<const T*>(Ofw) + off + c * 8, b);
#pragma unroll
            for (int j = 0; j < 8; ++j) acc = fmaf(a[j], b[j], acc);
          }
        }
        acc += __shfl_xor(acc, 1, 64);
        acc += __shfl_xor(acc, 2, 64);
        acc += __shfl_xor(acc, 4, 64);
        if (sub == 0) dls[q] = acc;
      }
      __syncthreads();
    }
  }

  s16x8 kf[D / 16], vf[D / 16];
#pragma unroll
  for (int ks = 0; ks < D / 16; ++ks) {
    kf[ks] = mykey < S ? *reinterpret_cast<const s16x8*>(K + base + (int64_t)mykey * ldi + 16 * ks + 8 * h) : s16x8{};
    vf[ks] = mykey < S ? *reinterpret_cast<const s16x8*>(V + base + (int64_t)mykey * ldi + 16 * ks + 8 * h) : s16x8{};
  }
  f32x16 dk[D / 32], dv[D / 32];
#pragma unroll
  for (int dt = 0; dt < D / 32; ++dt)
#pragma unroll
    for (int r = 0; r < 16; ++r) { dk[dt][r] = 0.f; dv[dt][r] = 0.f; }

  const int qstart = CAUSAL ? kb : 0;
  const int ntiles = qstart < S ? (S - qstart + BN2 - 1) / BN2 : 0;
  uint4 qr[D / 32], orr[D / 32];
  float st_l = 0.f, st_d = 0.f;
  const __amdgpu_buffer_rsrc_t q_rs = head_rsrc(Q + base, S, (int)ldi);
  const __amdgpu_buffer_rsrc_t o_rs = head_rsrc(dO + obase, S, o_ld<D>(onh));
  auto load_tile = [&](int i0) {
    if constexpr (BUF && EX == 0) {
      tile_load_buf<D>(qr, q_rs, i0, (int)ldi);
      tile_load_buf<D>(orr, o_rs, i0, o_ld<D>(onh));
    } else {
      tile_load<D>(qr, Q + base, i0, S, ldi);
      tile_load<D>(orr, dO + obase, i0, S, o_ld<D>(onh));
    }
    if (threadIdx.x < BN2) {
      const int q = i0 + threadIdx.x;
      const float dq_ = q < S ? ((FQ && Ofw) ? dls[q] : DELTA[bh * (int64_t)S + q]) : 0.f;
      st_l = q < S ? LSE[bh * (int64_t)S + q] * (INIT ? -1.f / scale : 1.4426950408889634f) : 0.f;
      st_d = INIT ? -dq_ : dq_;
    }
  };
  auto store_tile = [&](int stage) {
    uint16_t* b = smem + stage * 2 * TS;
    tile_put<D, SWQ>(b, qr);
    tile_put<D, SWO>(b + TS, orr);
    if (threadIdx.x < BN2) {
      stats[stage * 2 * BN2 + threadIdx.x] = st_l;
      stats[stage * 2 * BN2 + BN2 + threadIdx.x] = st_d;
    }
  };
  if (ntiles > 0) {
    load_tile(qstart);
    store_tile(0);
  }
  __syncthreads();
  for (int it = 0; it < ntiles; ++it) {
    const int i0 = qstart + it * BN2;
    const bool has_next = it + 1 < ntiles;
    // V3 stages the next tile in two halves (Q during the first 32-query half, dO during the
    // second) so only one half's registers are live at a time
    if (has_next) {
      if constexpr (V3) {
        tile_load_buf<D>(qr, q_rs, i0 + BN2, (int)ldi);
        if (threadIdx.x < BN2) {
          const int q = i0 + BN2 + threadIdx.x;
          // stored negated: they become the initial accumulators as they are
          st_l = q < S ? LSE[bh * (int64_t)S + q] * (INIT ? -1.f / scale : 1.4426950408889634f) : 0.f;
          st_d = q < S ? (INIT ? -DELTA[bh * (int64_t)S + q] : DELTA[bh * (int64_t)S + q]) : 0.f;
        }
      } else {
        load_tile(i0 + BN2);
      }
    }
    const uint16_t* Qs = smem + (it & 1) * 2 * TS;
    const uint16_t* Os = Qs + TS;
    const float* lse_s = stats + (it & 1) * 2 * BN2;
    const float* del_s = lse_s + BN2;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      if constexpr (V3) {
        if (t == 1 && has_next) {
          const int nx = (it + 1) & 1;
          tile_put<D, SWQ>(smem + nx * 2 * TS, qr);
          if (threadIdx.x < BN2) {
            stats[nx * 2 * BN2 + threadIdx.x] = st_l;
            stats[nx * 2 * BN2 + BN2 + threadIdx.x] = st_d;
          }
          tile_load_buf<D>(orr, o_rs, i0 + BN2, o_ld<D>(onh));
        }
      }
      f32x16 sacc, pacc;
      if constexpr (INIT) {
#pragma unroll
        for (int rb = 0; rb < 4; ++rb) {
          const float4 l4 = *reinterpret_cast<const float4*>(lse_s + 32 * t + 8 * rb + 4 * h);
          const float4 d4 = *reinterpret_cast<const float4*>(del_s + 32 * t + 8 * rb + 4 * h);
          sacc[4 * rb + 0] = l4.x; sacc[4 * rb + 1] = l4.y; sacc[4 * rb + 2] = l4.z; sacc[4 * rb + 3] = l4.w;
          pacc[4 * rb + 0] = d4.x; pacc[4 * rb + 1] = d4.y; pacc[4 * rb + 2] = d4.z; pacc[4 * rb + 3] = d4.w;
        }
      } else {
#pragma unroll
        for (int r = 0; r < 16; ++r) { sacc[r] = 0.f; pacc[r] = 0.f; }
      }
#pragma unroll
      for (int ks = 0; ks < D / 16; ++ks) {
        const int rp = (32 * t + c32) * LDP<D> + 16 * ks + 8 * h;
        sacc = Mfma32<T>::run(lds_row8(Qs + (SWQ ? sz.row(t, ks) : rp)), kf[ks], sacc);
        pacc = Mfma32<T>::run(lds_row8(Os + (SWO ? sz.row(t, ks) : rp)), vf[ks], pacc);
      }
      float pv[16], dsv[16];
      if constexpr (INIT) {
#pragma unroll
        for (int r = 0; r < 16; ++r) pv[r] = fast_exp2(BIAS ? fmaf(sacc[r], sl2, kb2) : sacc[r] * sl2);
      } else {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int qi = 32 * t + 8 * (r >> 2) + 4 * h + (r & 3);
          pv[r] = fast_exp2(fmaf(sacc[r], sl2, BIAS ? kb2 - lse_s[qi] : -lse_s[qi]));
        }
      }
      // wave-uniform: ragged tail or a query of this sub-tile before the wave's last key
      if ((i0 + 32 * t + 32 > S) || (kb + 32 * w + 32 > S) || (CAUSAL && kb + 32 * w + 31 > i0 + 32 * t)) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int q = i0 + 32 * t + 8 * (r >> 2) + 4 * h + (r & 3);
          if (q >= S || mykey >= S || (CAUSAL && mykey > q)) pv[r] = 0.f;
        }
      }
      if constexpr (DROP) {  // dV from the dropped P; dP = dP_dropped * Z / (1 - p)
        // lanes l and l^1 hold keys 2j and 2j+1 of the same 16 queries and need the same 16
        // pair draws: each computes 8 and takes the other 8 from its neighbour (DPP quad_perm)
        uint32_t own[8], nbr[8];
        const int half = (mykey & 1) * 8;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const int r = half + k;
          own[k] = drop_pair(hb, i0 + 32 * t + 8 * (r >> 2) + 4 * h + (r & 3), S >> 1, mykey >> 1);
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) nbr[k] = (uint32_t)__builtin_amdgcn_mov_dpp((int)own[k], 0xB1, 0xF, 0xF, true);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int qi = 32 * t + 8 * (r >> 2) + 4 * h + (r & 3);
          const uint32_t x = ((r >> 3) == (mykey & 1)) ? own[r & 7] : nbr[r & 7];
          const float zr = ((x >> dshift) & 0xffffu) < ex.thresh ? 0.f : ex.rscale;
          dsv[r] = pv[r] * fmaf(pacc[r], zr, -del_s[qi]);
          pv[r] *= zr;
        }
      } else if constexpr (INIT) {
#pragma unroll
        for (int r = 0; r < 16; ++r) dsv[r] = pv[r] * pacc[r];
      } else {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int qi = 32 * t + 8 * (r >> 2) + 4 * h + (r & 3);
          dsv[r] = pv[r] * (pacc[r] - del_s[qi]);
        }
      }
      if constexpr (FQ) {  // dS[q][key] for the tile's dQ (all 4 waves' keys)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          dSs[(32 * t + 8 * (r >> 2) + 4 * h + (r & 3)) * (BM2 + 8) + 32 * w + c32] = to16<T>(dsv[r]);
      }
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int ks = 2 * t + kk;
        const s16x8 pf = __is_same(T, bf16_t) ? pack8(pv, 8 * kk) : pack8_h(pv, 8 * kk);
        const s16x8 sf = __is_same(T, bf16_t) ? pack8(dsv, 8 * kk) : pack8_h(dsv, 8 * kk);
        const int row1 = 16 * ks + 4 * (g16 >> 1) + qd;
#pragma unroll
        for (int dt = 0; dt < D / 32; ++dt) {
          const int col = 32 * dt + 16 * (g16 & 1) + 4 * pc;
          const int px = row1 * LDP<D> + col, py = (row1 + 8) * LDP<D> + col;
          const s16x4 ox = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(Os + (SWO ? sz.tr(ks, 0, dt) : px)));
          const s16x4 oy = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(Os + (SWO ? sz.tr(ks, 1, dt) : py)));
          dv[dt] = Mfma32<T>::run(s16x8{ox[0], ox[1], ox[2], ox[3], oy[0], oy[1], oy[2], oy[3]}, pf, dv[dt]);
          const s16x4 qx = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(Qs + (SWQ ? sz.tr(ks, 0, dt) : px)));
          const s16x4 qy = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(Qs + (SWQ ? sz.tr(ks, 1, dt) : py)));
          dk[dt] = Mfma32<T>::run(s16x8{qx[0], qx[1], qx[2], qx[3], qy[0], qy[1], qy[2], qy[3]}, sf, dk[dt]);
        }
        if constexpr (V3) __builtin_amdgcn_sched_barrier(0);  // bounds the tr-read hoisting: 0 spills vs 12
      }
    }
    if constexpr (FQ) {
      // dQ^T[d, q] = sum_k K^T[d, k] dS^T[k, q] for this 64-query tile: wave w owns query block
      // w >> 1 and d blocks (w & 1) + 2j; K^T fragments by transposed LDS reads, dS^T fragments
      // are 4+4 keys of one query row (the C-layout key order the dQ kernel uses)
      __syncthreads();
      const int qb2 = w >> 1;
#pragma unroll
      for (int dj = 0; dj < D / 64; ++dj) {
        const int dt = (w & 1) + 2 * dj;
        f32x16 dq;
#pragma unroll
        for (int r = 0; r < 16; ++r) dq[r] = 0.f;
#pragma unroll
        for (int ks = 0; ks < BM2 / 16; ++ks) {
          const uint16_t* srow = dSs + (32 * qb2 + c32) * (BM2 + 8) + 16 * ks + 4 * h;
          const s16x4 lo = *reinterpret_cast<const s16x4*>(srow);
          const s16x4 hi = *reinterpret_cast<const s16x4*>(srow + 8);
          const int row1 = 16 * ks + 4 * (g16 >> 1) + qd;
          const int col = 32 * dt + 16 * (g16 & 1) + 4 * pc;
          const s16x4 x = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(Ks + row1 * LDP<D> + col));
          const s16x4 y = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(Ks + (row1 + 8) * LDP<D> + col));
          dq = Mfma32<T>::run(s16x8{x[0], x[1], x[2], x[3], y[0], y[1], y[2], y[3]},
                              s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]}, dq);
        }
        const int myq = i0 + 32 * qb2 + c32;
        if (myq < S) {
          uint16_t* dqr = dQ + base + (int64_t)myq * ldi;
#pragma unroll
          for (int rb = 0; rb < 4; ++rb) {
            ushort4 v4;
            v4.x = to16<T>(dq[4 * rb + 0] * scale); v4.y = to16<T>(dq[4 * rb + 1] * scale);
            v4.z = to16<T>(dq[4 * rb + 2] * scale); v4.w = to16<T>(dq[4 * rb + 3] * scale);
            *reinterpret_cast<ushort4*>(dqr + 32 * dt + 8 * rb + 4 * h) = v4;
          }
        }
      }
    }
    if (has_next) {
      if constexpr (V3)
        tile_put<D, SWO>(smem + ((it + 1) & 1) * 2 * TS + TS, orr);
      else
        store_tile((it + 1) & 1);
    }
    __syncthreads();
  }
  if (mykey < S) {
    uint16_t* dkr = dK + base + (int64_t)mykey * ldi;
    uint16_t* dvr = dV + base + (int64_t)mykey * ldi;
#pragma unroll
    for (int dt = 0; dt < D / 32; ++dt)
#pragma unroll
      for (int rb = 0; rb < 4; ++rb) {
        ushort4 a4, b4;
        a4.x = to16<T>(dk[dt][4 * rb + 0] * scale); a4.y = to16<T>(dk[dt][4 * rb + 1] * scale);
        a4.z = to16<T>(dk[dt][4 * rb + 2] * scale); a4.w = to16<T>(dk[dt][4 * rb + 3] * scale);
        b4.x = to16<T>(dv[dt][4 * rb + 0]); b4.y = to16<T>(dv[dt][4 * rb + 1]);
        b4.z = to16<T>(dv[dt][4 * rb + 2]); b4.w = to16<T>(dv[dt][4 * rb + 3]);
        *reinterpret_cast<ushort4*>(dkr + 32 * dt + 8 * rb + 4 * h) = a4;
        *reinterpret_cast<ushort4*>(dvr + 32 * dt + 8 * rb + 4 * h) = b4;
      }
  }
}

// dQ: one wave = 32 queries (lane = query column of S^T = K Q^T); Q and dO are B operands in
// registers; per 64-key tile: S^T, dP^T (A = K / V rows from LDS), dS^T in registers, then
//   dQ^T += K^T dS^T   (A = K^T via tr reads, B = dS^T from registers)
// FD (fused delta): the workgroup that owns a query row also forms its Delta = rowsum(dO * O)
// from the dO fragments it holds anyway plus the matching O fragments, uses it, and stores it
// for the dK/dV kernel that runs after it -- no separate Delta pass over dO and O.
template <typename T, int D, bool CAUSAL, int EX = 0, bool BUF = true, bool FD = false, bool NL = true>
__device__ __forceinline__ void dq_v2_body(int vblock, int nblock, const uint16_t* __restrict__ Q,
                                           const uint16_t* __restrict__ K, const uint16_t* __restrict__ V,
                                           const uint16_t* __restrict__ dO, const float* __restrict__ LSE,
                                           const float* __restrict__ DELTA, uint16_t* __restrict__ dQ, int S,
                                           float scale, int onh, const Extra& ex,
                                           const uint16_t* __restrict__ O = nullptr) {
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  constexpr int TS = BN2 * LDP<D>;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int h = lane >> 5, c32 = lane & 31;
  const int g16 = lane >> 4, qd = (lane & 15) >> 2, pc = lane & 3;
  const int nqb = (S + BM2 - 1) / BM2;
  const int task = xcd_task(vblock, nblock);
  const int64_t bh = task / nqb;
  const int qb = (CAUSAL ? nqb - 1 - (task - (int)bh * nqb) : task - (int)bh * nqb) * BM2;
  const int myq = qb + 32 * w + c32;
  const int64_t base = in_base<D, EX>(ex, bh, S), ldi = in_ld<D, EX>(ex);
  const float sl2 = scale * 1.4426950408889634f;
  constexpr bool BIAS = (EX & EX_BIAS) != 0, DROP = (EX & EX_DROP) != 0;
  constexpr bool SW = NL && D == 96 && EX == 0;  // K: swizzled dual-use image (row + transposed reads)
  const SwzLanes<D> sz(lane);
  const float* kbrow = BIAS ? ex.kbias + (bh / ex.hdiv) * (int64_t)S : nullptr;
  const uint32_t hb = DROP ? drop_head(ex_seed(ex), bh) : 0u;
  const float* kbs = BIAS ? stage_kbias<D>(smem, kbrow, S) : nullptr;

  s16x8 qf[D / 16], of[D / 16];
#pragma unroll
  for (int ks = 0; ks < D / 16; ++ks) {
    qf[ks] = myq < S ? *reinterpret_cast<const s16x8*>(Q + base + (int64_t)myq * ldi + 16 * ks + 8 * h) : s16x8{};
    of[ks] = myq < S ? *reinterpret_cast<const s16x8*>(dO + o_base<D>(bh, S, onh) + (int64_t)myq * o_ld<D>(onh) +
                                                         16 * ks + 8 * h)
                     : s16x8{};
  }
  const float lse2 = myq < S ? LSE[bh * (int64_t)S + myq] * 1.4426950408889634f : 0.f;
  float dl;
  if constexpr (FD) {
    // this lane holds half of its query's dO row (dims 16ks + 8h .. +7); the lane pair sums
    float part = 0.f;
    if (myq < S) {
      const uint16_t* orow = O + o_base<D>(bh, S, onh) + (int64_t)myq * o_ld<D>(onh) + 8 * h;
#pragma unroll
      for (int ks = 0; ks < D / 16; ++ks) {
        float a[8], b[8];
        Vec16<T>::load(reinterpret_cast<const T*>(orow) + 16 * ks, b);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          a[j] = __is_same(T, bf16_t) ? bf16_to_f32((uint16_t)of[ks][j]) : f16_to_f32((uint16_t)of[ks][j]);
          part = fmaf(a[j], b[j], part);
        }
      }
    }
    dl = xhalf_sum(part);
    if (myq < S && h == 0) const_cast<float*>(DELTA)[bh * (int64_t)S + myq] = dl;
  } else {
    dl = myq < S ? DELTA[bh * (int64_t)S + myq] : 0.f;
  }
  f32x16 dq[D / 32];
#pragma unroll
  for (int dt = 0; dt < D / 32; ++dt)
#pragma unroll
    for (int r = 0; r < 16; ++r) dq[dt][r] = 0.f;

  const int kend = CAUSAL ? min(S, qb + BM2) : S;
  const int ntiles = (kend + BN2 - 1) / BN2;
  uint4 kr[D / 32], vr[D / 32];
  const __amdgpu_buffer_rsrc_t k_rs = head_rsrc(K + base, S, (int)ldi), v_rs = head_rsrc(V + base, S, (int)ldi);
  if constexpr (BUF && EX == 0) {
    tile_load_buf<D>(kr, k_rs, 0, (int)ldi);
    tile_load_buf<D>(vr, v_rs, 0, (int)ldi);
  } else {
    tile_load<D>(kr, K + base, 0, S, ldi);
    tile_load<D>(vr, V + base, 0, S, ldi);
  }
  tile_put<D, SW>(smem, kr);
  tile_store<D>(smem + TS, vr);
  __syncthreads();
  for (int it = 0; it < ntiles; ++it) {
    const int j0 = it * BN2;
    const bool has_next = it + 1 < ntiles;
    if (has_next) {
      if constexpr (BUF && EX == 0) {
        tile_load_buf<D>(kr, k_rs, j0 + BN2, (int)ldi);
        tile_load_buf<D>(vr, v_rs, j0 + BN2, (int)ldi);
      } else {
        tile_load<D>(kr, K + base, j0 + BN2, S, ldi);
        tile_load<D>(vr, V + base, j0 + BN2, S, ldi);
      }
    }
    const uint16_t* Ks = smem + (it & 1) * 2 * TS;
    const uint16_t* Vs = Ks + TS;
    float4 kb4[BIAS ? 8 : 1];  // the tile's key biases from the LDS-staged row
    if constexpr (BIAS) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int key0 = j0 + 32 * (i >> 2) + 8 * (i & 3) + 4 * h;
        kb4[i] = key0 < S ? *reinterpret_cast<const float4*>(kbs + key0) : make_float4(0, 0, 0, 0);
      }
    }
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      f32x16 sacc, pacc;
#pragma unroll
      for (int r = 0; r < 16; ++r) { sacc[r] = 0.f; pacc[r] = 0.f; }
#pragma unroll
      for (int ks = 0; ks < D / 16; ++ks) {
        sacc = Mfma32<T>::run(lds_row8(SW ? Ks + sz.row(t, ks) : Ks + (32 * t + c32) * LDP<D> + 16 * ks + 8 * h),
                              qf[ks], sacc);
        pacc = Mfma32<T>::run(lds_row8(Vs + (32 * t + c32) * LDP<D> + 16 * ks + 8 * h), of[ks], pacc);
      }
      float dsv[16];
      if constexpr (BIAS) {
#pragma unroll
        for (int rb = 0; rb < 4; ++rb) {
          const float4 b4 = kb4[4 * t + rb];
          dsv[4 * rb + 0] = fast_exp2(fmaf(sacc[4 * rb + 0], sl2, fmaf(b4.x, LOG2E, -lse2)));
          dsv[4 * rb + 1] = fast_exp2(fmaf(sacc[4 * rb + 1], sl2, fmaf(b4.y, LOG2E, -lse2)));
          dsv[4 * rb + 2] = fast_exp2(fmaf(sacc[4 * rb + 2], sl2, fmaf(b4.z, LOG2E, -lse2)));
          dsv[4 * rb + 3] = fast_exp2(fmaf(sacc[4 * rb + 3], sl2, fmaf(b4.w, LOG2E, -lse2)));
        }
      } else {
#pragma unroll
        for (int r = 0; r < 16; ++r) dsv[r] = fast_exp2(fmaf(sacc[r], sl2, -lse2));
      }
      if ((j0 + 32 * t + 32 > S) || (qb + 32 * w + 32 > S) || (CAUSAL && j0 + 32 * t + 31 > qb + 32 * w)) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int key = j0 + 32 * t + 8 * (r >> 2) + 4 * h + (r & 3);
          if (key >= S || myq >= S || (CAUSAL && key > myq)) dsv[r] = 0.f;
        }
      }
      if constexpr (DROP) {  // values r, r+1 are keys 2j, 2j+1 of this lane's query
#pragma unroll
          for (int r = 0; r < 16; r += 2) {
            const int key = j0 + 32 * t + 8 * (r >> 2) + 4 * h + (r & 3);
            const uint32_t x = drop_pair(hb, myq, S >> 1, key >> 1);
            const float z0 = (x & 0xffffu) < ex.thresh ? 0.f : ex.rscale;
            const float z1 = (x >> 16) < ex.thresh ? 0.f : ex.rscale;
            dsv[r] = dsv[r] * fmaf(pacc[r], z0, -dl);
            dsv[r + 1] = dsv[r + 1] * fmaf(pacc[r + 1], z1, -dl);
          }
      } else {
#pragma unroll
        for (int r = 0; r < 16; ++r) dsv[r] = dsv[r] * (pacc[r] - dl);
      }
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int ks = 2 * t + kk;
        const s16x8 sf = __is_same(T, bf16_t) ? pack8(dsv, 8 * kk) : pack8_h(dsv, 8 * kk);
        const int row1 = 16 * ks + 4 * (g16 >> 1) + qd;
#pragma unroll
        for (int dt = 0; dt < D / 32; ++dt) {
          const int col = 32 * dt + 16 * (g16 & 1) + 4 * pc;
          const uint16_t* kx = SW ? Ks + sz.tr(ks, 0, dt) : Ks + row1 * LDP<D> + col;
          const uint16_t* ky = SW ? Ks + sz.tr(ks, 1, dt) : Ks + (row1 + 8) * LDP<D> + col;
          const s16x4 x = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(kx));
          const s16x4 y = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(ky));
          dq[dt] = Mfma32<T>::run(s16x8{x[0], x[1], x[2], x[3], y[0], y[1], y[2], y[3]}, sf, dq[dt]);
        }
      }
    }
    if (has_next) {
      uint16_t* nxt = smem + ((it + 1) & 1) * 2 * TS;
      tile_put<D, SW>(nxt, kr);
      tile_store<D>(nxt + TS, vr);
    }
    __syncthreads();
  }
  if (myq < S) {
    uint16_t* dqr = dQ + base + (int64_t)myq * ldi;
#pragma unroll
    for (int dt = 0; dt < D / 32; ++dt)
#pragma unroll
      for (int rb = 0; rb < 4; ++rb) {
        ushort4 v4;
        v4.x = to16<T>(dq[dt][4 * rb + 0] * scale); v4.y = to16<T>(dq[dt][4 * rb + 1] * scale);
        v4.z = to16<T>(dq[dt][4 * rb + 2] * scale); v4.w = to16<T>(dq[dt][4 * rb + 3] * scale);
        *reinterpret_cast<ushort4*>(dqr + 32 * dt + 8 * rb + 4 * h) = v4;
      }
  }
}


// kernel entry points: the two backward halves on their own, or both in one launch (dK/dV
// workgroups first, then dQ): at short sequences each half alone is latency-bound and leaves
// the chip idle in its tail, one grid lets the hardware overlap them
template <typename T, int D, bool CAUSAL, int EX = 0, bool BUF = true>
__global__ void __launch_bounds__(256, (D >= 128 ? 1 : 2)) bwd_dkdv_v2_kernel(
    const uint16_t* __restrict__ Q, const uint16_t* __restrict__ K, const uint16_t* __restrict__ V,
    const uint16_t* __restrict__ dO, const float* __restrict__ LSE, const float* __restrict__ DELTA,
    uint16_t* __restrict__ dK, uint16_t* __restrict__ dV, int S, float scale, int onh, Extra ex = Extra()) {
  dkdv_v2_body<T, D, CAUSAL, EX, false, BUF>(blockIdx.x, gridDim.x, Q, K, V, dO, LSE, DELTA, dK, dV, S, scale, onh,
                                             ex);
}

// dQ that also forms and stores Delta (runs before the dK/dV kernel, which reads it)
template <typename T, int D, bool CAUSAL, bool NL = true>
__global__ void __launch_bounds__(256, 2) bwd_dq_v3_kernel(
    const uint16_t* __restrict__ Q, const uint16_t* __restrict__ K, const uint16_t* __restrict__ V,
    const uint16_t* __restrict__ dO, const uint16_t* __restrict__ O, const float* __restrict__ LSE,
    float* __restrict__ DELTA, uint16_t* __restrict__ dQ, int S, float scale, int onh) {
  dq_v2_body<T, D, CAUSAL, 0, true, true, NL>(blockIdx.x, gridDim.x, Q, K, V, dO, LSE, DELTA, dQ, S, scale, onh, Extra(),
                                          O);
}

// dK/dV with the initial-accumulator row constants (V3), two waves per SIMD (D <= 96)
template <typename T, int D, bool CAUSAL>
__global__ void __launch_bounds__(256, 2) bwd_dkdv_v3_kernel(
    const uint16_t* __restrict__ Q, const uint16_t* __restrict__ K, const uint16_t* __restrict__ V,
    const uint16_t* __restrict__ dO, const float* __restrict__ LSE, const float* __restrict__ DELTA,
    uint16_t* __restrict__ dK, uint16_t* __restrict__ dV, int S, float scale, int onh) {
  dkdv_v2_body<T, D, CAUSAL, 0, false, true, true>(blockIdx.x, gridDim.x, Q, K, V, dO, LSE, DELTA, dK, dV, S,
                                                   scale, onh, Extra());
}

// ======================================================================== backward: dK/dV, wave pairs
// dkdv_v2_body keeps dK and dV (2 x D/2 accumulator registers), the K and V fragments (2 x D/4)
// and the staging of both tiles in ONE wave; at D = 128 that fits only at one wave per SIMD,
// which leaves nothing to hide the LDS latency (247 TF/s at B16 H16 S2048 causal vs 361 at
// D = 96 with two).  Here each 32-key group is owned by a PAIR of waves of a 512-thread
// workgroup, one per role, so every wave holds half that state and two run per SIMD:
//   role 0 (waves 0-3): S = Q K^T -> P, dV^T += dO^T P   (K fragments, dV; stages Q + LSE)
//   role 1 (waves 4-7): dP = dO V^T, dS = P (dP - Delta), dK^T += Q^T dS   (V, dK; dO + Delta)
// P crosses from role 0 to role 1 through LDS as the packed 16-bit B fragments role 0 feeds its
// own dV MFMAs: both sides hold the score tile in the same C layout (lane = key), so it is a
// plain per-lane copy.  The exchange is software-pipelined so both roles issue 16 MFMAs between
// the two barriers of a 64-query tile (half = 32 queries):
//   A: role 0: dV += previous tile's half 1 (P1 in registers); S of half 0 -> P0 to LDS
//      role 1: dK += previous tile's half 1 (P1 from LDS);     dP of half 0
//   -- barrier --
//   B: role 0: dV += half 0; S of half 1 -> P1 to LDS (and kept for the next A)
//      role 1: dK += half 0 (P0 from LDS); dP of half 1 (kept for the next A)
//      the next Q / dO tile goes into the other LDS buffer (its last readers ran in A)
//   -- barrier --
// The row constants enter as initial accumulators (S at -LSE/scale, dP at -Delta), as in V3.
template <int D>
__device__ __forceinline__ void tile_load_buf_t(uint4 (&r)[D / 32], __amdgpu_buffer_rsrc_t rs, int r0, int ld,
                                                int tid) {
  constexpr int CH = D / 8;
#pragma unroll
  for (int k = 0; k < D / 32; ++k) {
    const int c = tid + 256 * k;
    const int row = c / CH, ch = c - row * CH;
    const fa_u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, ((r0 + row) * ld + ch * 8) * 2, 0, 0);
    r[k] = make_uint4(v.x, v.y, v.z, v.w);
  }
}
template <int D>
__device__ __forceinline__ void tile_store_t(uint16_t* lds, const uint4 (&r)[D / 32], int tid) {
  constexpr int CH = D / 8;
#pragma unroll
  for (int k = 0; k < D / 32; ++k) {
    const int c = tid + 256 * k;
    const int row = c / CH, ch = c - row * CH;
    *reinterpret_cast<uint4*>(lds + row * LDP<D> + ch * 8) = r[k];
  }
}
__device__ __forceinline__ void tohold(f32x16& hold, const s16x8 (&f)[2]) {
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    const f32x4 v = __builtin_bit_cast(f32x4, f[kk]);
#pragma unroll
    for (int j = 0; j < 4; ++j) hold[4 * kk + j] = v[j];
  }
}
__device__ __forceinline__ void unhold(const f32x16& hold, s16x8 (&f)[2]) {
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) f[kk] = __builtin_bit_cast(s16x8, f32x4{hold[4 * kk], hold[4 * kk + 1], hold[4 * kk + 2], hold[4 * kk + 3]});
}
template <int D> constexpr int dkdv_pair_lds() { return 2 * 2 * BN2 * LDP<D> * 2 + 2 * 2 * BN2 * 4 + 2 * 4 * 2 * 64 * 16; }

template <typename T, int D, bool CAUSAL>
__global__ void __launch_bounds__(512, 2) bwd_dkdv_pair_kernel(
    const uint16_t* __restrict__ Q, const uint16_t* __restrict__ K, const uint16_t* __restrict__ V,
    const uint16_t* __restrict__ dO, const float* __restrict__ LSE, const float* __restrict__ DELTA,
    uint16_t* __restrict__ dK, uint16_t* __restrict__ dV, int S, float scale, int onh) {
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  constexpr int TS = BN2 * LDP<D>;
  // [2 stages][Q | dO] tiles, [2 stages][-LSE/scale 64 | -Delta 64], P slots [2 halves][4 groups][2][64]
  float* const stats = reinterpret_cast<float*>(smem + 4 * TS);
  s16x8* const pslot = reinterpret_cast<s16x8*>(stats + 4 * BN2);
  const int lane = threadIdx.x & 63, ltid = threadIdx.x & 255;
  const int role = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 8);
  const int kg = __builtin_amdgcn_readfirstlane(((int)threadIdx.x >> 6) & 3);
  const int h = lane >> 5, c32 = lane & 31;
  const int g16 = lane >> 4, qd = (lane & 15) >> 2, pc = lane & 3;
  const int nkb = (S + BM2 - 1) / BM2;
  const int task = xcd_task(blockIdx.x, gridDim.x);
  const int64_t bh = task / nkb;
  const int kb = (task - (int)bh * nkb) * BM2;
  const int mykey = kb + 32 * kg + c32;
  const int64_t base = bh * (int64_t)S * D;
  const float sl2 = scale * LOG2E;
  // each role stages its own A-row tile (role 0: Q, role 1: dO) and reads the other one transposed
  const int sld = role ? o_ld<D>(onh) : D;
  const __amdgpu_buffer_rsrc_t rs = head_rsrc(role ? dO + o_base<D>(bh, S, onh) : Q + base, S, sld);
  const float* const rowc = (role ? DELTA : LSE) + bh * (int64_t)S;
  const float cmul = role ? -1.f : -1.f / scale;

  s16x8 bfr[D / 16];  // B fragments of this lane's key: K (role 0) or V (role 1)
  {
    const uint16_t* brow = (role ? V : K) + base + (int64_t)mykey * D + 8 * h;
#pragma unroll
    for (int ks = 0; ks < D / 16; ++ks)
      bfr[ks] = mykey < S ? *reinterpret_cast<const s16x8*>(brow + 16 * ks) : s16x8{};
  }
  f32x16 acc[D / 32];
#pragma unroll
  for (int dt = 0; dt < D / 32; ++dt)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[dt][r] = 0.f;

  const int qstart = CAUSAL ? kb : 0;
  const int ntiles = (S - qstart + BN2 - 1) / BN2;
  uint4 stg[D / 32];
  float st = 0.f;
  auto fetch = [&](int i0) {
    tile_load_buf_t<D>(stg, rs, i0, sld, ltid);
    if (ltid < BN2) {
      const int q = i0 + ltid;
      st = q < S ? rowc[q] * cmul : 0.f;
    }
  };
  auto put = [&](int stage) {
    tile_store_t<D>(smem + stage * 2 * TS + role * TS, stg, ltid);
    if (ltid < BN2) stats[stage * 2 * BN2 + role * BN2 + ltid] = st;
  };
  // S (role 0) or dP (role 1) of one 32-query half, started at the row constants
  auto scores = [&](const uint16_t* X, const float* cs, int t) {
    f32x16 c;
#pragma unroll
    for (int rb = 0; rb < 4; ++rb) {
      const float4 v4 = *reinterpret_cast<const float4*>(cs + 32 * t + 8 * rb + 4 * h);
      c[4 * rb + 0] = v4.x; c[4 * rb + 1] = v4.y; c[4 * rb + 2] = v4.z; c[4 * rb + 3] = v4.w;
    }
#pragma unroll
    for (int ks = 0; ks < D / 16; ++ks)
      c = Mfma32<T>::run(lds_row8(X + (32 * t + c32) * LDP<D> + 16 * ks + 8 * h), bfr[ks], c);
    return c;
  };
  // acc^T += Y^T F for one half: Y^T fragments by transposed reads of the other role's tile
  auto accum = [&](const uint16_t* Y, int t, const s16x8 (&f)[2]) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int row1 = 16 * (2 * t + kk) + 4 * (g16 >> 1) + qd;
#pragma unroll
      for (int dt = 0; dt < D / 32; ++dt) {
        const int col = 32 * dt + 16 * (g16 & 1) + 4 * pc;
        const s16x4 x = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(Y + row1 * LDP<D> + col));
        const s16x4 y = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(Y + (row1 + 8) * LDP<D> + col));
        acc[dt] = Mfma32<T>::run(s16x8{x[0], x[1], x[2], x[3], y[0], y[1], y[2], y[3]}, f[kk], acc[dt]);
      }
      __builtin_amdgcn_sched_barrier(0);  // bounds the tr-read hoisting
    }
  };
  // role 0: P of one half (masked), packed as B fragments and published in slot t
  auto probs = [&](const f32x16& s, int i0, int t, s16x8 (&pf)[2]) {
    float pv[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) pv[r] = fast_exp2(s[r] * sl2);
    if ((i0 + 32 * t + 32 > S) || (kb + 32 * kg + 32 > S) || (CAUSAL && kb + 32 * kg + 31 > i0 + 32 * t)) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int q = i0 + 32 * t + 8 * (r >> 2) + 4 * h + (r & 3);
        if (q >= S || mykey >= S || (CAUSAL && mykey > q)) pv[r] = 0.f;
      }
    }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      pf[kk] = __is_same(T, bf16_t) ? pack8(pv, 8 * kk) : pack8_h(pv, 8 * kk);
      pslot[((t * 4 + kg) * 2 + kk) * 64 + lane] = pf[kk];
    }
  };
  // role 1: dS = P * (dP - Delta) of one half from the published P
  auto dsfrag = [&](const f32x16& dp, int t, s16x8 (&sf)[2]) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const s16x8 p = pslot[((t * 4 + kg) * 2 + kk) * 64 + lane];
      float ds[8];
#pragma unroll
      for (int j = 0; j < 8; ++j)
        ds[j] = (__is_same(T, bf16_t) ? bf16_to_f32((uint16_t)p[j]) : f16_to_f32((uint16_t)p[j])) * dp[8 * kk + j];
      sf[kk] = __is_same(T, bf16_t) ? pack8(ds, 0) : pack8_h(ds, 0);
    }
  };

  fetch(qstart);
  put(0);
  __syncthreads();
  // the half pending across a barrier, in ONE register block for both roles (the compiler cannot
  // tell the role branches apart, so separate variables would all be live at the barriers):
  // role 0 keeps its P fragments there (bit-cast into the first 8 elements), role 1 its dP
  f32x16 hold1;
  for (int it = 0; it < ntiles; ++it) {
    const int i0 = qstart + it * BN2;
    const bool has_next = it + 1 < ntiles;
    const int cur = it & 1;
    const uint16_t* const X = smem + cur * 2 * TS + role * TS;        // own tile, row reads
    const uint16_t* const Y = smem + cur * 2 * TS + (1 - role) * TS;  // other tile, transposed reads
    const uint16_t* const Yp = smem + (cur ^ 1) * 2 * TS + (1 - role) * TS;
    const float* const cs = stats + cur * 2 * BN2 + role * BN2;
    if (has_next) fetch(i0 + BN2);
    f32x16 hold0;
    if (role == 0) {
      if (it > 0) {
        s16x8 f[2];
        unhold(hold1, f);
        accum(Yp, 1, f);
      }
      s16x8 f[2];
      probs(scores(X, cs, 0), i0, 0, f);
      tohold(hold0, f);
    } else {
      if (it > 0) {
        s16x8 sf[2];
        dsfrag(hold1, 1, sf);
        accum(Yp, 1, sf);
      }
      hold0 = scores(X, cs, 0);
    }
    __syncthreads();
    if (role == 0) {
      s16x8 f[2];
      unhold(hold0, f);
      accum(Y, 0, f);
      probs(scores(X, cs, 1), i0, 1, f);
      tohold(hold1, f);
    } else {
      s16x8 sf[2];
      dsfrag(hold0, 0, sf);
      accum(Y, 0, sf);
      hold1 = scores(X, cs, 1);
    }
    if (has_next) put(cur ^ 1);
    __syncthreads();
  }
  {
    const uint16_t* const Yl = smem + ((ntiles - 1) & 1) * 2 * TS + (1 - role) * TS;
    s16x8 f[2];
    if (role == 0) unhold(hold1, f);
    else dsfrag(hold1, 1, f);
    accum(Yl, 1, f);
  }
  if (mykey < S) {
    uint16_t* const out = (role ? dK : dV) + base + (int64_t)mykey * D;
    const float m = role ? scale : 1.f;
#pragma unroll
    for (int dt = 0; dt < D / 32; ++dt)
#pragma unroll
      for (int rb = 0; rb < 4; ++rb) {
        ushort4 v4;
        v4.x = to16<T>(acc[dt][4 * rb + 0] * m); v4.y = to16<T>(acc[dt][4 * rb + 1] * m);
        v4.z = to16<T>(acc[dt][4 * rb + 2] * m); v4.w = to16<T>(acc[dt][4 * rb + 3] * m);
        *reinterpret_cast<ushort4*>(out + 32 * dt + 8 * rb + 4 * h) = v4;
      }
  }
}

template <typename T, int D, bool CAUSAL, int EX = 0, bool BUF = true>
__global__ void __launch_bounds__(256, 2) bwd_dq_v2_kernel(
    const uint16_t* __restrict__ Q, const uint16_t* __restrict__ K, const uint16_t* __restrict__ V,
    const uint16_t* __restrict__ dO, const float* __restrict__ LSE, const float* __restrict__ DELTA,
    uint16_t* __restrict__ dQ, int S, float scale, int onh, Extra ex = Extra()) {
  dq_v2_body<T, D, CAUSAL, EX, BUF>(blockIdx.x, gridDim.x, Q, K, V, dO, LSE, DELTA, dQ, S, scale, onh, ex);
}

template <int D> constexpr int dkdv_v2_lds() { return 2 * 2 * BN2 * LDP<D> * 2 + 2 * 2 * BN2 * 4; }
// + K [BM2][D+8] and one tile's dS [BN2][BM2+8] for the fused short-sequence backward
template <int D> constexpr int bwd_short_lds() { return dkdv_v2_lds<D>() + BM2 * LDP<D> * 2 + BN2 * (BM2 + 8) * 2 + BM2 * 4; }

// Whole backward of one head in one workgroup for S <= BM2 (= 128, BERT's sequence): dK / dV
// as in the dK/dV kernel, and dQ from the same dS tiles through LDS -- Q, K, V and dO are read
// once instead of twice, and the separate dQ launch disappears.
template <typename T, int D, int EX = 0>
__global__ void __launch_bounds__(256, (D >= 128 ? 1 : 2)) bwd_short_kernel(
    const uint16_t* __restrict__ Q, const uint16_t* __restrict__ K, const uint16_t* __restrict__ V,
    const uint16_t* __restrict__ dO, const float* __restrict__ LSE, const float* __restrict__ DELTA,
    uint16_t* __restrict__ dQ, uint16_t* __restrict__ dK, uint16_t* __restrict__ dV, int S, float scale, int onh,
    Extra ex = Extra(), const uint16_t* __restrict__ O = nullptr) {
  dkdv_v2_body<T, D, false, EX, true>(blockIdx.x, gridDim.x, Q, K, V, dO, LSE, DELTA, dK, dV, S, scale, onh, ex, dQ, O);
}

template <int D> constexpr int fwd_v2_lds() { return 2 * 2 * BN2 * LDP<D> * 2; }


// ======================================================================== block-sparse (LUT-driven)
// Flash attention restricted to the active blocks of a block-sparse layout (reference:
// deepspeed/ops/sparse_attention matmul.py SDD/DSD + softmax.py, fused here into one pass per
// query tile so the sparse score matrix is never written).  Granularity: 64-query x 64-key
// MFMA tiles, 2 waves (32 queries or keys each) per workgroup, whose 64 keys (forward / dQ) or
// 64 queries (dK / dV) are GATHERED from four 16-row blocks named by the LUT entry, so the work
// follows the layout's active 16-blocks instead of the 64-tiles they touch
// (ops/sparse_attention/flash.py builds the walks).  Per layout head:
//   fwd / dQ LUT : rowptr[nqt + 1]; cols[e] = int4 key 16-blocks; masks[e] bit (qsub * 4 + kslot)
//   dK / dV LUT  : tasks (key group, entry range, slot); kgroups[g] = int4 key 16-blocks of the
//                  group (the output rows); rows[e] = int4 query 16-blocks; masks_t[e] bit
//                  (qslot * 4 + kslot)
// Block lists are ascending (padding repeats the last block with its mask bits clear); only
// tiles whose mask is not full, or that reach past the causal diagonal, are masked element-wise.
// S must be a multiple of 64.  Causal masking (GPT) is applied on top of the layout.
constexpr int STILE = 64;

// g is one head's base (wave-uniform): the tile loads go through a buffer resource sized to the
// head's S rows (32-bit lane offsets, rows past S read 0 in hardware; see tile_load_buf)
template <int D, int NT>
__device__ __forceinline__ void stile_load(uint4 (&r)[8 * D / NT], const uint16_t* __restrict__ g, int r0, int S,
                                           int ld = D) {
  constexpr int CH = D / 8;
  const __amdgpu_buffer_rsrc_t rs = head_rsrc(g, S, ld);
#pragma unroll
  for (int k = 0; k < 8 * D / NT; ++k) {
    const int c = threadIdx.x + NT * k;
    const int row = c / CH, ch = c - row * CH;
    const fa_u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, ((r0 + row) * ld + ch * 8) * 2, 0, 0);
    r[k] = make_uint4(v.x, v.y, v.z, v.w);
  }
}

template <int D, int NT>
__device__ __forceinline__ void stile_store(uint16_t* lds, const uint4 (&r)[8 * D / NT]) {
  constexpr int CH = D / 8;
#pragma unroll
  for (int k = 0; k < 8 * D / NT; ++k) {
    const int c = threadIdx.x + NT * k;
    const int row = c / CH, ch = c - row * CH;
    *reinterpret_cast<uint4*>(lds + row * LDP<D> + ch * 8) = r[k];
  }
}

// One of the four gathered 16-row blocks of a tile (i is compile-time in every caller but the
// D = 96 tile loads, where it is a 3-deep select)
__device__ __forceinline__ int sel4(const int4& b, int i) {
  return i == 0 ? b.x : (i == 1 ? b.y : (i == 2 ? b.z : b.w));
}

// stile_load over a gathered tile: tile row `row` is row (row & 15) of 16-row block blk[row >> 4]
template <int D, int NT>
__device__ __forceinline__ void gtile_load(uint4 (&r)[8 * D / NT], const uint16_t* __restrict__ g, const int4 blk,
                                           int S, int ld = D) {
  constexpr int CH = D / 8;
  const __amdgpu_buffer_rsrc_t rs = head_rsrc(g, S, ld);
  if (blk.y == blk.x + 1 && blk.z == blk.x + 2 && blk.w == blk.x + 3) {  // one contiguous 64-row tile
    const int r0 = blk.x * 16;
#pragma unroll
    for (int k = 0; k < 8 * D / NT; ++k) {
      const int c = threadIdx.x + NT * k;
      const int row = c / CH, ch = c - row * CH;
      const fa_u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, ((r0 + row) * ld + ch * 8) * 2, 0, 0);
      r[k] = make_uint4(v.x, v.y, v.z, v.w);
    }
    return;
  }
#pragma unroll
  for (int k = 0; k < 8 * D / NT; ++k) {
    const int c = threadIdx.x + NT * k;
    const int row = c / CH, ch = c - row * CH;
    const int grow = sel4(blk, row >> 4) * 16 + (row & 15);
    const fa_u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, (grow * ld + ch * 8) * 2, 0, 0);
    r[k] = make_uint4(v.x, v.y, v.z, v.w);
  }
}

constexpr uint32_t GFULL = 0xffffu;  // all 4 x 4 (query 16-block, key 16-block) pairs of a tile active

// Score biases of the reference sparse softmax (softmax_fwd.tr:46-129), compiled in by SX bits
// (1: key-padding bias only -- BERT's case, no per-element loads; 3: both):
//   kbias [Z, S] fp32: the key-padding mask (additive; 'mul' masks arrive as 0 / -inf), z = bh / H
//   ebias [Z|1, H|1, S, S] in the input dtype: relative position embedding + attention mask
//         (additive, pre-summed on the host), element (bh, q, k) at (bh / H) * ez + (bh % H) * eh
//         + q * er + k (ez / eh = 0 broadcast)
// either pointer may be null.  Scores enter the softmax as s * scale + kbias + ebias.
struct SExtra {
  const float* kbias = nullptr;
  const uint16_t* ebias = nullptr;
  int64_t ez = 0, eh = 0, er = 0;
};
template <typename T> __device__ __forceinline__ float h16f(uint16_t v);
template <> __device__ __forceinline__ float h16f<bf16_t>(uint16_t v) { return bf16_to_f32(v); }
template <> __device__ __forceinline__ float h16f<f16_t>(uint16_t v) { return f16_to_f32(v); }
__device__ __forceinline__ const uint16_t* ebias_head(const SExtra& sx, int64_t bh, int H) {
  return sx.ebias + (bh / H) * sx.ez + (bh % H) * sx.eh;
}
// log2-domain bias of 4 consecutive keys key0..key0+3 of query row `q` (fwd / dQ layouts)
template <typename T, int SX>
__device__ __forceinline__ float4 sbias4(const SExtra& sx, const uint16_t* eh, int64_t z, int S, int q, int key0) {
  float4 b = make_float4(0.f, 0.f, 0.f, 0.f);
  if constexpr (SX != 0) {
    if ((SX & 1) && sx.kbias) b = *reinterpret_cast<const float4*>(sx.kbias + z * S + key0);
    if ((SX & 2) && sx.ebias) {
      const ushort4 e = *reinterpret_cast<const ushort4*>(eh + (int64_t)q * sx.er + key0);
      b.x += h16f<T>(e.x); b.y += h16f<T>(e.y); b.z += h16f<T>(e.z); b.w += h16f<T>(e.w);
    }
    b.x *= LOG2E; b.y *= LOG2E; b.z *= LOG2E; b.w *= LOG2E;
  }
  return b;
}

template <typename T, int D, bool CAUSAL, bool RP, int SX = 0>
__global__ void __launch_bounds__(128, RP ? ((SX == 3 || (SX && D >= 128)) ? 1 : 2) : 3) sfwd_kernel(const uint16_t* __restrict__ Q, const uint16_t* __restrict__ K,
                                                      const uint16_t* __restrict__ V, uint16_t* __restrict__ O,
                                                      float* __restrict__ LSE, const int* __restrict__ rowptr,
                                                      const int4* __restrict__ cols, const uint32_t* __restrict__ masks,
                                                      int S, float scale, int onh, int H, int Hl, int shift,
                                                      SExtra sx = SExtra()) {
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  constexpr int TS = STILE * LDP<D>;
  constexpr int NT = 128;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int h = lane >> 5, c32 = lane & 31;
  const int g16 = lane >> 4, qd = (lane & 15) >> 2, pc = lane & 3;
  const int nqt = S / STILE;
  const int task = xcd_task(blockIdx.x, gridDim.x);
  const int64_t bh = task / nqt;
  const int qt = task - (int)bh * nqt;
  const int lh = Hl == 1 ? 0 : (int)(bh % H);
  const int e0 = rowptr[lh * nqt + qt], e1 = rowptr[lh * nqt + qt + 1];
  const int qrow = 32 * w + c32;  // row inside the tile
  const int myq = qt * STILE + qrow;
  const int qsub = qrow >> 4;
  const uint16_t* Qb = Q + bh * (int64_t)S * D;
  const uint16_t* Kb = K + bh * (int64_t)S * D;
  const uint16_t* Vb = V + bh * (int64_t)S * D;

  s16x8 qf[D / 16];
#pragma unroll
  for (int ks = 0; ks < D / 16; ++ks) qf[ks] = *reinterpret_cast<const s16x8*>(Qb + (int64_t)myq * D + 16 * ks + 8 * h);
  f32x16 o[D / 32];
#pragma unroll
  for (int dt = 0; dt < D / 32; ++dt)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[dt][r] = 0.f;
  float m = -INFINITY, l = 0.f;
  const float sl2 = scale * 1.4426950408889634f;

  uint4 kr[8 * D / NT], vr[8 * D / NT];
  if (RP && e0 < e1) {
    gtile_load<D, NT>(kr, Kb, cols[e0], S);
    gtile_load<D, NT>(vr, Vb, cols[e0], S);
    stile_store<D, NT>(smem, kr);
    stile_store<D, NT>(smem + TS, vr);
  }
  __syncthreads();
  for (int e = e0; e < e1; ++e) {
    const int it = e - e0;
    const int4 kb = cols[e];
    const uint32_t mask = masks[e];
    const bool has_next = e + 1 < e1;
    if (RP && has_next) {
      gtile_load<D, NT>(kr, Kb, cols[e + 1], S);
      gtile_load<D, NT>(vr, Vb, cols[e + 1], S);
    }
    if (!RP) {  // single LDS stage: more workgroups per CU hide the load instead
      gtile_load<D, NT>(kr, Kb, kb, S);
      gtile_load<D, NT>(vr, Vb, kb, S);
      if (it > 0) __syncthreads();
      stile_store<D, NT>(smem, kr);
      stile_store<D, NT>(smem + TS, vr);
      __syncthreads();
    }
    const uint16_t* Ks = smem + (RP ? (it & 1) * 2 * TS : 0);
    const uint16_t* Vs = Ks + TS;
    float sv[32];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      f32x16 acc;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
      for (int ks = 0; ks < D / 16; ++ks)
        acc = Mfma32<T>::run(lds_row8(Ks + (32 * t + c32) * LDP<D> + 16 * ks + 8 * h), qf[ks], acc);
#pragma unroll
      for (int r = 0; r < 16; ++r) sv[16 * t + r] = acc[r];
    }
    // wave-uniform: a partially active tile, or keys past this wave's first query
    if (mask != GFULL || (CAUSAL && kb.w * 16 + 15 > qt * STILE + 32 * w)) {
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int slot = 2 * t + (r >> 3);  // gathered key block of tile column 32t + 8(r>>2) + 4h + (r&3)
          const int key = sel4(kb, slot) * 16 + 8 * ((r >> 2) & 1) + 4 * h + (r & 3);
          if (!((mask >> ((qsub << 2) + slot)) & 1u) || (CAUSAL && key > myq)) sv[16 * t + r] = -INFINITY;
        }
    }
    if constexpr (SX != 0) {  // scores to the log2 domain with the biases folded in
      const uint16_t* ehd = ((SX & 2) && sx.ebias) ? ebias_head(sx, bh, H) : nullptr;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int rb = 0; rb < 4; ++rb) {
          const int key0 = sel4(kb, 2 * t + (rb >> 1)) * 16 + 8 * (rb & 1) + 4 * h;
          const float4 b4 = sbias4<T, SX>(sx, ehd, bh / H, S, myq, key0);
          float* s4 = sv + 16 * t + 4 * rb;
          s4[0] = fmaf(s4[0], sl2, b4.x); s4[1] = fmaf(s4[1], sl2, b4.y);
          s4[2] = fmaf(s4[2], sl2, b4.z); s4[3] = fmaf(s4[3], sl2, b4.w);
        }
    }
    const float a2 = SX != 0 ? 1.f : sl2;
    float mx = -INFINITY;
#pragma unroll
    for (int i = 0; i < 32; ++i) mx = fmaxf(mx, sv[i]);
    mx = xhalf_max(mx);
    const float mt = mx * a2;
    if (__any(mt > m + LAZY_TH)) {
      const float mn = fmaxf(m, mt);
      const float alpha = fast_exp2(m - ((mn == -INFINITY) ? 0.f : mn));
      l *= alpha;
      m = mn;
#pragma unroll
      for (int dt = 0; dt < D / 32; ++dt)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[dt][r] *= alpha;
    }
    const float mu = (m == -INFINITY) ? 0.f : m;
    float ps = 0.f, ps1 = 0.f;
#pragma unroll
    for (int i = 0; i < 32; i += 2) {
      sv[i] = fast_exp2(fmaf(sv[i], a2, -mu));
      sv[i + 1] = fast_exp2(fmaf(sv[i + 1], a2, -mu));
      ps += sv[i];
      ps1 += sv[i + 1];
    }
    ps += ps1;
    ps = xhalf_sum(ps);
    l += ps;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const s16x8 pf = __is_same(T, bf16_t) ? pack8(sv, 8 * ks) : pack8_h(sv, 8 * ks);
      const int row1 = 16 * ks + 4 * (g16 >> 1) + qd;
#pragma unroll
      for (int dt = 0; dt < D / 32; ++dt) {
        const uint16_t* a0 = Vs + row1 * LDP<D> + 32 * dt + 16 * (g16 & 1) + 4 * pc;
        const s16x4 x = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0));
        const s16x4 y = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0 + 8 * LDP<D>));
        o[dt] = Mfma32<T>::run(s16x8{x[0], x[1], x[2], x[3], y[0], y[1], y[2], y[3]}, pf, o[dt]);
      }
    }
    if (RP) {
      if (has_next) {
        uint16_t* nxt = smem + ((it + 1) & 1) * 2 * TS;
        stile_store<D, NT>(nxt, kr);
        stile_store<D, NT>(nxt + TS, vr);
      }
      __syncthreads();
    }
  }
  const float inv = l > 0.f ? 1.f / l : 0.f;
  uint16_t* orow = O + o_base<D>(bh, S, onh) + (int64_t)myq * o_ld<D>(onh);
#pragma unroll
  for (int dt = 0; dt < D / 32; ++dt)
#pragma unroll
    for (int rb = 0; rb < 4; ++rb) {
      ushort4 v4;
      v4.x = to16<T>(o[dt][4 * rb + 0] * inv);
      v4.y = to16<T>(o[dt][4 * rb + 1] * inv);
      v4.z = to16<T>(o[dt][4 * rb + 2] * inv);
      v4.w = to16<T>(o[dt][4 * rb + 3] * inv);
      *reinterpret_cast<ushort4*>(orow + 32 * dt + 8 * rb + 4 * h) = v4;
    }
  // a row with no unmasked key stores +inf: the backward then recomputes P = 0 for it
  if (h == 0) LSE[bh * (int64_t)S + myq] = (l > 0.f) ? (m + log2f(l)) * 0.6931471805599453f : INFINITY;
}

// dK / dV over the query tiles listed for this key tile (transposed LUT)
// Row constants enter as the MFMAs' initial accumulators (S at -LSE / scale, dP at -Delta,
// stored negated in LDS and read as one float4 per 4 C-layout rows), as in dkdv_v2_body V3.
template <typename T, int D, bool CAUSAL, bool RP, int SX = 0>
__global__ void __launch_bounds__(128, RP ? 1 : 3) sdkdv_kernel(const uint16_t* __restrict__ Q, const uint16_t* __restrict__ K,
                                                       const uint16_t* __restrict__ V, const uint16_t* __restrict__ dO,
                                                       const float* __restrict__ LSE, const float* __restrict__ DELTA,
                                                       uint16_t* __restrict__ dK, uint16_t* __restrict__ dV,
                                                       const int4* __restrict__ rows,
                                                       const uint32_t* __restrict__ masks,
                                                       const int4* __restrict__ tasks, int ntask,
                                                       const int4* __restrict__ kgroups,
                                                       float* __restrict__ ws, int nslot, int S, float scale, int onh,
                                                       int H, int Hl, int shift, SExtra sx = SExtra()) {
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  constexpr int TS = STILE * LDP<D>;
  constexpr int NT = 128;
  float* stats = reinterpret_cast<float*>(smem + (RP ? 4 : 2) * TS);  // [stages][LSE 64 | DELTA 64]
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int h = lane >> 5, c32 = lane & 31;
  const int g16 = lane >> 4, qd = (lane & 15) >> 2, pc = lane & 3;
  // task = (key group, entry range of its query list, partial slot or -1): groups whose list is
  // long (the global columns of BigBird / Longformer / fixed layouts) are split into chunks
  // that write fp32 partials, summed by sdkdv_finish_kernel -- no single workgroup walks them all
  const int task = xcd_task(blockIdx.x, gridDim.x);
  const int64_t bh = task / ntask;
  const int lh = Hl == 1 ? 0 : (int)(bh % H);
  const int4 tk = tasks[lh * ntask + (task - (int)bh * ntask)];
  const int kg = tk.x, e0 = tk.y, e1 = tk.z, slot = tk.w;
  if (kg < 0) return;  // padding task (whole workgroup, before any barrier)
  const int4 kblk = kgroups[lh * (S / STILE) + kg];  // this group's four key 16-blocks (ascending)
  const int kcol = 32 * w + c32;
  const int ksub = kcol >> 4;
  const int mykey = sel4(kblk, ksub) * 16 + (kcol & 15);
  const int wmaxkey = sel4(kblk, 2 * w + 1) * 16 + 15;  // this wave's last key
  const int64_t base = bh * (int64_t)S * D;
  const int64_t obase = o_base<D>(bh, S, onh);
  const float sl2 = scale * 1.4426950408889634f;

  s16x8 kf[D / 16], vf[D / 16];
#pragma unroll
  for (int ks = 0; ks < D / 16; ++ks) {
    kf[ks] = *reinterpret_cast<const s16x8*>(K + base + (int64_t)mykey * D + 16 * ks + 8 * h);
    vf[ks] = *reinterpret_cast<const s16x8*>(V + base + (int64_t)mykey * D + 16 * ks + 8 * h);
  }
  f32x16 dk[D / 32], dv[D / 32];
#pragma unroll
  for (int dt = 0; dt < D / 32; ++dt)
#pragma unroll
    for (int r = 0; r < 16; ++r) { dk[dt][r] = 0.f; dv[dt][r] = 0.f; }

  uint4 qr[8 * D / NT], orr[8 * D / NT];
  float st_l = 0.f, st_d = 0.f;
  auto load_tile = [&](const int4 qb) {
    gtile_load<D, NT>(qr, Q + base, qb, S);
    gtile_load<D, NT>(orr, dO + obase, qb, S, o_ld<D>(onh));
    if (threadIdx.x < STILE) {
      const int qp = sel4(qb, threadIdx.x >> 4) * 16 + (threadIdx.x & 15);
      st_l = LSE[bh * (int64_t)S + qp] * (-1.f / scale);
      st_d = -DELTA[bh * (int64_t)S + qp];
    }
  };
  // this lane's key: key-padding bias (log2 units) and its column of the element bias
  float kb2 = 0.f;
  const uint16_t* ecol = nullptr;
  if constexpr (SX != 0) {
    if (sx.kbias) kb2 = sx.kbias[(bh / H) * (int64_t)S + mykey] * LOG2E;
    if ((SX & 2) && sx.ebias) ecol = ebias_head(sx, bh, H) + mykey;
  }
  auto store_tile = [&](int stage) {
    uint16_t* b = smem + stage * 2 * TS;
    stile_store<D, NT>(b, qr);
    stile_store<D, NT>(b + TS, orr);
    if (threadIdx.x < STILE) {
      stats[stage * 2 * STILE + threadIdx.x] = st_l;
      stats[stage * 2 * STILE + STILE + threadIdx.x] = st_d;
    }
  };
  if (RP && e0 < e1) {
    load_tile(rows[e0]);
    store_tile(0);
  }
  __syncthreads();
  for (int e = e0; e < e1; ++e) {
    const int it = e - e0;
    const int4 qb = rows[e];
    const uint32_t mask = masks[e];
    const bool has_next = e + 1 < e1;
    if (RP && has_next) load_tile(rows[e + 1]);
    if (!RP) {
      load_tile(qb);
      if (it > 0) __syncthreads();
      store_tile(0);
      __syncthreads();
    }
    const uint16_t* Qs = smem + (RP ? (it & 1) * 2 * TS : 0);
    const uint16_t* Os = Qs + TS;
    const float* lse_s = stats + (RP ? (it & 1) * 2 * STILE : 0);
    const float* del_s = lse_s + STILE;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      f32x16 sacc, pacc;
#pragma unroll
      for (int rb = 0; rb < 4; ++rb) {
        const float4 l4 = *reinterpret_cast<const float4*>(lse_s + 32 * t + 8 * rb + 4 * h);
        const float4 d4 = *reinterpret_cast<const float4*>(del_s + 32 * t + 8 * rb + 4 * h);
        sacc[4 * rb + 0] = l4.x; sacc[4 * rb + 1] = l4.y; sacc[4 * rb + 2] = l4.z; sacc[4 * rb + 3] = l4.w;
        pacc[4 * rb + 0] = d4.x; pacc[4 * rb + 1] = d4.y; pacc[4 * rb + 2] = d4.z; pacc[4 * rb + 3] = d4.w;
      }
#pragma unroll
      for (int ks = 0; ks < D / 16; ++ks) {
        sacc = Mfma32<T>::run(lds_row8(Qs + (32 * t + c32) * LDP<D> + 16 * ks + 8 * h), kf[ks], sacc);
        pacc = Mfma32<T>::run(lds_row8(Os + (32 * t + c32) * LDP<D> + 16 * ks + 8 * h), vf[ks], pacc);
      }
      float pv[16], dsv[16];
      if constexpr (SX != 0) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          float b = kb2;
          if ((SX & 2) && ecol)
            b += h16f<T>(ecol[(int64_t)(sel4(qb, 2 * t + (r >> 3)) * 16 + 8 * ((r >> 2) & 1) + 4 * h + (r & 3)) *
                              sx.er]) * LOG2E;
          pv[r] = fast_exp2(fmaf(sacc[r], sl2, b));
        }
      } else {
#pragma unroll
        for (int r = 0; r < 16; ++r) pv[r] = fast_exp2(sacc[r] * sl2);
      }
      if (mask != GFULL || (CAUSAL && wmaxkey > sel4(qb, 2 * t) * 16)) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int qslot = 2 * t + (r >> 3);
          const int qpos = sel4(qb, qslot) * 16 + 8 * ((r >> 2) & 1) + 4 * h + (r & 3);
          if (!((mask >> ((qslot << 2) + ksub)) & 1u) || (CAUSAL && mykey > qpos)) pv[r] = 0.f;
        }
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) dsv[r] = pv[r] * pacc[r];
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int ks = 2 * t + kk;
        const s16x8 pf = __is_same(T, bf16_t) ? pack8(pv, 8 * kk) : pack8_h(pv, 8 * kk);
        const s16x8 sf = __is_same(T, bf16_t) ? pack8(dsv, 8 * kk) : pack8_h(dsv, 8 * kk);
        const int row1 = 16 * ks + 4 * (g16 >> 1) + qd;
#pragma unroll
        for (int dt = 0; dt < D / 32; ++dt) {
          const int col = 32 * dt + 16 * (g16 & 1) + 4 * pc;
          const s16x4 ox = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(Os + row1 * LDP<D> + col));
          const s16x4 oy = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(Os + (row1 + 8) * LDP<D> + col));
          dv[dt] = Mfma32<T>::run(s16x8{ox[0], ox[1], ox[2], ox[3], oy[0], oy[1], oy[2], oy[3]}, pf, dv[dt]);
          const s16x4 qx = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(Qs + row1 * LDP<D> + col));
          const s16x4 qy = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(Qs + (row1 + 8) * LDP<D> + col));
          dk[dt] = Mfma32<T>::run(s16x8{qx[0], qx[1], qx[2], qx[3], qy[0], qy[1], qy[2], qy[3]}, sf, dk[dt]);
        }
      }
    }
    if (RP) {
      if (has_next) store_tile((it + 1) & 1);
      __syncthreads();
    }
  }
  if (slot >= 0) {  // partial of a split key tile: fp32 [bh][slot][dK | dV][64][D]
    float* pk = ws + ((bh * nslot + slot) * 2 * STILE + kcol) * (int64_t)D;
    float* pv = pk + STILE * D;
#pragma unroll
    for (int dt = 0; dt < D / 32; ++dt)
#pragma unroll
      for (int rb = 0; rb < 4; ++rb) {
        const int c = 32 * dt + 8 * rb + 4 * h;
        *reinterpret_cast<float4*>(pk + c) = make_float4(dk[dt][4 * rb], dk[dt][4 * rb + 1], dk[dt][4 * rb + 2],
                                                         dk[dt][4 * rb + 3]);
        *reinterpret_cast<float4*>(pv + c) = make_float4(dv[dt][4 * rb], dv[dt][4 * rb + 1], dv[dt][4 * rb + 2],
                                                         dv[dt][4 * rb + 3]);
      }
    return;
  }
  uint16_t* dkr = dK + base + (int64_t)mykey * D;
  uint16_t* dvr = dV + base + (int64_t)mykey * D;
#pragma unroll
  for (int dt = 0; dt < D / 32; ++dt)
#pragma unroll
    for (int rb = 0; rb < 4; ++rb) {
      ushort4 a4, b4;
      a4.x = to16<T>(dk[dt][4 * rb + 0] * scale); a4.y = to16<T>(dk[dt][4 * rb + 1] * scale);
      a4.z = to16<T>(dk[dt][4 * rb + 2] * scale); a4.w = to16<T>(dk[dt][4 * rb + 3] * scale);
      b4.x = to16<T>(dv[dt][4 * rb + 0]); b4.y = to16<T>(dv[dt][4 * rb + 1]);
      b4.z = to16<T>(dv[dt][4 * rb + 2]); b4.w = to16<T>(dv[dt][4 * rb + 3]);
      *reinterpret_cast<ushort4*>(dkr + 32 * dt + 8 * rb + 4 * h) = a4;
      *reinterpret_cast<ushort4*>(dvr + 32 * dt + 8 * rb + 4 * h) = b4;
    }
}

// Sum the fp32 partials of each split key tile and write its bf16/fp16 dK (scaled) and dV.
// fin[lh][j] = (key group, first slot, chunk count, -), padded with key group -1.
// One workgroup per 256 float4 granules of one split key tile (SDKDV_FPARTS per tile): the
// partial sums spread over the whole chip instead of one workgroup per tile.
template <int D> constexpr int sdkdv_fparts() { return (2 * STILE * D / 4 + 255) / 256; }
template <typename T, int D>
__global__ void __launch_bounds__(256) sdkdv_finish_kernel(const float* __restrict__ ws, const int4* __restrict__ fin,
                                                           int nfin, int nslot, uint16_t* __restrict__ dK,
                                                           uint16_t* __restrict__ dV, int S, float scale, int H,
                                                           int Hl, const int4* __restrict__ kgroups) {
  constexpr int NP = sdkdv_fparts<D>();
  const int part = blockIdx.x % NP;
  const int tile = blockIdx.x / NP;
  const int64_t bh = tile / nfin;
  const int lh = Hl == 1 ? 0 : (int)(bh % H);
  const int4 f = fin[lh * nfin + (tile - (int)bh * nfin)];
  if (f.x < 0) return;
  const int64_t base = bh * (int64_t)S * D;
  {
    const int i = part * 256 + threadIdx.x;  // float4 granule of dK | dV
    if (i >= 2 * STILE * D / 4) return;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int c = 0; c < f.z; ++c) {
      const float4 v = reinterpret_cast<const float4*>(ws + (bh * nslot + f.y + c) * 2 * STILE * (int64_t)D)[i];
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
    const int e = 4 * i;
    const bool is_k = e < STILE * D;
    const int off = is_k ? e : e - STILE * D;
    const float sc = is_k ? scale : 1.f;
    ushort4 o4;
    o4.x = to16<T>(acc.x * sc); o4.y = to16<T>(acc.y * sc); o4.z = to16<T>(acc.z * sc); o4.w = to16<T>(acc.w * sc);
    const int4 kb = kgroups[lh * (S / STILE) + f.x];
    const int row = off / D;
    uint16_t* dst = (is_k ? dK : dV) + base + (int64_t)(sel4(kb, row >> 4) * 16 + (row & 15)) * D + (off - row * D);
    *reinterpret_cast<ushort4*>(dst) = o4;
  }
}

// dQ over the key tiles listed for this query tile (forward LUT)
// FD: also forms Delta = rowsum(dO * O) for its rows and stores it (runs before sdkdv_kernel)
template <typename T, int D, bool CAUSAL, bool RP, int SX = 0, bool FD = false>
__global__ void __launch_bounds__(128, RP ? 1 : 3) sdq_kernel(const uint16_t* __restrict__ Q, const uint16_t* __restrict__ K,
                                                     const uint16_t* __restrict__ V, const uint16_t* __restrict__ dO,
                                                     const float* __restrict__ LSE, const float* __restrict__ DELTA,
                                                     uint16_t* __restrict__ dQ, const int* __restrict__ rowptr,
                                                     const int4* __restrict__ cols, const uint32_t* __restrict__ masks,
                                                     int S, float scale, int onh, int H, int Hl, int shift,
                                                     SExtra sx = SExtra(), const uint16_t* __restrict__ O = nullptr) {
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  constexpr int TS = STILE * LDP<D>;
  constexpr int NT = 128;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int h = lane >> 5, c32 = lane & 31;
  const int g16 = lane >> 4, qd = (lane & 15) >> 2, pc = lane & 3;
  const int nqt = S / STILE;
  const int task = xcd_task(blockIdx.x, gridDim.x);
  const int64_t bh = task / nqt;
  const int qt = task - (int)bh * nqt;
  const int lh = Hl == 1 ? 0 : (int)(bh % H);
  const int e0 = rowptr[lh * nqt + qt], e1 = rowptr[lh * nqt + qt + 1];
  const int qrow = 32 * w + c32;
  const int myq = qt * STILE + qrow;
  const int qsub = qrow >> 4;
  const int64_t base = bh * (int64_t)S * D;
  const float sl2 = scale * 1.4426950408889634f;

  s16x8 qf[D / 16], of[D / 16];
#pragma unroll
  for (int ks = 0; ks < D / 16; ++ks) {
    qf[ks] = *reinterpret_cast<const s16x8*>(Q + base + (int64_t)myq * D + 16 * ks + 8 * h);
    of[ks] = *reinterpret_cast<const s16x8*>(dO + o_base<D>(bh, S, onh) + (int64_t)myq * o_ld<D>(onh) + 16 * ks + 8 * h);
  }
  const float lse2 = LSE[bh * (int64_t)S + myq] * 1.4426950408889634f;
  float dl;
  if constexpr (FD) {
    float part = 0.f;
    const uint16_t* orow = O + o_base<D>(bh, S, onh) + (int64_t)myq * o_ld<D>(onh) + 8 * h;
#pragma unroll
    for (int ks = 0; ks < D / 16; ++ks) {
      float b[8];
      Vec16<T>::load(reinterpret_cast<const T*>(orow) + 16 * ks, b);
#pragma unroll
      for (int j = 0; j < 8; ++j) part = fmaf(h16f<T>((uint16_t)of[ks][j]), b[j], part);
    }
    dl = xhalf_sum(part);
    if (h == 0) const_cast<float*>(DELTA)[bh * (int64_t)S + myq] = dl;
  } else {
    dl = DELTA[bh * (int64_t)S + myq];
  }
  const uint16_t* ehd = ((SX & 2) && sx.ebias) ? ebias_head(sx, bh, H) : nullptr;
  f32x16 dq[D / 32];
#pragma unroll
  for (int dt = 0; dt < D / 32; ++dt)
#pragma unroll
    for (int r = 0; r < 16; ++r) dq[dt][r] = 0.f;

  uint4 kr[8 * D / NT], vr[8 * D / NT];
  if (RP && e0 < e1) {
    gtile_load<D, NT>(kr, K + base, cols[e0], S);
    gtile_load<D, NT>(vr, V + base, cols[e0], S);
    stile_store<D, NT>(smem, kr);
    stile_store<D, NT>(smem + TS, vr);
  }
  __syncthreads();
  for (int e = e0; e < e1; ++e) {
    const int it = e - e0;
    const int4 kb = cols[e];
    const uint32_t mask = masks[e];
    const bool has_next = e + 1 < e1;
    if (RP && has_next) {
      gtile_load<D, NT>(kr, K + base, cols[e + 1], S);
      gtile_load<D, NT>(vr, V + base, cols[e + 1], S);
    }
    if (!RP) {
      gtile_load<D, NT>(kr, K + base, kb, S);
      gtile_load<D, NT>(vr, V + base, kb, S);
      if (it > 0) __syncthreads();
      stile_store<D, NT>(smem, kr);
      stile_store<D, NT>(smem + TS, vr);
      __syncthreads();
    }
    const uint16_t* Ks = smem + (RP ? (it & 1) * 2 * TS : 0);
    const uint16_t* Vs = Ks + TS;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      f32x16 sacc, pacc;
#pragma unroll
      for (int r = 0; r < 16; ++r) { sacc[r] = 0.f; pacc[r] = 0.f; }
#pragma unroll
      for (int ks = 0; ks < D / 16; ++ks) {
        sacc = Mfma32<T>::run(lds_row8(Ks + (32 * t + c32) * LDP<D> + 16 * ks + 8 * h), qf[ks], sacc);
        pacc = Mfma32<T>::run(lds_row8(Vs + (32 * t + c32) * LDP<D> + 16 * ks + 8 * h), of[ks], pacc);
      }
      float dsv[16];
      if constexpr (SX != 0) {
#pragma unroll
        for (int rb = 0; rb < 4; ++rb) {
          const int key0 = sel4(kb, 2 * t + (rb >> 1)) * 16 + 8 * (rb & 1) + 4 * h;
          const float4 b4 = sbias4<T, SX>(sx, ehd, bh / H, S, myq, key0);
          dsv[4 * rb + 0] = fast_exp2(fmaf(sacc[4 * rb + 0], sl2, b4.x - lse2));
          dsv[4 * rb + 1] = fast_exp2(fmaf(sacc[4 * rb + 1], sl2, b4.y - lse2));
          dsv[4 * rb + 2] = fast_exp2(fmaf(sacc[4 * rb + 2], sl2, b4.z - lse2));
          dsv[4 * rb + 3] = fast_exp2(fmaf(sacc[4 * rb + 3], sl2, b4.w - lse2));
        }
      } else {
#pragma unroll
        for (int r = 0; r < 16; ++r) dsv[r] = fast_exp2(fmaf(sacc[r], sl2, -lse2));
      }
      if (mask != GFULL || (CAUSAL && sel4(kb, 2 * t + 1) * 16 + 15 > qt * STILE + 32 * w)) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int slot = 2 * t + (r >> 3);
          const int key = sel4(kb, slot) * 16 + 8 * ((r >> 2) & 1) + 4 * h + (r & 3);
          if (!((mask >> ((qsub << 2) + slot)) & 1u) || (CAUSAL && key > myq)) dsv[r] = 0.f;
        }
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) dsv[r] = dsv[r] * (pacc[r] - dl);
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int ks = 2 * t + kk;
        const s16x8 sf = __is_same(T, bf16_t) ? pack8(dsv, 8 * kk) : pack8_h(dsv, 8 * kk);
        const int row1 = 16 * ks + 4 * (g16 >> 1) + qd;
#pragma unroll
        for (int dt = 0; dt < D / 32; ++dt) {
          const int col = 32 * dt + 16 * (g16 & 1) + 4 * pc;
          const s16x4 x = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(Ks + row1 * LDP<D> + col));
          const s16x4 y = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(Ks + (row1 + 8) * LDP<D> + col));
          dq[dt] = Mfma32<T>::run(s16x8{x[0], x[1], x[2], x[3], y[0], y[1], y[2], y[3]}, sf, dq[dt]);
        }
      }
    }
    if (RP) {
      if (has_next) {
        uint16_t* nxt = smem + ((it + 1) & 1) * 2 * TS;
        stile_store<D, NT>(nxt, kr);
        stile_store<D, NT>(nxt + TS, vr);
      }
      __syncthreads();
    }
  }
  uint16_t* dqr = dQ + base + (int64_t)myq * D;
#pragma unroll
  for (int dt = 0; dt < D / 32; ++dt)
#pragma unroll
    for (int rb = 0; rb < 4; ++rb) {
      ushort4 v4;
      v4.x = to16<T>(dq[dt][4 * rb + 0] * scale); v4.y = to16<T>(dq[dt][4 * rb + 1] * scale);
      v4.z = to16<T>(dq[dt][4 * rb + 2] * scale); v4.w = to16<T>(dq[dt][4 * rb + 3] * scale);
      *reinterpret_cast<ushort4*>(dqr + 32 * dt + 8 * rb + 4 * h) = v4;
    }
}

template <int D> constexpr int sfwd_lds(bool rp) { return (rp ? 2 : 1) * 2 * STILE * LDP<D> * 2; }
template <int D> constexpr int sdkdv_lds(bool rp) { return (rp ? 2 : 1) * (2 * STILE * LDP<D> * 2 + 2 * STILE * 4); }

}  // namespace fa

#define FA_DISPATCH(dt, D, causal, ...)                                                              \
  do {                                                                                               \
    auto _go = [&](auto tt, auto dd, auto cc) {                                                      \
      using T = decltype(tt);                                                                        \
      constexpr int DD = decltype(dd)::value;                                                        \
      constexpr bool CC = decltype(cc)::value;                                                       \
      __VA_ARGS__;                                                                                   \
    };                                                                                               \
    auto _d = [&](auto tt, auto cc) {                                                                \
      if (D == 64) _go(tt, std::integral_constant<int, 64>{}, cc);                                  \
      else if (D == 96) _go(tt, std::integral_constant<int, 96>{}, cc);                             \
      else _go(tt, std::integral_constant<int, 128>{}, cc);                                         \
    };                                                                                               \
    auto _c = [&](auto tt) {                                                                         \
      if (causal) _d(tt, std::true_type{}); else _d(tt, std::false_type{});                          \
    };                                                                                               \
    if (dt == kBF16) _c(bf16_t{}); else _c(f16_t{});                                                 \
  } while (0)

bool flash_supported(int D) { return D == 64 || D == 96 || D == 128; }

void launch_flash_fwd(const void* q, const void* k, const void* v, void* o, float* lse, int BH, int S, int D,
                      bool causal, float scale, int dt, hipStream_t s, int onh) {
  // K / V tiles are addressed per head with 32-bit buffer offsets
  if ((int64_t)S * D * 2 >= (1LL << 31))
    throw std::runtime_error("flash fwd: S * head dim too large for 32-bit buffer offsets");
  // v2: lazy rescale, buffer-resource tile loads, transposed-read V layout.  Measured and removed
  // (round 6): a software-pipelined v3 (0.357 vs 0.339 ms at B4 H64 S2048 D96 causal: it needs 2
  // waves/SIMD where v2 runs 3, profiles/r5c_notes.md), the round-1 64-row kernel, eager rescale,
  // pointer-form loads and the round-4 padded layouts.
  const unsigned grid = (unsigned)((S + fa::BM2 - 1) / fa::BM2 * BH);
  FA_DISPATCH(dt, D, causal,
    hipLaunchKernelGGL((fa::fwd_v2_kernel<T, DD, CC, true>), dim3(grid), dim3(256), fa::fwd_v2_lds<DD>(), s,
                       (const uint16_t*)q, (const uint16_t*)k, (const uint16_t*)v, (uint16_t*)o, lse, S, scale, onh));
}

// dQ (+ Delta) first, then dK/dV reading that Delta: two launches, no separate Delta pass.  The
// row constants enter the MFMAs as initial accumulators (v3).  Measured and removed (round 6):
// the round-1 kernels, one merged dK/dV + dQ launch (neutral, r2v) and the v2 bodies behind a
// Delta pass (slower, r4-r5).
void launch_flash_bwd(const void* dout, const void* q, const void* k, const void* v, const void* o, const float* lse,
                      float* delta, void* dq, void* dk, void* dv, int BH, int S, int D, bool causal, float scale,
                      int dt, hipStream_t s, int onh) {
  // the buffer resources of the dK/dV tile loads address one head's rows with 32-bit offsets
  if ((int64_t)S * (onh ? onh * D : D) * 2 >= (1LL << 31))
    throw std::runtime_error("flash bwd: S * row stride too large for 32-bit buffer offsets");
  const unsigned g = (unsigned)((S + fa::BM2 - 1) / fa::BM2 * BH);
  FA_DISPATCH(dt, D, causal,
    hipLaunchKernelGGL((fa::bwd_dq_v3_kernel<T, DD, CC>), dim3(g), dim3(256), fa::fwd_v2_lds<DD>(), s,
                       (const uint16_t*)q, (const uint16_t*)k, (const uint16_t*)v, (const uint16_t*)dout,
                       (const uint16_t*)o, lse, delta, (uint16_t*)dq, S, scale, onh);
    // D = 128: the wave-pair kernel (one wave per SIMD held the whole working set of the
    // single-wave body and shuffled it through AGPRs: 1.50 -> 1.44 ms for the whole backward at
    // B4 H64 S2048 causal, profiles/r6h_dkdv_pair.md); at D = 96 / 64 the single-wave body runs
    // two waves per SIMD on its own and is faster (1.01 vs 1.15 ms at D = 96)
    if constexpr (DD >= 128)
      hipLaunchKernelGGL((fa::bwd_dkdv_pair_kernel<T, DD, CC>), dim3(g), dim3(512), fa::dkdv_pair_lds<DD>(), s,
                         (const uint16_t*)q, (const uint16_t*)k, (const uint16_t*)v, (const uint16_t*)dout, lse,
                         delta, (uint16_t*)dk, (uint16_t*)dv, S, scale, onh);
    else
      hipLaunchKernelGGL((fa::bwd_dkdv_v3_kernel<T, DD, CC>), dim3(g), dim3(256), fa::dkdv_v2_lds<DD>(), s,
                         (const uint16_t*)q, (const uint16_t*)k, (const uint16_t*)v, (const uint16_t*)dout, lse,
                         delta, (uint16_t*)dk, (uint16_t*)dv, S, scale, onh));
}

// Encoder attention (non-causal) with a per-key additive bias and/or in-kernel dropout.
// kbias: [BH / hdiv, S] fp32 or null; p_drop in [0, 1); S % 8 == 0; D in {64, 128}.
// inh > 0: q/k/v and dq/dk/dv are token-major with row stride ild (see fa::Extra).
#define FA_EX_DISPATCH(dt, D, kbias, pdrop, ...)                                                     \
  do {                                                                                               \
    auto _go = [&](auto tt, auto dd, auto ee) {                                                      \
      using T = decltype(tt);                                                                        \
      constexpr int DD = decltype(dd)::value;                                                        \
      constexpr int EE = decltype(ee)::value;                                                        \
      __VA_ARGS__;                                                                                   \
    };                                                                                               \
    auto _q = [&](auto tt, auto dd, auto ee) {                                                       \
      constexpr int E0 = decltype(ee)::value;                                                        \
      if (inh > 0) _go(tt, dd, std::integral_constant<int, E0 | fa::EX_QKV>{});                      \
      else _go(tt, dd, ee);                                                                          \
    };                                                                                               \
    auto _e = [&](auto tt, auto dd) {                                                                \
      if (kbias && pdrop > 0.f) _q(tt, dd, std::integral_constant<int, fa::EX_BIAS | fa::EX_DROP>{}); \
      else if (kbias) _q(tt, dd, std::integral_constant<int, fa::EX_BIAS>{});                       \
      else if (pdrop > 0.f) _q(tt, dd, std::integral_constant<int, fa::EX_DROP>{});                 \
      else _q(tt, dd, std::integral_constant<int, 0>{});                                            \
    };                                                                                               \
    auto _d = [&](auto tt) {                                                                         \
      if (D == 64) _e(tt, std::integral_constant<int, 64>{});                                       \
      else _e(tt, std::integral_constant<int, 128>{});                                              \
    };                                                                                               \
    if (dt == kBF16) _d(bf16_t{}); else _d(f16_t{});                                                 \
  } while (0)

static fa::Extra make_extra(const float* kbias, int hdiv, float pdrop, uint64_t seed, int inh = 0,
                            int64_t ild = 0, const int64_t* rng = nullptr) {
  fa::Extra ex;
  ex.rng = rng;
  ex.inh = inh;
  ex.ild = ild;
  ex.kbias = kbias;
  ex.hdiv = hdiv;
  ex.seed = (uint32_t)(seed ^ (seed >> 32));
  ex.thresh = pdrop > 0.f ? (uint32_t)fminf(65536.f, rintf(pdrop * 65536.f)) : 0u;
  ex.rscale = pdrop > 0.f ? 1.f / (1.f - pdrop) : 1.f;
  return ex;
}

void launch_flash_fwd_ex(const void* q, const void* k, const void* v, void* o, float* lse, int BH, int S, int D,
                         float scale, const float* kbias, int hdiv, float pdrop, uint64_t seed, int dt, hipStream_t s,
                         int onh, int inh, int64_t ild, const int64_t* rng) {
  const fa::Extra ex = make_extra(kbias, hdiv, pdrop, seed, inh, ild, rng);
  const unsigned grid = (unsigned)((S + fa::BM2 - 1) / fa::BM2 * BH);
  const int kb_lds = kbias ? 4 * S : 0;  // the LDS-staged key-bias row
  if (kb_lds && fa::fwd_v2_lds<128>() + kb_lds > 160 * 1024)
    throw std::runtime_error("flash fwd: key-bias row too long for LDS staging");
  if ((int64_t)S * (ild > 0 ? ild : D) * 2 >= (1LL << 31))
    throw std::runtime_error("flash fwd: S * row stride too large for 32-bit buffer offsets");
  FA_EX_DISPATCH(dt, D, kbias, pdrop,
    hipLaunchKernelGGL((fa::fwd_v2_kernel<T, DD, false, true, EE>), dim3(grid), dim3(256), fa::fwd_v2_lds<DD>() + kb_lds, s,
                       (const uint16_t*)q, (const uint16_t*)k, (const uint16_t*)v, (uint16_t*)o, lse, S, scale, onh,
                       ex));
}

void launch_flash_bwd_ex(const void* dout, const void* q, const void* k, const void* v, const void* o,
                         const float* lse, float* delta, void* dq, void* dk, void* dv, int BH, int S, int D,
                         float scale, const float* kbias, int hdiv, float pdrop, uint64_t seed, int dt, hipStream_t s,
                         int onh, int inh, int64_t ild, const int64_t* rng) {
  const fa::Extra ex = make_extra(kbias, hdiv, pdrop, seed, inh, ild, rng);
  const int64_t rows = (int64_t)BH * S;
  const int kb_lds = kbias ? 4 * S : 0;  // the dQ kernel's LDS-staged key-bias row
  if (kb_lds && fa::fwd_v2_lds<128>() + kb_lds > 160 * 1024)
    throw std::runtime_error("flash bwd: key-bias row too long for LDS staging");
  const unsigned grid = (unsigned)((S + fa::BM2 - 1) / fa::BM2 * BH);
  // S <= 128: one workgroup per head does dK, dV and dQ
  const bool use_short = S <= fa::BM2;
  // the buffer resources of the dK/dV tile loads address one head's rows with 32-bit offsets
  if ((int64_t)S * std::max<int64_t>(ild > 0 ? ild : D, onh ? (int64_t)onh * D : D) * 2 >= (1LL << 31))
    throw std::runtime_error("flash bwd: S * row stride too large for 32-bit buffer offsets");
  // Delta from its own pass: the short backward forming it per workgroup measured slower (BERT-Large
  // seq 128: 2,530 vs 2,551 samples/s, profiles/r5f_bert_short_delta_ab2.jsonl), removed in round 6
  FA_EX_DISPATCH(dt, D, kbias, pdrop,
    hipLaunchKernelGGL((fa::delta_kernel<T, DD>), dim3((unsigned)((rows * 8 + 255) / 256)), dim3(256), 0, s,
                       (const uint16_t*)dout, (const uint16_t*)o, delta, rows, S, onh);
    if (use_short)
      hipLaunchKernelGGL((fa::bwd_short_kernel<T, DD, EE>), dim3(grid), dim3(256), fa::bwd_short_lds<DD>(), s,
                         (const uint16_t*)q, (const uint16_t*)k, (const uint16_t*)v, (const uint16_t*)dout, lse, delta,
                         (uint16_t*)dq, (uint16_t*)dk, (uint16_t*)dv, S, scale, onh, ex);
    else {
      hipLaunchKernelGGL((fa::bwd_dkdv_v2_kernel<T, DD, false, EE>), dim3(grid), dim3(256), fa::dkdv_v2_lds<DD>(), s,
                         (const uint16_t*)q, (const uint16_t*)k, (const uint16_t*)v, (const uint16_t*)dout, lse, delta,
                         (uint16_t*)dk, (uint16_t*)dv, S, scale, onh, ex);
      hipLaunchKernelGGL((fa::bwd_dq_v2_kernel<T, DD, false, EE>), dim3(grid), dim3(256), fa::fwd_v2_lds<DD>() + kb_lds, s,
                         (const uint16_t*)q, (const uint16_t*)k, (const uint16_t*)v, (const uint16_t*)dout, lse, delta,
                         (uint16_t*)dq, S, scale, onh, ex);
    });
}

// (sparse kernels: register prefetch + double-buffered LDS, 2 workgroups / CU -- measured faster
// than one LDS stage at 3 workgroups / CU, which was removed in round 6)

// kbias / ebias (SExtra): null when absent; either one selects the SX = 1 kernels
void launch_sparse_flash_fwd(const void* q, const void* k, const void* v, void* o, float* lse, const int* rowptr,
                             const int* cols_, const uint32_t* masks, int BH, int H, int Hl, int S, int D, bool causal,
                             float scale, int shift, int dt, hipStream_t s, int onh, const float* kbias,
                             const void* ebias, int64_t ez, int64_t eh, int64_t er) {
  const int4* cols = reinterpret_cast<const int4*>(cols_);
  const unsigned grid = (unsigned)(BH * (S / fa::STILE));
  fa::SExtra sx;
  sx.kbias = kbias;
  sx.ebias = (const uint16_t*)ebias;
  sx.ez = ez; sx.eh = eh; sx.er = er;
  FA_DISPATCH(dt, D, causal,
    if (ebias)
      hipLaunchKernelGGL((fa::sfwd_kernel<T, DD, CC, true, 3>), dim3(grid), dim3(128), fa::sfwd_lds<DD>(true), s,
                         (const uint16_t*)q, (const uint16_t*)k, (const uint16_t*)v, (uint16_t*)o, lse, rowptr, cols,
                         masks, S, scale, onh, H, Hl, shift, sx);
    else if (kbias)
      hipLaunchKernelGGL((fa::sfwd_kernel<T, DD, CC, true, 1>), dim3(grid), dim3(128), fa::sfwd_lds<DD>(true), s,
                         (const uint16_t*)q, (const uint16_t*)k, (const uint16_t*)v, (uint16_t*)o, lse, rowptr, cols,
                         masks, S, scale, onh, H, Hl, shift, sx);
    else
      hipLaunchKernelGGL((fa::sfwd_kernel<T, DD, CC, true>), dim3(grid), dim3(128), fa::sfwd_lds<DD>(true), s,
                         (const uint16_t*)q, (const uint16_t*)k, (const uint16_t*)v, (uint16_t*)o, lse, rowptr, cols,
                         masks, S, scale, onh, H, Hl, shift, fa::SExtra()));
}

// Backward: dQ first (it also forms Delta for its rows), then dK / dV reading that Delta, then the
// sums of split key tiles' partials.
void launch_sparse_flash_bwd(const void* dout, const void* q, const void* k, const void* v, const void* o,
                             const float* lse, float* delta, void* dq, void* dk, void* dv, const int* rowptr,
                             const int* cols_, const uint32_t* masks, const int* rows_, const uint32_t* masks_t,
                             const int* tasks, int ntask, const int* fin, int nfin, const int* kgroups_, float* ws,
                             int nslot, int BH, int H, int Hl, int S, int D, bool causal, float scale, int shift,
                             int dt, hipStream_t s, int onh, const float* kbias, const void* ebias, int64_t ez,
                             int64_t eh, int64_t er) {
  const int4* cols = reinterpret_cast<const int4*>(cols_);
  const int4* rows = reinterpret_cast<const int4*>(rows_);
  const int4* kgroups = reinterpret_cast<const int4*>(kgroups_);
  const unsigned grid = (unsigned)(BH * (S / fa::STILE));
  const unsigned tgrid = (unsigned)(BH * ntask);
  const int4* tk = reinterpret_cast<const int4*>(tasks);
  fa::SExtra sx;
  sx.kbias = kbias;
  sx.ebias = (const uint16_t*)ebias;
  sx.ez = ez; sx.eh = eh; sx.er = er;
  FA_DISPATCH(dt, D, causal,
    if (ebias) {
      hipLaunchKernelGGL((fa::sdq_kernel<T, DD, CC, true, 3, true>), dim3(grid), dim3(128), fa::sfwd_lds<DD>(true), s,
                         (const uint16_t*)q, (const uint16_t*)k, (const uint16_t*)v, (const uint16_t*)dout, lse, delta,
                         (uint16_t*)dq, rowptr, cols, masks, S, scale, onh, H, Hl, shift, sx, (const uint16_t*)o);
      hipLaunchKernelGGL((fa::sdkdv_kernel<T, DD, CC, true, 3>), dim3(tgrid), dim3(128), fa::sdkdv_lds<DD>(true), s,
                         (const uint16_t*)q, (const uint16_t*)k, (const uint16_t*)v, (const uint16_t*)dout, lse, delta,
                         (uint16_t*)dk, (uint16_t*)dv, rows, masks_t, tk, ntask, kgroups, ws, nslot, S, scale, onh, H, Hl,
                         shift, sx);
    } else if (kbias) {
      hipLaunchKernelGGL((fa::sdq_kernel<T, DD, CC, true, 1, true>), dim3(grid), dim3(128), fa::sfwd_lds<DD>(true), s,
                         (const uint16_t*)q, (const uint16_t*)k, (const uint16_t*)v, (const uint16_t*)dout, lse, delta,
                         (uint16_t*)dq, rowptr, cols, masks, S, scale, onh, H, Hl, shift, sx, (const uint16_t*)o);
      hipLaunchKernelGGL((fa::sdkdv_kernel<T, DD, CC, true, 1>), dim3(tgrid), dim3(128), fa::sdkdv_lds<DD>(true), s,
                         (const uint16_t*)q, (const uint16_t*)k, (const uint16_t*)v, (const uint16_t*)dout, lse, delta,
                         (uint16_t*)dk, (uint16_t*)dv, rows, masks_t, tk, ntask, kgroups, ws, nslot, S, scale, onh, H, Hl,
                         shift, sx);
    } else {
      hipLaunchKernelGGL((fa::sdq_kernel<T, DD, CC, true, 0, true>), dim3(grid), dim3(128), fa::sfwd_lds<DD>(true), s,
                         (const uint16_t*)q, (const uint16_t*)k, (const uint16_t*)v, (const uint16_t*)dout, lse, delta,
                         (uint16_t*)dq, rowptr, cols, masks, S, scale, onh, H, Hl, shift, fa::SExtra(),
                         (const uint16_t*)o);
      hipLaunchKernelGGL((fa::sdkdv_kernel<T, DD, CC, true>), dim3(tgrid), dim3(128), fa::sdkdv_lds<DD>(true), s,
                         (const uint16_t*)q, (const uint16_t*)k, (const uint16_t*)v, (const uint16_t*)dout, lse, delta,
                         (uint16_t*)dk, (uint16_t*)dv, rows, masks_t, tk, ntask, kgroups, ws, nslot, S, scale, onh, H, Hl,
                         shift, fa::SExtra());
    }
    if (nfin > 0)
      hipLaunchKernelGGL((fa::sdkdv_finish_kernel<T, DD>), dim3((unsigned)(BH * nfin * fa::sdkdv_fparts<DD>())),
                         dim3(256), 0, s, ws, reinterpret_cast<const int4*>(fin), nfin, nslot, (uint16_t*)dk,
                         (uint16_t*)dv, S, scale, H, Hl, kgroups));
}

}  // namespace dsa
