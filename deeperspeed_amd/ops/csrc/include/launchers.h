// Host-side launcher declarations shared by the .hip translation units and the
// torch binding unit. Kernels never include torch headers (keeps device compiles
// fast); bindings never include kernel code.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dsa {

enum DTypeCode : int { kCodeF32 = 0, kCodeBF16 = 1, kCodeF16 = 2 };

struct AdamArgs {
  float lr, beta1, beta2, eps, weight_decay;
  float bc1, bc2;
  float grad_scale;
  int adamw;
};

struct LambArgs {
  float lr, beta1, beta2, eps, weight_decay, bc1, bc2, grad_scale;
  float max_coeff, min_coeff;
  int adamw;
  // optional device-resident factor multiplied into grad_scale (unscale x clip computed on the
  // GPU after backward, no host round trip); a non-finite value skips the whole update
  const float* scale_ptr = nullptr;
  // optional device-resident step size replacing lr (the bias correction of a step counter kept
  // on the GPU, so a captured HIP graph of the whole training step advances it on every replay)
  const float* lr_ptr = nullptr;
};

// optim.hip
void launch_adam_flat(void* w, int wt, const void* g, int gt, float* m, float* v, void* out, int ot, int64_t n,
                      AdamArgs a, hipStream_t s);
void launch_adam_compact(void* hi, void* res, const void* g, int gt, float* m, float* v, int64_t n, AdamArgs a,
                         hipStream_t s);
void launch_adam_multi(const int64_t* meta, int T, int64_t total_chunks, int64_t chunk, int wt, int gt, int ot,
                       AdamArgs a, hipStream_t s);
void launch_sumsq_accum(const void* x, int xt, int64_t n, float* workspace, float* out, hipStream_t s);
void launch_sumsq_multi(const int64_t* meta, int nt, int64_t total_chunks, int64_t chunk, int xt, float* partial,
                        float* out, hipStream_t s);
void launch_copy_narrow(const void* src, void* dst, int64_t bytes, int wgs, hipStream_t s);
void launch_scale_copy(const void* x, int xt, void* y, int yt, int64_t n, const float* scale_ptr, float scale,
                       hipStream_t s, int accumulate = 0);
void launch_lamb(void* w, int wt, const void* g, int gt, float* m, float* v, float* upd, void* out, int ot,
                 int64_t n, LambArgs a, float* workspace, float* coeff_out, hipStream_t s);
void launch_lamb_multi(const int64_t* meta, int T, int64_t total_chunks, int64_t chunk, int wt, int gt, int ot,
                       LambArgs a, float* partial, float* coeff, hipStream_t s);

// norm_act.hip
int ln_max_hidden(int dt);
int ln_bwd_grid(int64_t rows);
void launch_ln_fwd(const void* x, const void* res, const void* bias, void* sum_out, const void* gamma,
                   const void* beta, void* y, float* mean, float* rstd, int64_t rows, int H, float eps, int dt,
                   hipStream_t s);
void launch_ln_bwd(const void* dy, const void* x, const void* gamma, const float* mean, const float* rstd,
                   const void* dres, void* dx, void* dgamma, void* dbeta, float* partial, int64_t rows, int H,
                   int dt, hipStream_t s, int accum = 0);  // accum: dgamma / dbeta += the new sums
// y = a + b (+ c), n % (16 B / elem) == 0
void launch_sum_slices(const void* part, int S, int64_t n, void* out, bool out_f32, int accum, int dt,
                       hipStream_t s);
void launch_sum_slices_f32(const float* part, int S, int64_t n, void* out, int accum, int out_dt, hipStream_t s);
void dropout_bwd_colsum_dims(int64_t rows, int C, int dt, int* cblocks, int* rchunks, int* prows);
void launch_dropout_bwd_colsum(const void* dy, const uint8_t* mask, void* dx, void* db, float* partial, int64_t rows,
                               int C, float p, int dt, hipStream_t s);
void launch_add3(const void* a, const void* b, const void* c, void* y, int64_t n, int dt, hipStream_t s);
void launch_bias_gelu_fwd(const void* x, const void* b, void* y, int64_t rows, int C, int approx, int dt,
                          hipStream_t s);
int bias_gelu_row_chunks(int64_t rows, int C, int dt);
void launch_bias_gelu_bwd(const void* dy, const void* x, const void* b, void* dx, void* db, float* partial,
                          int64_t rows, int C, int approx, int dt, hipStream_t s, int db_accum = 0);
void launch_colsum(const void* x, void* out, float* partial, int64_t rows, int C, int accum, int dt,
                   hipStream_t s);
// out[c] (+)= sum_r partial[r][c] (fp32 partials, out in dtype dt)
void launch_colsum_partials(const float* partial, int R, int C, void* out, int accum, int dt, hipStream_t s);
// three consecutive [R, C] partial blocks into out1, out2 (accum12) and out3 (accum3) in one launch;
// a null out skips its block
void launch_colsum3(const float* partial, int R, int C, void* out1, void* out2, void* out3, int accum12, int accum3,
                    int dt, hipStream_t s);
// embedding.hip: sync-free deterministic embedding backward over sorted ids (H % 8 == 0)
int64_t embedding_bwd_chunks(int64_t n);
void launch_embedding_bwd_sorted(const int64_t* sorted_ids, const int64_t* perm, const void* dy, void* dw,
                                 float* head, float* cont, int64_t n, int H, int64_t padding_idx, int accumulate,
                                 int dt, hipStream_t s);
// empty trace-marker kernel (timed-region boundaries in a rocprofv3 kernel trace)
void launch_profile_marker(int tag, hipStream_t s);

// transpose.hip: y[C][R] = x[R][C] (16-bit; R % 128 == 0, C % 64 == 0, x row stride ldx).  With
// `partial` ([R/128, C] fp32 scratch) the column sums of x are also (accumulated) into colsum_out[C].
bool transpose_supported(int64_t R, int64_t C);
int64_t transpose_partial_rows(int64_t R);
// [L][R][C] (row stride ldx) -> [L][C][R], one launch (plain copy, no column sums)
void launch_transpose_batched(const void* x, void* y, int L, int64_t R, int C, int64_t ldx, int dt, hipStream_t s);
void launch_transpose(const void* x, void* y, float* partial, void* colsum_out, int colsum_accum, int64_t R, int C,
                      int64_t ldx, int dt, hipStream_t s);
// yt[C][R] = gelu(x[R][C] + b)^T (same shape rules, x contiguous)
void launch_bias_gelu_fwd_t(const void* x, const void* b, void* yt, int64_t R, int C, int approx, int dt,
                            hipStream_t s);
// dx = dy * gelu'(x + b) row-major and dxt = dx^T; db = column sums of dx (when partial != null)
void launch_bias_gelu_bwd_t(const void* dy, const void* x, const void* b, void* dx, void* dxt, float* partial,
                            void* db, int64_t R, int C, int approx, int dt, hipStream_t s);

// attn_elem.hip
void launch_rotary_split_fwd(const void* qkv, void* q, void* k, void* v, const float* cs, int B, int S, int NH,
                             int HD, int ROT, float qscale, int dt, hipStream_t s);
void launch_rotary_split_bwd(const void* dq, const void* dk, const void* dv, void* dqkv, const float* cs, int B,
                             int S, int NH, int HD, int ROT, float qscale, int dt, hipStream_t s);
// 16-bit layout moves (HD, D multiples of 8): qkv [B,S,3,NH,HD] <-> q,k,v [B,NH,S,HD]; x [A,P,Q,D] -> [A,Q,P,D]
void launch_heads_split(const void* qkv, void* q, void* k, void* v, int B, int S, int NH, int HD, hipStream_t s);
void launch_heads_merge(const void* q, const void* k, const void* v, void* qkv, int B, int S, int NH, int HD,
                        hipStream_t s);
void launch_swap12(const void* x, void* y, int64_t A, int P, int Q, int D, hipStream_t s);
int softmax_max_cols();
void launch_softmax_fwd(const void* x, void* y, const void* mask, int64_t R, int C, int Sq, int heads, float scale,
                        int causal, int mask_rows, int dt, hipStream_t s);
void launch_softmax_bwd(const void* dy, const void* y, void* dx, int64_t R, int C, float scale, int dt,
                        hipStream_t s);

// loss.hip: fused softmax cross-entropy over [rows, V] 16-bit logits
void launch_xent_fwd(const void* x, const int64_t* labels, float* loss, float* lse, int64_t rows, int V, int dt,
                     hipStream_t s);
void launch_xent_bwd(const void* x, const int64_t* labels, const float* lse, const float* dloss, int64_t dloss_stride,
                     void* dx, int64_t rows, int V, int dt, hipStream_t s);

// onebit.hip: 1-bit error-compensated compression (ws >= 1024 floats)
void launch_onebit_worker(const float* m, float* err, int64_t n, uint8_t* packed, float* scale_out, float* ws,
                          hipStream_t s);
void launch_onebit_server(const uint8_t* signs, const float* scales, int P, int64_t nbytes, float* server_err,
                          uint8_t* packed, float* scale_out, float* ws, hipStream_t s);
void launch_onebit_unpack(const uint8_t* signs, const float* scales, int P, int64_t nbytes_per, float* out,
                          hipStream_t s);

// sparse_attn.hip: block-sparse attention (LUTs from ops/sparse_attention)
// strides are {z, h, row, k} in elements; at/bt/dtr/ctr = the row dim (not k) is the unit-stride one
void launch_sparse_sdd(const void* A, const int64_t* sa, bool at, const void* B, const int64_t* sb, bool bt, void* C,
                       const int* nz, int nnz, int Z, int K, int blk, float alpha, int dt, hipStream_t s);
void launch_sparse_dsd(const void* S, const int* seg, int nseg, const int* fin, int nfin, const int* cols,
                       const int* perm, const void* D, const int64_t* sd, bool dtr, void* C, const int64_t* sc,
                       bool ctr, float* ws, int nslots, int nnz, int Z, int nbr, int N, int blk, int dt,
                       hipStream_t s);
void launch_sparse_softmax_fwd(const void* x, void* y, const int* rowptr, const int* cols, int nnz, int Z, int H,
                               int nbr, int blk, int max_row, const void* rpe, int64_t rpe_sz, int64_t rpe_sh,
                               int64_t rpe_sr, const void* kpm, int64_t kpm_sz, const void* attn, int64_t attn_sr,
                               int kpm_mul, int attn_mul, float scale, int causal, int dt, hipStream_t s);
void launch_sparse_softmax_bwd(const void* y, const void* dy, void* dx, const int* rowptr, int nnz, int Z, int H,
                               int nbr, int blk, int max_row, float scale, int dt, hipStream_t s);

// dropout.hip: counter-based Philox dropout (seed, offset) with uint8 keep-masks
// rng: optional device int64 [seed, step] read by the kernels (graph-replayable masks, dropout.hip)
void launch_dropout_fwd(const void* x, void* y, uint8_t* mask, int64_t n, float p, uint64_t seed, uint64_t offset,
                        int dt, hipStream_t s, const int64_t* rng = nullptr);
void launch_bias_dropout_residual(const void* x, const void* bias, const void* res, void* y, uint8_t* mask,
                                  int64_t rows, int C, float p, uint64_t seed, uint64_t offset, int dt, hipStream_t s,
                                  const int64_t* rng = nullptr);
void launch_dropout_bwd(const void* dy, const uint8_t* mask, void* dx, int64_t n, float p, int dt, hipStream_t s);
// out = res + dropout(x + bias) and y = LayerNorm(out) in one pass (16-bit, H % 8 == 0, H <= 1024)
bool bdr_ln_supported(int H, int dt);
int bdr_ln_bwd_grid(int64_t rows);
void launch_bdr_ln_fwd(const void* x, const void* bias, const void* res, void* out, uint8_t* mask, const void* gamma,
                       const void* beta, void* y, float* mean, float* rstd, int64_t rows, int H, float p, float eps,
                       uint64_t seed, uint64_t offset, int dt, hipStream_t s, const int64_t* rng = nullptr);
// its backward: dtot = LN-backward(dy) + dres, dxb = dtot * mask / (1 - p); gamma / beta / bias
// gradients from one set of partials (3 * bdr_ln_bwd_grid(rows) * H floats); accum: dgamma / dbeta
// +=, accum_bias: dbias +=
void launch_bdr_ln_bwd(const void* dy, const void* xo, const void* gamma, const float* mean, const float* rstd,
                       const void* dres, const uint8_t* mask, void* dtot, void* dxb, void* dgamma, void* dbeta,
                       void* dbias, float* partial, int64_t rows, int H, float p, int accum, int accum_bias, int dt,
                       hipStream_t s);

// flash_attn.hip: q,k,v,o [BH, S, D] (D in 64/96/128), lse/delta [BH, S] fp32
bool flash_supported(int D);
void launch_flash_fwd(const void* q, const void* k, const void* v, void* o, float* lse, int BH, int S, int D,
                      bool causal, float scale, int dt, hipStream_t s, int onh = 0);
void launch_flash_bwd(const void* dout, const void* q, const void* k, const void* v, const void* o, const float* lse,
                      float* delta, void* dq, void* dk, void* dv, int BH, int S, int D, bool causal, float scale,
                      int dt, hipStream_t s, int onh = 0);
// block-sparse flash attention (S % 64 == 0): LUTs per layout head (Hl = 1 or H), shift =
// min(6, log2(layout block))
void launch_flash_fwd_ex(const void* q, const void* k, const void* v, void* o, float* lse, int BH, int S, int D,
                         float scale, const float* kbias, int hdiv, float pdrop, uint64_t seed, int dt, hipStream_t s,
                         int onh, int inh = 0, int64_t ild = 0, const int64_t* rng = nullptr);
void launch_flash_bwd_ex(const void* dout, const void* q, const void* k, const void* v, const void* o,
                         const float* lse, float* delta, void* dq, void* dk, void* dv, int BH, int S, int D,
                         float scale, const float* kbias, int hdiv, float pdrop, uint64_t seed, int dt, hipStream_t s,
                         int onh, int inh = 0, int64_t ild = 0, const int64_t* rng = nullptr);
void launch_sparse_flash_fwd(const void* q, const void* k, const void* v, void* o, float* lse, const int* rowptr,
                             const int* cols, const uint32_t* masks, int BH, int H, int Hl, int S, int D, bool causal,
                             float scale, int shift, int dt, hipStream_t s, int onh = 0,
                             const float* kbias = nullptr, const void* ebias = nullptr, int64_t ez = 0,
                             int64_t eh = 0, int64_t er = 0);
void launch_sparse_flash_bwd(const void* dout, const void* q, const void* k, const void* v, const void* o,
                             const float* lse, float* delta, void* dq, void* dk, void* dv, const int* rowptr,
                             const int* cols, const uint32_t* masks, const int* rows, const uint32_t* masks_t,
                             const int* tasks, int ntask, const int* fin, int nfin, const int* kgroups, float* ws,
                             int nslot, int BH, int H, int Hl, int S, int D, bool causal, float scale, int shift,
                             int dt, hipStream_t s, int onh = 0, const float* kbias = nullptr, const void* ebias = nullptr, int64_t ez = 0,
                             int64_t eh = 0, int64_t er = 0);

}  // namespace dsa
