// Block-sparse layout -> lookup tables for the HIP block-sparse attention kernels.
//
// Reference parity: csrc/sparse_attention/utils.cpp (`sdd_segment`, OpenMP LUT
// segmentation for the Triton kernels).  Our kernels consume a CSR view of the layout:
// for every (head, block-row) the list of non-zero block-columns and, for each, the
// index of that block in the packed sparse tensor (row-major order of non-zeros over
// [head, row, col]) -- plus the transposed (column-major) CSR used by the backward /
// DSD / DDS products.
#include <torch/extension.h>
#include <omp.h>

#include <vector>

namespace {

// layout: int [H, R, C] (0/1). Returns {row_ptr [H*R+1], col_idx [nnz], blk_id [nnz],
// col_ptr [H*C+1], row_idx [nnz], blk_id_t [nnz]}.
std::vector<at::Tensor> block_lut(at::Tensor layout) {
  TORCH_CHECK(layout.dim() == 3, "block_lut: layout must be [heads, rows, cols]");
  auto L = layout.to(at::kInt).contiguous();
  const int64_t H = L.size(0), R = L.size(1), C = L.size(2);
  const int* lp = L.data_ptr<int>();
  // row counts
  std::vector<int64_t> row_cnt(H * R, 0), col_cnt(H * C, 0);
#pragma omp parallel for
  for (int64_t hr = 0; hr < H * R; ++hr) {
    int64_t c = 0;
    for (int64_t j = 0; j < C; ++j) c += lp[hr * C + j] != 0;
    row_cnt[hr] = c;
  }
  auto opts = at::TensorOptions().dtype(at::kInt);
  at::Tensor row_ptr = at::empty({H * R + 1}, opts);
  int* rp = row_ptr.data_ptr<int>();
  rp[0] = 0;
  for (int64_t i = 0; i < H * R; ++i) rp[i + 1] = rp[i] + (int)row_cnt[i];
  const int64_t nnz = rp[H * R];
  at::Tensor col_idx = at::empty({nnz}, opts), blk_id = at::empty({nnz}, opts);
  int* ci = col_idx.data_ptr<int>();
  int* bi = blk_id.data_ptr<int>();
#pragma omp parallel for
  for (int64_t hr = 0; hr < H * R; ++hr) {
    int64_t k = rp[hr];
    for (int64_t j = 0; j < C; ++j)
      if (lp[hr * C + j]) {
        ci[k] = (int)j;
        bi[k] = (int)k;
        ++k;
      }
  }
  // transposed (per head, per block-column)
  for (int64_t h = 0; h < H; ++h)
    for (int64_t r = 0; r < R; ++r)
      for (int64_t j = 0; j < C; ++j) col_cnt[h * C + j] += lp[(h * R + r) * C + j] != 0;
  at::Tensor col_ptr = at::empty({H * C + 1}, opts);
  int* cp = col_ptr.data_ptr<int>();
  cp[0] = 0;
  for (int64_t i = 0; i < H * C; ++i) cp[i + 1] = cp[i] + (int)col_cnt[i];
  at::Tensor row_idx = at::empty({nnz}, opts), blk_t = at::empty({nnz}, opts);
  int* ri = row_idx.data_ptr<int>();
  int* bt = blk_t.data_ptr<int>();
  std::vector<int64_t> fill(H * C, 0);
  for (int64_t h = 0; h < H; ++h)
    for (int64_t r = 0; r < R; ++r)
      for (int64_t k = rp[h * R + r]; k < rp[h * R + r + 1]; ++k) {
        const int64_t j = ci[k];
        const int64_t pos = cp[h * C + j] + fill[h * C + j]++;
        ri[pos] = (int)r;
        bt[pos] = (int)k;
      }
  return {row_ptr, col_idx, blk_id, col_ptr, row_idx, blk_t};
}

// Reference-compatible segmentation helper: splits each row's non-zero count into
// segments of at most `start_width` blocks (used to bound per-workgroup work).
std::vector<at::Tensor> sdd_segment(at::Tensor layout, int64_t start_width) {
  auto L = layout.to(at::kInt).contiguous();
  TORCH_CHECK(L.dim() == 3, "sdd_segment: layout must be [heads, rows, cols]");
  const int64_t H = L.size(0), R = L.size(1), C = L.size(2);
  const int* lp = L.data_ptr<int>();
  std::vector<int> segs;  // (head, row, start_col_index_in_row, width)
  for (int64_t h = 0; h < H; ++h)
    for (int64_t r = 0; r < R; ++r) {
      int64_t cnt = 0;
      for (int64_t j = 0; j < C; ++j) cnt += lp[(h * R + r) * C + j] != 0;
      for (int64_t s = 0; s < cnt; s += start_width) {
        segs.push_back((int)h);
        segs.push_back((int)r);
        segs.push_back((int)s);
        segs.push_back((int)std::min<int64_t>(start_width, cnt - s));
      }
    }
  at::Tensor out = at::empty({(int64_t)segs.size() / 4, 4}, at::TensorOptions().dtype(at::kInt));
  if (!segs.empty()) std::memcpy(out.data_ptr<int>(), segs.data(), segs.size() * sizeof(int));
  return {out};
}

}  // namespace

void register_sparse_utils(pybind11::module& m) {
  m.def("block_lut", &block_lut, "CSR + CSC lookup tables of a block-sparse layout");
  m.def("sdd_segment", &sdd_segment, "row segmentation of a block-sparse layout");
}
