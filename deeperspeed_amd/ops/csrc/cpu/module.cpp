// `_cpu_ops`: host-side native ops (CPU Adam, async NVMe I/O, flatten/unflatten, sparse
// attention LUT segmentation).  Reference parity: csrc/adam/cpu_adam.cpp:682-690,
// csrc/aio/py_lib/py_ds_aio.cpp:12-41, csrc/utils/flatten_unflatten.cpp:21-25,
// csrc/sparse_attention/utils.cpp:119.
#include <torch/extension.h>
#include <torch/csrc/utils/tensor_flatten.h>

void cpu_adam_update(at::Tensor p, at::Tensor g, at::Tensor m, at::Tensor v, double lr, double b1, double b2,
                     double eps, double wd, int64_t step, bool bias_correction, double grad_scale, bool adamw,
                     c10::optional<at::Tensor> out);
int64_t cpu_adam_isa();
void register_aio(pybind11::module& m);
void register_sparse_utils(pybind11::module& m);

at::Tensor flatten(std::vector<at::Tensor> tensors) { return torch::utils::flatten_dense_tensors(tensors); }

std::vector<at::Tensor> unflatten(at::Tensor flat, std::vector<at::Tensor> tensors) {
  return torch::utils::unflatten_dense_tensors(flat, tensors);
}

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "deeperspeed_amd host-side native ops";
  m.def("adam_update", &cpu_adam_update, "fused Adam/AdamW step on host tensors (AVX-512/AVX2/scalar)");
  m.def("adam_isa", &cpu_adam_isa, "0=scalar 1=avx2 2=avx512");
  m.def("flatten", &flatten, "Flatten dense tensors");
  m.def("unflatten", &unflatten, "Unflatten dense tensors");
  register_aio(m);
  register_sparse_utils(m);
}
