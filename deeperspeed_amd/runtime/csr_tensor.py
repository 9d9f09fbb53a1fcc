"""Row-compressed gradient of an embedding table.

Behaviour of reference deepspeed/runtime/csr_tensor.py:11-59 (same class name, `type()`
string, `indices` / `values` / `dense_size` attributes, `add` concatenating duplicates and
`to_dense` summing them): only the rows an embedding gradient touched travel over the
data-parallel all-gather, and duplicates from different ranks are summed on densify.

Implementation: rows are selected with `any(dim=1)` and densified with `index_add_` (one
kernel, row-granular) instead of an expanded column index + scatter.
"""

import torch


class CSRTensor:
    def __init__(self, dense_tensor=None):
        self.orig_dense_tensor = dense_tensor
        self.indices = self.values = self.dense_size = None
        if dense_tensor is None:
            return
        dense = dense_tensor.coalesce().to_dense() if dense_tensor.is_sparse else dense_tensor
        rows = dense.reshape(dense.shape[0], -1).ne(0).any(dim=1)
        self.indices = torch.nonzero(rows, as_tuple=True)[0]
        self.values = dense.index_select(0, self.indices)
        self.dense_size = list(dense.shape)

    @staticmethod
    def type():
        return "deepspeed.CSRTensor"

    def to_dense(self):
        out = torch.zeros(self.dense_size, dtype=self.values.dtype, device=self.values.device)
        return out.index_add_(0, self.indices, self.values)

    def sparse_size(self):
        """(elements stored sparsely, elements of the dense tensor)."""
        dense_elems = 1
        for d in self.dense_size:
            dense_elems *= d
        row_len = dense_elems // max(self.dense_size[0], 1)
        return self.indices.numel() + self.values.shape[0] * row_len, dense_elems

    def add(self, b):
        """Append another tensor's rows (duplicates are summed by to_dense)."""
        assert self.dense_size == b.dense_size, "CSRTensor.add needs equal dense sizes"
        self.indices = torch.cat((self.indices, b.indices))
        self.values = torch.cat((self.values, b.values))

    def __str__(self):
        stored, dense = self.sparse_size()
        dev = self.indices.get_device() if self.indices.is_cuda else -1
        return (f"DeepSpeed.CSRTensor(indices_size={self.indices.size()}, values_size={self.values.size()}, "
                f"dense_size={self.dense_size}, device={dev}, reduction_factor={dense / max(stored, 1)})")

    __repr__ = __str__
