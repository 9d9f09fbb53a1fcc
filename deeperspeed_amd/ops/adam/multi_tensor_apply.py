"""Apex-style multi-tensor launcher object (reference deepspeed/ops/adam/multi_tensor_apply.py).

`MultiTensorApply(chunk)(op, noop_flag, tensor_lists, *args)` calls `op(chunk, noop_flag,
tensor_lists, *args)`.  The framework's own multi-tensor kernels (FusedAdam `adam_multi`, FusedLamb
`lamb_multi`) build a device meta table of tensor pointers and a chunk prefix instead of the
reference's fixed-size kernel-argument structs; this object is kept for callers that pass their
own op."""


class MultiTensorApply:
    available = True
    warned = False

    def __init__(self, chunk_size: int):
        self.chunk_size = int(chunk_size)

    def __call__(self, op, noop_flag_buffer, tensor_lists, *args):
        return op(self.chunk_size, noop_flag_buffer, tensor_lists, *args)
