"""Mantissa/exponent-split all-reduce (reference deepspeed/runtime/comm/compressed_ar.py, a
DeeperSpeed experiment).

`decompose(t)` splits a tensor into an fp16 mantissa in [0.5, 1) and an int8 exponent
(frexp); `compressed_all_reduce` all-reduces the two parts separately (2 + 1 bytes per element
on the wire instead of 4) and rebuilds ldexp(sum(m), sum(e)).  Like the reference, the rebuilt
value equals the input at world size 1 but is NOT the element-wise sum of the inputs for larger
groups; it is kept for API parity, not used by the engine.  torch.frexp replaces the CuPy path
(torch >= 1.9 is always true here)."""

import torch
import torch.distributed as dist


def decompose(t: torch.Tensor):
    mantissa, exponent = torch.frexp(t.float())
    return mantissa.half(), exponent.to(torch.int8)


def reconstruct(mantissa: torch.Tensor, exponent: torch.Tensor, original_dtype=torch.bfloat16):
    return torch.ldexp(mantissa.float(), exponent.to(torch.int32)).to(original_dtype)


def compressed_all_reduce(tensor, op=dist.ReduceOp.SUM, group=None, async_op=False):
    m, e = decompose(tensor)
    if dist.is_available() and dist.is_initialized():
        w1 = dist.all_reduce(m, op=op, group=group, async_op=async_op)
        w2 = dist.all_reduce(e, op=op, group=group, async_op=async_op)
        if async_op:
            w1.wait()
            w2.wait()
    return reconstruct(m, e, tensor.dtype)


compressed_all_reduce_torch = compressed_all_reduce
