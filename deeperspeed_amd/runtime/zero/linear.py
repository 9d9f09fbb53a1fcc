"""Linear layer whose autograd graph does not pin gathered ZeRO-3 weights.

Reference parity: deepspeed/runtime/zero/linear.py:29-168 (`LinearFunctionForZeroStage3`,
`LinearModuleForZeroStage3`).  The autograd context keeps the *Parameter object* (not the
gathered storage): ZeRO-3 swaps `param.data` between the shard placeholder and the gathered
tensor, and the pre-backward hook re-gathers it, so backward always sees the full weight
without the forward keeping a second reference to it alive.  The weight gradient is produced
in the parameter dtype with fp32 accumulation (hipBLASLt) and the bias gradient by the HIP
column-sum kernel.
"""

import torch
import torch.nn.functional as F

from ...ops import native


class LinearFunctionForZeroStage3(torch.autograd.Function):
    @staticmethod
    def forward(ctx, input, weight, bias=None):
        ctx.save_for_backward(input)
        ctx.weight = weight  # the Parameter: its .data is re-gathered before backward runs
        ctx.has_bias = bias is not None
        ctx.bias_dtype = bias.dtype if bias is not None else None
        return F.linear(input, weight, bias)

    @staticmethod
    def backward(ctx, grad_output):
        (input,) = ctx.saved_tensors
        weight = ctx.weight
        grad_input = grad_weight = grad_bias = None
        if ctx.needs_input_grad[0]:
            grad_input = grad_output.matmul(weight)
        if ctx.needs_input_grad[1]:
            go = grad_output.reshape(-1, grad_output.shape[-1])
            grad_weight = go.t().matmul(input.reshape(-1, input.shape[-1]))
        if ctx.has_bias and ctx.needs_input_grad[2]:
            grad_bias = native.colsum(grad_output.reshape(-1, grad_output.shape[-1])).to(ctx.bias_dtype)
        return grad_input, grad_weight, grad_bias


def zero3_linear_wrap(input, weight, bias=None):
    return LinearFunctionForZeroStage3.apply(input, weight, bias)


class LinearModuleForZeroStage3(torch.nn.Linear):
    """nn.Linear with the ZeRO-3-friendly autograd function above."""

    def forward(self, input):
        return LinearFunctionForZeroStage3.apply(input, self.weight, self.bias)
