"""TiledLinear: split a large linear layer into a grid of smaller ones.

Reference parity: deepspeed/runtime/zero/tiling.py:26-294 (`TiledLinear`,
`TiledLinearReturnBias`).  With ZeRO-3 every tile is its own module and therefore its own
gather unit, so only one [out/out_splits, in/in_splits] tile is materialised at a time instead
of the whole weight (useful for very wide projections such as vocabulary heads).
"""

import copy

import torch
import torch.nn as nn


def split_tensor_along_last_dim(tensor, partitions, contiguous_split_chunks=False):
    """Split `tensor` on its last dim into pieces of the given sizes."""
    chunks = torch.split(tensor, partitions, dim=-1)
    return tuple(c.contiguous() for c in chunks) if contiguous_split_chunks else chunks


def partition_sizes(total, num_parts):
    base, rem = divmod(total, num_parts)
    return [base + (1 if i < rem else 0) for i in range(num_parts)]


class TiledLinear(nn.Module):
    def __init__(self, in_features, out_features, bias=True, in_splits=1, out_splits=1,
                 input_is_already_split=False, combine_out_splits=True, linear_cls=nn.Linear, init_linear=None,
                 **kwargs):
        super().__init__()
        if in_splits < 1 or in_splits > in_features:
            raise RuntimeError("in splits must be in range [1, in_features].")
        if out_splits < 1 or out_splits > out_features:
            raise RuntimeError("out splits must be in range [1, out_features].")
        self.in_features, self.out_features = in_features, out_features
        self.use_bias = bias
        self.out_splits, self.in_splits = out_splits, in_splits
        self.input_is_already_split = input_is_already_split
        self.combine_out_splits = combine_out_splits
        self.in_parts = partition_sizes(in_features, in_splits)
        self.out_parts = partition_sizes(out_features, out_splits)
        # bias lives only in the in-split-0 column of tiles so it is added once
        self.linears = nn.ModuleList()
        for out_id in range(out_splits):
            row = nn.ModuleList()
            for in_id in range(in_splits):
                row.append(linear_cls(self.in_parts[in_id], self.out_parts[out_id], bias=(bias and in_id == 0),
                                      **kwargs))
            self.linears.append(row)
        if init_linear is not None:
            self.copy_params_from(init_linear)

    def forward(self, input_):
        if self.in_splits > 1 and not self.input_is_already_split:
            inputs = split_tensor_along_last_dim(input_, self.in_parts)
        elif self.in_splits > 1:
            inputs = input_
            assert len(inputs) == self.in_splits, f"expected {self.in_splits} input splits, got {len(inputs)}"
        else:
            inputs = [input_]
        outputs = []
        for out_id in range(self.out_splits):
            acc = None
            for in_id in range(self.in_splits):
                y = self.linears[out_id][in_id](inputs[in_id])
                acc = y if acc is None else acc + y
            outputs.append(acc)
        if self.combine_out_splits:
            return torch.cat(outputs, dim=-1)
        return outputs

    @torch.no_grad()
    def copy_params_from(self, other):
        """Copy weights (and bias) of a dense `other` linear into the tiles."""
        assert other.weight.shape == (self.out_features, self.in_features)
        o0 = 0
        for out_id in range(self.out_splits):
            i0 = 0
            for in_id in range(self.in_splits):
                lin = self.linears[out_id][in_id]
                oh, ih = self.out_parts[out_id], self.in_parts[in_id]
                lin.weight.copy_(other.weight[o0:o0 + oh, i0:i0 + ih])
                if in_id == 0 and self.use_bias and other.bias is not None:
                    lin.bias.copy_(other.bias[o0:o0 + oh])
                i0 += ih
            o0 += oh


class TiledLinearReturnBias(TiledLinear):
    """TiledLinear for layers that return (output, bias) (Megatron style): tiles are built
    without bias add in forward; the combined bias is returned separately."""

    def forward(self, input_):
        if self.in_splits > 1 and not self.input_is_already_split:
            inputs = split_tensor_along_last_dim(input_, self.in_parts)
        elif self.in_splits > 1:
            inputs = input_
        else:
            inputs = [input_]
        outputs, biases = [], []
        for out_id in range(self.out_splits):
            acc = None
            for in_id in range(self.in_splits):
                lin = self.linears[out_id][in_id]
                y = torch.nn.functional.linear(inputs[in_id], lin.weight)
                acc = y if acc is None else acc + y
                if lin.bias is not None:
                    biases.append(lin.bias)
            outputs.append(acc)
        bias = torch.cat(biases) if biases else None
        if self.combine_out_splits:
            return torch.cat(outputs, dim=-1), bias
        return outputs, bias
