"""Compact fp32 master weights: an exact fp32 master stored as (bf16 weight, int16 residual).

MI355X-specific memory layout (no reference counterpart; the reference keeps a separate
fp32 copy, deepspeed/runtime/zero/stage2.py:single_partition_of_fp32_groups).  For a bf16
model the high 16 bits of every fp32 master value, rounded half-away on the magnitude, ARE
the bf16 model weight, so only a 16-bit signed residual has to be stored next to it:

    bits(master) = (bits(bf16) << 16) + residual,   residual in [-32768, 32767]

The reconstruction is exact (integer arithmetic on the IEEE bit pattern, valid across
exponent boundaries), so the optimizer math is bit-identical fp32 Adam; the only difference
from a separate master is that the bf16 weights are rounded half-away instead of
half-to-even (they differ on exact ties only).  Cost: 2 B/param instead of 4 B, which lets a
20B-parameter model keep weights + grads + fp32 master + moments (14 B/param) inside one
288 GiB MI355X without offloading anything over PCIe.
"""

import torch


def encode(master: torch.Tensor):
    """fp32 -> (bf16 high half, int16 residual)."""
    bits = master.contiguous().float().view(torch.int32)
    hi = torch.bitwise_right_shift(bits + 0x8000, 16)  # arithmetic shift keeps the sign bits
    res = (bits - torch.bitwise_left_shift(hi, 16)).to(torch.int16)
    return hi.to(torch.int16).view(torch.bfloat16), res


def decode(hi: torch.Tensor, res: torch.Tensor) -> torch.Tensor:
    """(bf16 high half, int16 residual) -> exact fp32."""
    h = hi.contiguous().view(torch.int16).to(torch.int32)
    return (torch.bitwise_left_shift(h, 16) + res.to(torch.int32)).view(torch.float32)


def decode_chunked(hi: torch.Tensor, res: torch.Tensor, out: torch.Tensor, chunk: int = 1 << 26):
    """Decode into `out` (any device) without materialising a full-size int32 temporary."""
    n = hi.numel()
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        out[s:e].copy_(decode(hi[s:e], res[s:e]))
    return out


def encode_into(master: torch.Tensor, hi_out: torch.Tensor, res_out: torch.Tensor, chunk: int = 1 << 26):
    """Encode fp32 `master` (any device) into existing bf16 / int16 buffers."""
    n = master.numel()
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        h, r = encode(master[s:e].to(hi_out.device))
        hi_out[s:e].copy_(h)
        res_out[s:e].copy_(r)
