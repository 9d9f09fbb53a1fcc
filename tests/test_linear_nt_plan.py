"""Planning predicate of the reduction-contiguous weight-gradient path (ops/linear.py): producers
of pre-transposed operands (the dual-output GeLU backward, the shared block-output gradient)
only offer one when the consuming weight gradient will take that path."""

import torch

from deeperspeed_amd.ops import linear as lin


def test_nt_wgrad_planned_shapes():
    # GPT-NeoX-20B at 8192 / 16384 tokens: every projection takes the transposed path
    for M in (8192, 16384):
        for out, inp in ((18432, 6144), (6144, 6144), (24576, 6144), (6144, 24576)):
            assert lin.nt_wgrad_planned(M, out, inp, g_ready=(out == 24576)), (M, out, inp)
    # BERT-Large weights have few 256x256 output tiles: split-K instead
    assert not lin.nt_wgrad_planned(8192, 4096, 1024)
    assert not lin.nt_wgrad_planned(8192, 1024, 1024)
    # below the size threshold: plain GEMM
    assert not lin.nt_wgrad_planned(256, 384, 384)
    # transient copies beyond the byte cap, unless the big operand is already transposed
    assert not lin.nt_wgrad_planned(16384, 32768, 8192)
    assert lin.nt_wgrad_planned(16384, 32768, 8192, g_ready=True)


def test_transposed_registry_fifo_and_match():
    lin.clear_transposed()
    a = torch.zeros(4, 8)
    b = torch.zeros(4, 8)
    c = torch.zeros(4, 8)
    lin.offer_transposed(a, a.t().contiguous())
    lin.offer_transposed(b, b.t().contiguous())
    lin.offer_transposed(c, c.t().contiguous())  # oldest entry (a) evicted
    assert lin._take_transposed(a) is None
    assert lin._take_transposed(b) is not None
    assert lin._take_transposed(b) is None  # consumed once
    assert lin._take_transposed(torch.zeros(8, 4)) is None  # shape mismatch never matches
    assert lin._take_transposed(c) is not None
    lin.clear_transposed()
