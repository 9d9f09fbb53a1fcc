"""Side-stream prefetch of the dgrad weight transposes (ops/linear.py WeightTPrefetch): from the
second backward on, W^T of the next linear is made on a side stream while the current one's GEMMs
run.  Gradients must be bit-identical to just-in-time transposes, through activation checkpointing
(recompute inside backward) and gradient accumulation."""

import os

import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(prefetch, steps=3):
    from deeperspeed_amd.models.gpt_neox import GPTNeoX, get_config
    from deeperspeed_amd.ops import linear
    linear.WT_PREFETCH = prefetch
    linear._wt_prefetch = linear.WeightTPrefetch()
    torch.manual_seed(0)
    dev = torch.device("cuda")
    cfg = get_config("gpt-neox-125m", hidden_size=1024, num_heads=8, num_layers=3, max_seq_len=512,
                     checkpoint_activations=True)
    m = GPTNeoX(cfg, device=dev, dtype=torch.bfloat16).train()
    g = torch.Generator(device=dev).manual_seed(1)
    for _ in range(steps):
        ids = torch.randint(0, cfg.vocab_size, (2, 512), device=dev, generator=g)
        m(ids, labels=ids).backward()
        linear.end_backward_pass()
    torch.cuda.synchronize()
    return [p.grad.clone() for p in m.parameters()], linear._wt_prefetch.hits


def test_prefetched_weight_transposes_are_exact():
    ref, hits0 = _run(False)
    got, hits = _run(True)
    assert hits0 == 0 and hits > 0
    for a, b in zip(ref, got):
        assert torch.equal(a, b)
