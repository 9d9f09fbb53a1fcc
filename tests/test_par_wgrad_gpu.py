"""Input / weight gradients of small linears on two streams (ops/linear.py `_linear_backward`):
bit-identical to the serial order for a BERT-Large encoder (split-K weight gradients, bound
gradients accumulated in place, bias gradients)."""

import pytest
import torch

pytestmark = pytest.mark.gpu


def _grads(par):
    from deeperspeed_amd.models.bert import BertForPreTraining, get_config
    from deeperspeed_amd.ops import linear
    linear.PAR_WGRAD = par  # opt-in path (default off); pinned exact here
    torch.manual_seed(0)
    dev = torch.device("cuda")
    cfg = get_config("bert-large", num_layers=2, vocab_size=4096, max_position=128, hidden_dropout=0.0,
                     attn_dropout=0.0)
    m = BertForPreTraining(cfg, device=dev, dtype=torch.bfloat16).train()
    g = torch.Generator(device=dev).manual_seed(1)
    B, S, npred = 32, 128, 20
    before = linear._par_count[0]
    for _ in range(2):  # second pass accumulates into the gradients of the first
        ids = torch.randint(0, cfg.vocab_size, (B, S), device=dev, generator=g)
        tt = torch.zeros(B, S, dtype=torch.long, device=dev)
        am = torch.ones(B, S, dtype=torch.long, device=dev)
        pos = torch.stack([torch.randperm(S, device=dev, generator=g)[:npred].sort().values for _ in range(B)])
        lab = torch.randint(0, cfg.vocab_size, (B, npred), device=dev, generator=g)
        nsp = torch.randint(0, 2, (B,), device=dev, generator=g)
        m(ids, tt, am, pos, lab, nsp).backward()
    torch.cuda.synchronize()
    linear.PAR_WGRAD = False
    return [p.grad.clone() for p in m.parameters() if p.grad is not None], linear._par_count[0] - before


def test_parallel_dgrad_wgrad_is_exact():
    ref, n0 = _grads(False)
    got, n1 = _grads(True)
    assert n0 == 0 and n1 > 0
    assert len(ref) == len(got)
    for a, b in zip(ref, got):
        assert torch.equal(a, b)
