"""Fused bias + dropout + residual + LayerNorm (ops/csrc/kernels/dropout.hip bdr_ln_*) against a
plain fp32 PyTorch reference of the same op (same keep mask), against the two-kernel path it
replaces, and the layer-to-layer LayerNorm hand-over of a BERT encoder (chain_layer_norms)."""

import pytest
import torch

from deeperspeed_amd.ops import native
from deeperspeed_amd.ops.transformer import DeepSpeedTransformerConfig, DeepSpeedTransformerLayer
from deeperspeed_amd.ops.transformer.transformer import chain_layer_norms, take_chained_norm

pytestmark = pytest.mark.gpu


def _inputs(rows, H, dtype=torch.bfloat16, seed=0):
    g = torch.Generator().manual_seed(seed)
    dev = torch.device("cuda")
    mk = lambda *s, sc=1.0: (torch.randn(*s, generator=g) * sc).to(dev, dtype)
    return mk(rows, H), mk(H, sc=0.1), mk(rows, H), (1 + mk(H, sc=0.1)), mk(H, sc=0.1)


@pytest.mark.parametrize("H", [1024, 768, 256])
def test_bdr_ln_matches_fp32_reference(H):
    rows, p, eps = 1000, 0.1, 1e-12
    x, b, r, gm, bt = _inputs(rows, H)
    y, out, mask, mean, rstd = native.hip_ops().bdr_ln_fwd(x, b, r, gm, bt, p, eps, 1234, 0, None)
    keep = mask.float()
    assert abs(1 - keep.mean().item() - p) < 0.01
    # fp32 reference with the kernel's keep mask
    xf, bf, rf, gf, btf = (t.float().requires_grad_(True) for t in (x, b, r, gm, bt))
    of = rf + (xf + bf) * keep / (1 - p)
    yf = torch.nn.functional.layer_norm(of, (H,), gf, btf, eps)
    assert (out.float() - of).abs().max().item() <= 2e-2 * of.abs().max().item()
    assert (y.float() - yf).abs().max().item() <= 3e-2 * yf.abs().max().item()
    # backward: dy into y, dres into out (the residual path's gradient)
    g = torch.Generator().manual_seed(9)
    dy = torch.randn(rows, H, generator=g).cuda().to(x.dtype)
    dres = torch.randn(rows, H, generator=g).cuda().to(x.dtype)
    (yf * dy.float()).sum().add_((of * dres.float()).sum()).backward()
    dtot, dxb, dg, dbt, dbias = native.hip_ops().bdr_ln_bwd(dy, out, gm, mean, rstd, True, dres, mask, p)
    for got, ref in ((dtot, rf.grad), (dxb, xf.grad), (dg, gf.grad), (dbt, btf.grad), (dbias, bf.grad)):
        scale = ref.abs().max().item()
        assert (got.float() - ref).abs().max().item() <= 3e-2 * scale, (got, ref)


def test_bdr_ln_same_as_unfused_path():
    """Fused autograd op vs bias_dropout_residual + layer_norm_residual: same masks and values."""
    rows, H, p, eps = 512, 1024, 0.1, 1e-5
    x, b, r, gm, bt = _inputs(rows, H, seed=3)
    res = []
    for fused in (True, False):
        ts = [t.clone().requires_grad_(True) for t in (x, b, r, gm, bt)]
        gen = torch.Generator().manual_seed(77)
        if fused:
            y, out = native.bias_dropout_residual_ln(ts[0], ts[1], ts[2], ts[3], ts[4], eps, p, True, gen)
        else:
            o = native.bias_dropout_residual(ts[0], ts[1], ts[2], p, True, gen)
            y, out = native.layer_norm_residual(o, ts[3], ts[4], eps)
        (y.float().pow(2).sum() + out.float().sum()).backward()
        res.append([y.detach(), out.detach()] + [t.grad for t in ts])
    assert torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1])
    for a, c in zip(res[0][2:], res[1][2:]):
        assert (a.float() - c.float()).abs().max().item() <= 1e-2 * max(1.0, c.float().abs().max().item())


def _encoder(n, H, dev):
    cfg = DeepSpeedTransformerConfig(batch_size=4, hidden_size=H, heads=H // 64, attn_dropout_ratio=0.1,
                                     hidden_dropout_ratio=0.1, num_hidden_layers=n, initializer_range=0.02,
                                     seed=11, pre_layer_norm=True, layer_norm_eps=1e-12, bf16=True)
    torch.manual_seed(5)
    DeepSpeedTransformerLayer.layer_id = 0
    import copy
    layers = torch.nn.ModuleList([DeepSpeedTransformerLayer(copy.copy(cfg)) for _ in range(n)]).to(dev).train()
    final = native.FusedLayerNorm(H, 1e-12).to(dev, torch.bfloat16)
    return layers, final


def test_chained_layer_norms_match_unchained():
    dev = torch.device("cuda")
    B, S, H = 4, 128, 256
    outs = []
    for chain in (False, True):
        layers, final = _encoder(3, H, dev)
        x = torch.randn(B, S, H, generator=torch.Generator().manual_seed(7)).to(dev, torch.bfloat16)
        x.requires_grad_(True)
        chain_layer_norms(layers, final if chain else None)
        if not chain:
            for l in layers:
                object.__setattr__(l, "_dsa_next_norm", None)
        h = x
        for l in layers:
            h = l(h, None)
        y = take_chained_norm(h, final)
        if chain:
            assert y is not None
        y = final(h) if y is None else y
        y.float().pow(2).sum().backward()
        outs.append([y.detach().float(), x.grad.float()] + [p.grad.float() for p in layers.parameters()]
                    + [p.grad.float() for p in final.parameters()])
    for a, c in zip(*outs):
        assert (a - c).abs().max().item() <= 2e-2 * max(1.0, c.abs().max().item())
