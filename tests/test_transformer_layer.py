"""DeepSpeedTransformerLayer (reference tests/unit/test_cuda_forward.py / test_cuda_backward.py):
equivalence with a HuggingFace BertLayer (post-LN) and a hand-written pre-LN layer, forward and
backward, module_inject round trip, dropout reproducibility."""

import copy

import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from deeperspeed_amd.module_inject import replace_transformer_layer, revert_transformer_layer
from deeperspeed_amd.ops.transformer import DeepSpeedTransformerConfig, DeepSpeedTransformerLayer

transformers = pytest.importorskip("transformers")
from transformers.models.bert.modeling_bert import BertConfig, BertLayer  # noqa: E402


def _hf_config():
    return BertConfig(hidden_size=64, num_attention_heads=4, intermediate_size=256, hidden_act="gelu_new",
                      hidden_dropout_prob=0.1, attention_probs_dropout_prob=0.1, num_hidden_layers=2,
                      initializer_range=0.02, layer_norm_eps=1e-12, attn_implementation="eager")


class _Wrap(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.layer = BertLayer(cfg)


def _mask(B, S):
    m = torch.ones(B, S)
    m[0, -5:] = 0
    return ((1.0 - m) * -10000.0)[:, None, None, :]


def test_postln_matches_huggingface_fwd_bwd():
    torch.manual_seed(0)
    cfg = _hf_config()
    hf = _Wrap(cfg).eval()
    ds = replace_transformer_layer(BertLayer, copy.deepcopy(hf), micro_batch_size=2, bert_config=cfg, seed=1,
                                   preln=False, fp16=False, training=False).eval()
    assert isinstance(ds.layer, DeepSpeedTransformerLayer)
    x = torch.randn(2, 24, 64, requires_grad=True)
    x2 = x.detach().clone().requires_grad_(True)
    m = _mask(2, 24)
    r = hf.layer(x, attention_mask=m)
    ref = r[0] if isinstance(r, tuple) else r
    out = ds.layer(x2, m)
    torch.testing.assert_close(out, ref, atol=1e-4, rtol=1e-4)
    g = torch.randn_like(ref)
    ref.backward(g)
    out.backward(g)
    torch.testing.assert_close(x2.grad, x.grad, atol=1e-4, rtol=1e-3)
    torch.testing.assert_close(ds.layer.inter_w.grad, hf.layer.intermediate.dense.weight.grad, atol=1e-4, rtol=1e-3)
    q, k, v = ds.layer.attn_qkvw.grad.split(64, 0)
    torch.testing.assert_close(k, hf.layer.attention.self.key.weight.grad, atol=1e-4, rtol=1e-3)
    back = revert_transformer_layer(BertLayer, ds, cfg, preln=False)
    for (n1, p1), (n2, p2) in zip(hf.named_parameters(), back.named_parameters()):
        assert n1 == n2 and torch.equal(p1, p2), n1


def _preln_reference(layer, x, m):
    c = layer.config
    H, nh = c.hidden_size, c.heads
    B, S, _ = x.shape
    h = F.layer_norm(x, (H,), layer.norm_w, layer.norm_b, c.layer_norm_eps)
    q, k, v = F.linear(h, layer.attn_qkvw, layer.attn_qkvb).view(B, S, 3, nh, H // nh).permute(2, 0, 3, 1, 4)
    p = torch.softmax(q @ k.transpose(-1, -2) / (H // nh) ** 0.5 + m, -1)
    ctx = (p @ v).transpose(1, 2).reshape(B, S, H)
    a = x + F.linear(ctx, layer.attn_ow, layer.attn_ob)
    h2 = F.layer_norm(a, (H,), layer.attn_nw, layer.attn_nb, c.layer_norm_eps)
    f = F.gelu(F.linear(h2, layer.inter_w, layer.inter_b), approximate="tanh")
    return a + F.linear(f, layer.output_w, layer.output_b)


def test_preln_matches_reference_math():
    torch.manual_seed(0)
    cfg = DeepSpeedTransformerConfig(batch_size=2, hidden_size=64, heads=4, attn_dropout_ratio=0.1,
                                     hidden_dropout_ratio=0.1, num_hidden_layers=2, initializer_range=0.02,
                                     pre_layer_norm=True, training=False)
    layer = DeepSpeedTransformerLayer(cfg).eval()
    with torch.no_grad():
        for p in layer.parameters():
            p.add_(0.05 * torch.randn_like(p))
    x = torch.randn(2, 16, 64)
    m = _mask(2, 16)
    torch.testing.assert_close(layer(x, m), _preln_reference(layer, x, m), atol=1e-4, rtol=1e-4)


def test_dropout_training_reproducible():
    cfg = DeepSpeedTransformerConfig(batch_size=2, hidden_size=64, heads=4, attn_dropout_ratio=0.2,
                                     hidden_dropout_ratio=0.2, num_hidden_layers=2, initializer_range=0.02, seed=7)
    torch.manual_seed(0)
    a = DeepSpeedTransformerLayer(cfg).train()
    b = copy.deepcopy(a)
    b._generator = torch.Generator().manual_seed(cfg.seed + a.config.layer_id)
    a._generator = torch.Generator().manual_seed(cfg.seed + a.config.layer_id)
    x = torch.randn(2, 16, 64)
    ya, yb = a(x), b(x)
    assert torch.equal(ya, yb)
    assert not torch.allclose(ya, a.eval()(x))


def _saved_bytes(fn):
    """Bytes of distinct storages autograd saves while running fn()."""
    seen = {}

    def pack(t):
        seen[t.untyped_storage().data_ptr()] = t.untyped_storage().nbytes()
        return t

    with torch.autograd.graph.saved_tensors_hooks(pack, lambda t: t):
        out = fn()
    return out, sum(seen.values())


@pytest.mark.parametrize("pre_ln", [True, False])
def test_memory_modes_same_gradients_less_saved(pre_ln):
    """normalize_invertible + attn_dropout_checkpoint (reference ds_transformer_cuda.cpp:185-193):
    identical forward / gradients (same dropout masks), fewer bytes held for backward."""
    torch.manual_seed(3)
    B, S, H = 2, 16, 64
    outs = {}
    for flags in (False, True):
        cfg = DeepSpeedTransformerConfig(batch_size=B, hidden_size=H, heads=4, attn_dropout_ratio=0.1,
                                         hidden_dropout_ratio=0.1, num_hidden_layers=2, initializer_range=0.02,
                                         seed=11, pre_layer_norm=pre_ln, normalize_invertible=flags,
                                         attn_dropout_checkpoint=flags, layer_norm_eps=1e-12)
        torch.manual_seed(5)
        DeepSpeedTransformerLayer.layer_id = 0  # same per-layer dropout seed stream in both runs
        layer = DeepSpeedTransformerLayer(cfg).train()
        x = torch.randn(B, S, H, requires_grad=True, generator=torch.Generator().manual_seed(7))
        y, nbytes = _saved_bytes(lambda: layer(x, _mask(B, S)))
        y.sum().backward()
        outs[flags] = (y.detach(), x.grad.clone(), {n: p.grad.clone() for n, p in layer.named_parameters()},
                       nbytes)
    (y0, gx0, gp0, b0), (y1, gx1, gp1, b1) = outs[False], outs[True]
    assert torch.allclose(y0, y1, atol=1e-6)
    assert torch.allclose(gx0, gx1, atol=1e-4, rtol=1e-3)
    for n in gp0:
        assert torch.allclose(gp0[n], gp1[n], atol=1e-4, rtol=1e-3), n
    assert b1 < b0, (b0, b1)


@pytest.mark.gpu
def test_memory_modes_gpu_kernels(monkeypatch):
    """Same equivalence on the HIP kernels (bf16): invertible LayerNorm backward through the
    fused LN-backward kernel, dropout mask re-applied with the dropout-backward kernel (the
    materialised attention path, so the encoder flash kernel is switched off here)."""
    from deeperspeed_amd.ops.transformer import transformer as tmod
    monkeypatch.setattr(tmod, "_ENCODER_FLASH", False)
    torch.manual_seed(3)
    B, S, H = 4, 64, 256
    dev = torch.device("cuda")
    res = {}
    for flags in (False, True):
        cfg = DeepSpeedTransformerConfig(batch_size=B, hidden_size=H, heads=4, attn_dropout_ratio=0.1,
                                         hidden_dropout_ratio=0.1, num_hidden_layers=2, initializer_range=0.02,
                                         seed=11, pre_layer_norm=True, normalize_invertible=flags,
                                         attn_dropout_checkpoint=flags, layer_norm_eps=1e-12, bf16=True)
        torch.manual_seed(5)
        DeepSpeedTransformerLayer.layer_id = 0
        layer = DeepSpeedTransformerLayer(cfg).to(dev).train()
        x = torch.randn(B, S, H, generator=torch.Generator().manual_seed(7)).to(dev, torch.bfloat16).requires_grad_(True)
        y = layer(x, _mask(B, S).to(dev, torch.bfloat16))
        y.float().sum().backward()
        res[flags] = (y.detach().float(), x.grad.float(), layer.attn_qkvw.grad.float(), layer.norm_w.grad.float())
    for a, b in zip(res[False], res[True]):
        assert (a - b).abs().max().item() <= 3e-2 * max(1.0, a.abs().max().item())


@pytest.mark.gpu
@pytest.mark.parametrize("pre_ln", [True, False])
def test_encoder_flash_matches_materialised_path(monkeypatch, pre_ln):
    """Without attention dropout the fused encoder flash path (key-padding bias in the kernel,
    token-major output) gives the materialised softmax path's outputs and gradients."""
    from deeperspeed_amd.ops.transformer import transformer as tmod
    B, S, H = 4, 128, 512
    dev = torch.device("cuda")
    res = {}
    for flash in (False, True):
        monkeypatch.setattr(tmod, "_ENCODER_FLASH", flash)
        cfg = DeepSpeedTransformerConfig(batch_size=B, hidden_size=H, heads=8, attn_dropout_ratio=0.0,
                                         hidden_dropout_ratio=0.0, num_hidden_layers=2, initializer_range=0.02,
                                         seed=11, pre_layer_norm=pre_ln, layer_norm_eps=1e-12, bf16=True)
        torch.manual_seed(5)
        DeepSpeedTransformerLayer.layer_id = 0
        layer = DeepSpeedTransformerLayer(cfg).to(dev).train()
        x = torch.randn(B, S, H, generator=torch.Generator().manual_seed(7)).to(dev, torch.bfloat16).requires_grad_(True)
        y = layer(x, _mask(B, S).to(dev, torch.bfloat16))
        y.float().pow(2).sum().backward()
        res[flash] = (y.detach().float(), x.grad.float(), layer.attn_qkvw.grad.float(), layer.attn_ow.grad.float())
    for a, b in zip(res[False], res[True]):  # bf16 activations: a few ulp of the largest entry
        assert (a - b).abs().max().item() <= 5e-2 * max(1.0, a.abs().max().item())


def test_encoder_flash_keep_mask_statistics():
    """The in-kernel attention-dropout mask (counter hash of seed, head, query, key): drop rate
    matches p, heads and seeds give different masks, neighbouring keys are uncorrelated."""
    from deeperspeed_amd.ops import native
    keep = native.flash_dropout_keep_mask(2, 4, 256, 0.1, 99)
    assert keep.shape == (2, 4, 256, 256)
    assert abs(1.0 - keep.float().mean().item() - 0.1) < 0.005
    assert not torch.equal(keep[0, 0], keep[0, 1]) and not torch.equal(keep[0, 0], keep[1, 0])
    assert not torch.equal(keep, native.flash_dropout_keep_mask(2, 4, 256, 0.1, 100))
    d = (~keep).float()
    both = (d[..., 0::2] * d[..., 1::2]).mean().item()  # the two halves of one hash
    assert abs(both - 0.01) < 0.003
    assert native.flash_dropout_keep_mask(1, 1, 64, 0.0, 5).all()


def test_layer_norm_residual_passthrough_gradients():
    """(LN(x), x) with the residual gradient summed in the LN backward equals LN(x) + separate
    residual use of x (CPU reference path of native.layer_norm_residual)."""
    from deeperspeed_amd.ops import native
    torch.manual_seed(0)
    x = torch.randn(6, 10, 32, dtype=torch.float32)
    w = torch.randn(32, dtype=torch.float32) * 0.1 + 1
    b = torch.randn(32, dtype=torch.float32) * 0.1
    gy, gr = torch.randn(6, 10, 32, dtype=torch.float32), torch.randn(6, 10, 32, dtype=torch.float32)
    res = []
    for fused in (True, False):
        xi, wi, bi = (t.clone().requires_grad_(True) for t in (x, w, b))
        if fused:
            y, xr = native.layer_norm_residual(xi, wi, bi, 1e-5)
        else:
            y, xr = torch.nn.functional.layer_norm(xi, (32,), wi, bi, 1e-5), xi
        ((y * gy).sum() + (xr * gr).sum()).backward()
        res.append((y.detach(), xi.grad, wi.grad, bi.grad))
    for a, c in zip(*res):
        assert torch.allclose(a, c, atol=1e-4, rtol=1e-4)


def test_device_rng_advances_once_per_checkpointed_forward():
    """Device-RNG dropout step under activation checkpointing: the first (no_grad)
    forward of the checkpoint advances the step, the recompute inside backward does not (it
    must redraw the same masks) -- so two checkpointed training steps use two different steps."""
    from deeperspeed_amd.runtime.activation_checkpointing import checkpointing as ckpt
    torch.manual_seed(0)
    cfg = DeepSpeedTransformerConfig(batch_size=2, hidden_size=64, intermediate_size=256, heads=4,
                                     attn_dropout_ratio=0.1, hidden_dropout_ratio=0.1, num_hidden_layers=1,
                                     initializer_range=0.02, pre_layer_norm=True, training=True)
    layer = DeepSpeedTransformerLayer(cfg).train()
    layer.enable_device_rng(11)
    x = torch.randn(2, 16, 64, requires_grad=True)
    m = torch.zeros(2, 1, 1, 16)
    for step in (1, 2):
        out = ckpt.checkpoint(lambda h: layer(h, m), x)
        assert int(layer._rng[1]) == step
        out.sum().backward()
        assert int(layer._rng[1]) == step  # the recompute did not advance it
    layer(x, m)  # plain (non-checkpointed) training forward
    assert int(layer._rng[1]) == 3
