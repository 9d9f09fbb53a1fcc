"""Block-sparse flash attention (ops/sparse_attention/flash.py + flash_attn.hip sfwd / sdkdv / sdq).

CPU: the LUT builder against a brute-force walk of the layout (tile activity, sub-block
bitmasks, CSR order, transposed LUT, causal tile drop).
GPU: output and q/k/v gradients against an fp32 PyTorch reference of the same op (dense
scores masked by the element-expanded layout [+ causal], softmax, P V) for blocks 16 / 32 /
64 / 128, head dims 64 / 96 / 128, bf16 and fp16, shared and per-head layouts.
"""

import random

import numpy as np
import pytest
import torch

from deeperspeed_amd.ops.sparse_attention.flash import SparseFlashLUT


def _rand_layout(H, nb, density, seed, lower=False):
    g = torch.Generator().manual_seed(seed)
    lay = (torch.rand(H, nb, nb, generator=g) < density).long()
    for h in range(H):
        lay[h].fill_diagonal_(1)
    if lower:
        lay = torch.tril(lay)
    return lay


@pytest.mark.parametrize("block,causal", [(16, False), (32, True), (64, False), (128, True)])
def test_lut_matches_bruteforce(block, causal):
    S, H = 512, 3
    lay = _rand_layout(H, S // block, 0.3, 1)
    lut = SparseFlashLUT(lay, block, causal=causal)
    rp, cols, masks, cp, rows, masks_t = lut._host[:6]
    nt = S // 64
    r = max(1, 64 // block)
    for h in range(H):
        fwd = []
        for i in range(nt):
            for j in range(nt):
                if causal and j > i:
                    continue
                bits = 0
                for qs in range(r):
                    for ks in range(r):
                        qb = (i * 64 + qs * block) // block if block < 64 else (i * 64) // block
                        kb = (j * 64 + ks * block) // block if block < 64 else (j * 64) // block
                        if lay[h, qb, kb]:
                            bits |= 1 << (qs * r + ks)
                if bits:
                    fwd.append((i, j, bits))
        got = [(i, int(cols[e]), int(masks[e]) & 0xffffffff) for i in range(nt)
               for e in range(rp[h * nt + i], rp[h * nt + i + 1])]
        assert got == fwd
        got_t = sorted((int(rows[e]), j, int(masks_t[e]) & 0xffffffff) for j in range(nt)
                       for e in range(cp[h * nt + j], cp[h * nt + j + 1]))
        assert got_t == sorted(fwd)


def test_dkdv_tasks_cover_transposed_lut():
    """Key tiles with more than CHUNK query tiles (global columns) are split into chunks whose
    partial slots are summed by the finish pass; every entry is covered exactly once."""
    S = 2048
    lay = torch.zeros(2, S // 64, S // 64, dtype=torch.long)
    lay[:, :, 0] = 1  # global column
    for i in range(S // 64):
        lay[:, i, max(0, i - 2): i + 1] = 1
    lay[1, :, 5] = 1
    lut = SparseFlashLUT(lay, 64, causal=True)
    rp, cols, masks, cp, rows, masks_t, tasks, fin = lut._host
    nt = S // 64
    for h in range(2):
        seen = []
        for kt, e0, e1, slot in tasks[h]:
            if kt < 0:
                continue
            assert e1 - e0 <= lut.CHUNK
            seen += list(range(e0, e1))
            assert cp[h * nt + kt] <= e0 < e1 <= cp[h * nt + kt + 1]
        assert sorted(seen) == list(range(cp[h * nt], cp[h * nt + nt]))
        heavy = [f for f in fin[h] if f[0] >= 0]
        assert heavy and heavy[0][0] == 0 and heavy[0][2] == -(-nt // lut.CHUNK)
    assert lut.nslot >= max(int(fin[h][:, 2].clip(min=0).sum()) for h in range(2))


def test_lut_shared_heads_dedup():
    lay = _rand_layout(1, 8, 0.4, 2).repeat(4, 1, 1)
    assert SparseFlashLUT(lay, 64).heads == 1
    lay[2, 0, 5] = 1 - lay[2, 0, 5]
    assert SparseFlashLUT(lay, 64).heads == 4


def _reference(q, k, v, lay, block, causal, scale):
    S = q.shape[2]
    m = lay.bool().repeat_interleave(block, 1).repeat_interleave(block, 2)[:, :S, :S].to(q.device)
    if m.shape[0] == 1:
        m = m.expand(q.shape[1], S, S)
    if causal:
        m = m & torch.tril(torch.ones(S, S, dtype=torch.bool, device=q.device))
    s = (q.float() @ k.float().transpose(-1, -2)) * scale
    s = s.masked_fill(~m[None], float("-inf"))
    p = torch.softmax(s, dim=-1).nan_to_num(0.0)
    return p @ v.float()


@pytest.mark.gpu
@pytest.mark.parametrize("block,causal,D,dtype,per_head", [
    (16, False, 64, torch.bfloat16, False), (32, True, 96, torch.bfloat16, True),
    (64, True, 96, torch.bfloat16, True), (64, False, 128, torch.float16, False),
    (128, True, 64, torch.float16, True), (16, True, 128, torch.bfloat16, True)])
def test_sparse_flash_matches_reference(block, causal, D, dtype, per_head):
    from deeperspeed_amd.ops.sparse_attention.flash import sparse_flash_attention, supported
    torch.manual_seed(0)
    B, H, S = 2, 4, 512
    lay = _rand_layout(H if per_head else 1, S // block, 0.35, 3, lower=causal)
    lut = SparseFlashLUT(lay, block, causal=causal)
    dev = torch.device("cuda")
    q, k, v = (torch.randn(B, H, S, D, device=dev, dtype=dtype, requires_grad=True) for _ in range(3))
    assert supported(q, lut)
    scale = D ** -0.5
    o = sparse_flash_attention(q, k, v, lut, scale)
    g = torch.randn_like(o)
    o.backward(g)
    qr, kr, vr = (t.detach().float().requires_grad_(True) for t in (q, k, v))
    ref = _reference(qr, kr, vr, lay, block, causal, scale)
    ref.backward(g.float())
    tol = 2e-2 if dtype == torch.bfloat16 else 5e-3
    assert (o.float() - ref).abs().max().item() < tol * max(1.0, ref.abs().max().item())
    for a, b in ((q.grad, qr.grad), (k.grad, kr.grad), (v.grad, vr.grad)):
        err = (a.float() - b).abs().max().item()
        assert err < 4 * tol * max(1.0, b.abs().max().item()), err


@pytest.mark.gpu
def test_sparse_flash_bshd_output_and_bigbird():
    """NeoX usage: BigBird layout, pre-scaled q, causal, token-major output."""
    from deeperspeed_amd.ops.sparse_attention.flash import sparse_flash_attention
    from deeperspeed_amd.ops.sparse_attention.sparsity_config import BigBirdSparsityConfig
    random.seed(0)
    torch.manual_seed(1)
    B, H, S, D = 1, 4, 1024, 96
    cfg = BigBirdSparsityConfig(num_heads=H, block=64, different_layout_per_head=True, attention="unidirectional")
    lay = cfg.make_layout(S)
    lut = SparseFlashLUT(lay, 64, causal=True)
    dev = torch.device("cuda")
    q, k, v = (torch.randn(B, H, S, D, device=dev, dtype=torch.bfloat16) for _ in range(3))
    o = sparse_flash_attention(q, k, v, lut, 1.0, out_bshd=True)
    assert o.shape == (B, S, H, D)
    ref = _reference(q, k, v, lay, 64, True, 1.0)
    assert (o.float().transpose(1, 2) - ref).abs().max().item() < 3e-2
    assert lut.density < 0.5


@pytest.mark.gpu
def test_sparse_self_attention_fused_matches_unfused():
    """SparseSelfAttention takes the fused kernel when no masks / RPE are given; it must agree
    with its SDD / softmax / DSD path (forced with an all-ones attention mask)."""
    from deeperspeed_amd.ops.sparse_attention import FixedSparsityConfig, SparseSelfAttention
    random.seed(0)
    torch.manual_seed(2)
    B, H, S, D = 2, 4, 512, 64
    attn = SparseSelfAttention(FixedSparsityConfig(num_heads=H, block=16, num_local_blocks=4), max_seq_length=S)
    dev = torch.device("cuda")
    q, k, v = (torch.randn(B, H, S, D, device=dev, dtype=torch.float16, requires_grad=True) for _ in range(3))
    fused = attn(q, k, v)
    assert attn.get_lut(S) is not None
    attn.fused_masks = False  # an all-ones 'mul' attention mask through SDD / softmax / DSD
    unfused = attn(q, k, v, attn_mask=torch.ones(S, S, device=dev, dtype=torch.float16))
    attn.fused_masks = True
    assert (fused.float() - unfused.float()).abs().max().item() < 1e-2
    fused.float().sum().backward()
    assert all(t.grad is not None and torch.isfinite(t.grad).all() for t in (q, k, v))


@pytest.mark.gpu
def test_neox_bigbird_fused_path_trains():
    from deeperspeed_amd.models.gpt_neox import GPTNeoX, get_config
    random.seed(0)
    torch.manual_seed(0)
    dev = torch.device("cuda")
    cfg = get_config("gpt-neox-125m", num_layers=2, max_seq_len=1024,
                     sparse_attention={"mode": "bigbird", "block": 64})
    m = GPTNeoX(cfg, device=dev, dtype=torch.bfloat16)
    ids = torch.randint(0, cfg.vocab_size, (1, 1024), device=dev)
    loss = m(ids, labels=ids)
    loss.backward()
    att = m.layers[0].attention
    assert att._sp_ops[1024][3] is not None  # the fused LUT was built and used
    assert torch.isfinite(loss) and all(torch.isfinite(p.grad).all() for p in m.parameters() if p.grad is not None)


def _masked_reference(q, k, v, lay, block, scale, kbias, ebias):
    S = q.shape[2]
    m = lay.bool().repeat_interleave(block, 1).repeat_interleave(block, 2)[:, :S, :S].to(q.device)
    if m.shape[0] == 1:
        m = m.expand(q.shape[1], S, S)
    s = (q.float() @ k.float().transpose(-1, -2)) * scale
    if kbias is not None:
        s = s + kbias.float()[:, None, None, :]
    if ebias is not None:
        s = s + ebias.float()
    s = s.masked_fill(~m[None], float("-inf"))
    p = torch.softmax(s, dim=-1).nan_to_num(0.0)
    return p @ v.float()


@pytest.mark.gpu
@pytest.mark.parametrize("block,D,dtype,kp_mode,attn_mode", [
    (32, 64, torch.bfloat16, "mul", "mul"), (64, 96, torch.float16, "add", "add"),
    (16, 128, torch.bfloat16, "add", "mul")])
def test_sparse_flash_masks_and_rpe_match_reference(block, D, dtype, kp_mode, attn_mode):
    """Key-padding mask, attention mask and relative position embedding inside the fused
    kernels (reference Softmax semantics, add / mul modes) against the fp32 dense reference."""
    from deeperspeed_amd.ops.sparse_attention.flash import score_biases, sparse_flash_attention
    torch.manual_seed(4)
    B, H, S = 2, 4, 512
    dev = torch.device("cuda")
    lay = _rand_layout(H, S // block, 0.35, 5)
    lut = SparseFlashLUT(lay, block)
    q, k, v = (torch.randn(B, H, S, D, device=dev, dtype=dtype, requires_grad=True) for _ in range(3))
    if kp_mode == "mul":  # batch 1 pads its last 100 keys
        kpm = torch.ones(B, S, device=dev, dtype=dtype)
        kpm[1, -100:] = 0
    else:
        kpm = (torch.randn(B, S, device=dev) * 0.5).to(dtype)
    attn = (torch.rand(S, S, device=dev) > 0.2).to(dtype) if attn_mode == "mul" else \
        (torch.randn(S, S, device=dev) * 0.3).to(dtype)
    rpe = (torch.randn(1, H, S, S, device=dev) * 0.2).to(dtype)
    kbias, ebias = score_biases(q, rpe, kpm, attn, kp_mode, attn_mode)
    scale = D ** -0.5
    o = sparse_flash_attention(q, k, v, lut, scale, kbias=kbias, ebias=ebias)
    g = torch.randn_like(o)
    o.backward(g)
    qr, kr, vr = (t.detach().float().requires_grad_(True) for t in (q, k, v))
    ref = _masked_reference(qr, kr, vr, lay, block, scale, kbias, ebias)
    ref.backward(g.float())
    tol = 2e-2 if dtype == torch.bfloat16 else 5e-3
    assert (o.float() - ref).abs().max().item() < tol * max(1.0, ref.abs().max().item())
    for a, b in ((q.grad, qr.grad), (k.grad, kr.grad), (v.grad, vr.grad)):
        err = (a.float() - b).abs().max().item()
        assert err < 4 * tol * max(1.0, b.abs().max().item()), err


@pytest.mark.gpu
def test_sparse_self_attention_masked_fused_matches_unfused():
    """SparseSelfAttention / BertSparseSelfAttention with masks: the fused kernels agree with the
    SDD / softmax / DSD path given the same masks and RPE."""
    from deeperspeed_amd.ops.sparse_attention import FixedSparsityConfig, SparseSelfAttention
    random.seed(0)
    torch.manual_seed(6)
    B, H, S, D = 2, 4, 512, 64
    attn = SparseSelfAttention(FixedSparsityConfig(num_heads=H, block=16, num_local_blocks=4), max_seq_length=S)
    dev = torch.device("cuda")
    q, k, v = (torch.randn(B, H, S, D, device=dev, dtype=torch.bfloat16) for _ in range(3))
    kpm = torch.zeros(B, 1, 1, S, device=dev, dtype=torch.bfloat16)
    kpm[0, ..., -64:] = -10000.0  # HF-style additive padding mask
    rpe = (torch.randn(H, S, S, device=dev) * 0.1).to(torch.bfloat16)
    fused = attn(q, k, v, rpe=rpe, key_padding_mask=kpm)
    attn.fused_masks = False
    unfused = attn(q, k, v, rpe=rpe, key_padding_mask=kpm)
    assert (fused.float() - unfused.float()).abs().max().item() < 3e-2
