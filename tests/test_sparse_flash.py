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


def _expand16(lay, block, causal):
    L = lay.bool().numpy()
    r = block // 16
    L = np.repeat(np.repeat(L, r, axis=1), r, axis=2)
    if causal:
        L = L & np.tril(np.ones(L.shape[-2:], dtype=bool))[None]
    return L


@pytest.mark.parametrize("block,causal", [(16, False), (32, True), (64, False), (128, True), (16, True)])
def test_lut_covers_layout_exactly_once(block, causal):
    """Forward / dQ walk: every active (query 16-block, key 16-block) pair of the layout appears in
    exactly one entry of its query tile, with its mask bit set; no inactive pair has a bit; the
    dK / dV walk covers the same pairs once per key group, and the groups partition the keys."""
    S, H = 512, 3
    lay = _rand_layout(H, S // block, 0.3, 1)
    lut = SparseFlashLUT(lay, block, causal=causal)
    rp, cols, masks, cp, rows, masks_t, tasks, fin, kgroups = lut._host
    L = _expand16(lay, block, causal)
    nqt, n16 = S // 64, S // 16
    for h in range(H):
        seen = np.zeros((n16, n16), dtype=int)
        for qt in range(nqt):
            for e in range(rp[h * nqt + qt], rp[h * nqt + qt + 1]):
                blk, m = cols[e], int(masks[e]) & 0xffff
                assert list(blk) == sorted(blk)
                for qs in range(4):
                    for ks in range(4):
                        if (m >> (qs * 4 + ks)) & 1:
                            seen[qt * 4 + qs, blk[ks]] += 1
        assert np.array_equal(seen, L[h].astype(int))
        assert sorted(kgroups[h].reshape(-1).tolist()) == list(range(n16))
        seen_t = np.zeros((n16, n16), dtype=int)
        for g in range(nqt):
            kb = kgroups[h, g]
            assert list(kb) == sorted(kb)
            for e in range(cp[h * nqt + g], cp[h * nqt + g + 1]):
                qb, m = rows[e], int(masks_t[e]) & 0xffff
                assert list(qb) == sorted(qb)
                for qs in range(4):
                    for ks in range(4):
                        if (m >> (qs * 4 + ks)) & 1:
                            seen_t[qb[qs], kb[ks]] += 1
        assert np.array_equal(seen_t, L[h].astype(int))


def _emulate_fwd(q, k, v, lut, scale, causal):
    """The forward kernel's walk in float64 numpy: per query tile, each entry gathers its four key
    16-blocks, masks by the entry bits (+ causal on true positions) and folds into a softmax."""
    rp, cols, masks = lut._host[:3]
    B, H, S, D = q.shape
    nqt = S // 64
    out = np.zeros((B, H, S, D))
    for b in range(B):
        for hh in range(H):
            lh = 0 if lut.heads == 1 else hh
            for qt in range(nqt):
                qrows = np.arange(qt * 64, qt * 64 + 64)
                sc_all, vv_all = [], []
                for e in range(rp[lh * nqt + qt], rp[lh * nqt + qt + 1]):
                    keys = np.concatenate([np.arange(bk * 16, bk * 16 + 16) for bk in cols[e]])
                    m = int(masks[e]) & 0xffff
                    act = np.array([[(m >> ((i // 16) * 4 + j // 16)) & 1 for j in range(64)] for i in range(64)],
                                   dtype=bool)
                    if causal:
                        act &= keys[None, :] <= qrows[:, None]
                    s_ = q[b, hh, qrows] @ k[b, hh, keys].T * scale
                    sc_all.append(np.where(act, s_, -np.inf))
                    vv_all.append(v[b, hh, keys])
                if not sc_all:
                    continue
                s_ = np.concatenate(sc_all, axis=1)
                mx = s_.max(axis=1, keepdims=True)
                p = np.where(np.isfinite(s_), np.exp(s_ - np.where(np.isfinite(mx), mx, 0)), 0.0)
                l = p.sum(axis=1, keepdims=True)
                out[b, hh, qrows] = (p @ np.concatenate(vv_all, axis=0)) / np.where(l > 0, l, 1)
    return out


@pytest.mark.parametrize("block,causal", [(16, True), (32, False)])
def test_gathered_walk_equals_dense_reference(block, causal):
    """CPU check of the gathered-tile semantics the kernels implement (no GPU)."""
    rng = np.random.default_rng(0)
    B, H, S, D = 1, 2, 256, 8
    lay = _rand_layout(H, S // block, 0.3, 7)
    lut = SparseFlashLUT(lay, block, causal=causal)
    q, k, v = (rng.standard_normal((B, H, S, D)) for _ in range(3))
    got = _emulate_fwd(q, k, v, lut, 0.3, causal)
    ref = _reference(torch.from_numpy(q), torch.from_numpy(k), torch.from_numpy(v), lay, block, causal, 0.3)
    assert np.abs(got - ref.double().numpy()).max() < 1e-5  # _reference computes in fp32


def test_fixed16_gathers_fewer_tiles_than_dense():
    """The reference's default sparse layout (fixed, block 16): one global key block per 64-key
    window made every 64-tile active; gathered 16-blocks cut the forward walk ~3.5x."""
    from deeperspeed_amd.ops.sparse_attention.sparsity_config import FixedSparsityConfig
    lay = FixedSparsityConfig(num_heads=4, block=16, attention="unidirectional").make_layout(4096)
    lut = SparseFlashLUT(lay, 16, causal=True)
    dense_tiles = 64 * 65 // 2
    assert lut.tiles < 0.3 * dense_tiles
    assert lut._host[4].shape[0] < 0.35 * dense_tiles  # dK / dV entries (count-sorted key groups)


def test_dkdv_tasks_cover_transposed_lut():
    """Key groups with more than CHUNK entries (global columns) are split into chunks whose
    partial slots are summed by the finish pass; every entry is covered exactly once."""
    S = 2048
    lay = torch.zeros(2, S // 64, S // 64, dtype=torch.long)
    lay[:, :, 0] = 1  # global column
    for i in range(S // 64):
        lay[:, i, max(0, i - 2): i + 1] = 1
    lay[1, :, 5] = 1
    lut = SparseFlashLUT(lay, 64, causal=True)
    rp, cols, masks, cp, rows, masks_t, tasks, fin, kgroups = lut._host
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
        assert heavy and heavy[0][2] == -(-nt // lut.CHUNK)
        assert list(kgroups[h, heavy[0][0]]) == [0, 1, 2, 3]  # the global column's group
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
