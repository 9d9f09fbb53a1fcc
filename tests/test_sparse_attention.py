"""Block-sparse attention (reference tests/unit/test_sparse_attention.py): layouts identical to
the reference's pure-Python configs, MatMul sdd/dsd/dds (all transpositions) and Softmax (scale,
rpe, masks) vs dense PyTorch, gradients, and SparseSelfAttention == dense attention on a dense
layout.  CPU here; the HIP kernels are compared against these in test_kernels_gpu.py."""

import importlib.util
import os
import random

import pytest
import torch

import deeperspeed_amd.ops.sparse_attention as sa

REF = "/root/reference/deepspeed/ops/sparse_attention/sparsity_config.py"


def _ref_module():
    if not os.path.exists(REF):
        pytest.skip("reference sources not mounted")
    spec = importlib.util.spec_from_file_location("ref_sparsity_config", REF)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)  # plain torch + random, no native code
    return mod


CASES = [
    ("DenseSparsityConfig", dict(num_heads=2, block=16)),
    ("FixedSparsityConfig", dict(num_heads=4, block=16, num_local_blocks=4, num_global_blocks=1)),
    ("FixedSparsityConfig", dict(num_heads=4, block=16, num_local_blocks=4, num_global_blocks=2,
                                 attention="unidirectional")),
    ("FixedSparsityConfig", dict(num_heads=4, block=16, different_layout_per_head=True, num_local_blocks=4,
                                 num_global_blocks=1, horizontal_global_attention=True,
                                 num_different_global_patterns=4)),
    ("VariableSparsityConfig", dict(num_heads=2, block=16, num_random_blocks=2, local_window_blocks=[2, 3],
                                    global_block_indices=[0, 5])),
    ("VariableSparsityConfig", dict(num_heads=2, block=16, local_window_blocks=[4], global_block_indices=[1],
                                    global_block_end_indices=[3], attention="unidirectional")),
    ("BigBirdSparsityConfig", dict(num_heads=2, block=16, num_random_blocks=2, num_sliding_window_blocks=3)),
    ("BigBirdSparsityConfig", dict(num_heads=2, block=16, attention="unidirectional")),
    ("BSLongformerSparsityConfig", dict(num_heads=2, block=16, num_sliding_window_blocks=5,
                                        global_block_indices=[0, 4], global_block_end_indices=[2, 6])),
    ("BSLongformerSparsityConfig", dict(num_heads=2, block=16, attention="unidirectional")),
    ("LocalSlidingWindowSparsityConfig", dict(num_heads=2, block=16, num_sliding_window_blocks=3)),
]


@pytest.mark.parametrize("name,kw", CASES)
@pytest.mark.parametrize("seq", [256, 336])
def test_layouts_match_reference(name, kw, seq):
    ref = _ref_module()
    random.seed(1234)
    a = getattr(ref, name)(**kw).make_layout(seq)
    random.seed(1234)
    b = getattr(sa, name)(**kw).make_layout(seq)
    assert torch.equal(a, b)


def _layout(H=2, nb=6, seed=0):
    g = torch.Generator().manual_seed(seed)
    lay = (torch.rand(H, nb, nb, generator=g) < 0.5).long()
    lay[:, torch.arange(nb), torch.arange(nb)] = 1  # every row has a block
    return lay


def _mask(lay, blk):
    return lay.repeat_interleave(blk, 1).repeat_interleave(blk, 2).bool()


def _to_sparse(dense, lay, blk):
    nz = lay.nonzero()
    Z, H, S, _ = dense.shape
    v = dense.view(Z, H, S // blk, blk, S // blk, blk).permute(0, 1, 2, 4, 3, 5)
    return v[:, nz[:, 0], nz[:, 1], nz[:, 2]]


def _to_dense(sp, lay, blk):
    nz = lay.nonzero()
    H, nb, _ = lay.shape
    Z = sp.shape[0]
    out = torch.zeros(Z, H, nb, nb, blk, blk, dtype=sp.dtype)
    out[:, nz[:, 0], nz[:, 1], nz[:, 2]] = sp
    return out.permute(0, 1, 2, 4, 3, 5).reshape(Z, H, nb * blk, nb * blk)


@pytest.mark.parametrize("mode", ["sdd", "dsd", "dds"])
@pytest.mark.parametrize("ta", [False, True])
@pytest.mark.parametrize("tb", [False, True])
def test_matmul_matches_dense(mode, ta, tb):
    torch.manual_seed(0)
    blk, H, nb, Z, D = 16, 2, 5, 2, 24
    S = nb * blk
    lay = _layout(H, nb)
    mm = sa.MatMul(lay, blk, mode, trans_a=ta, trans_b=tb)
    mask = _mask(lay, blk)
    if mode == "sdd":
        a = torch.randn(Z, H, *((D, S) if ta else (S, D)), requires_grad=True)
        b = torch.randn(Z, H, *((S, D) if tb else (D, S)), requires_grad=True)
        out = mm(a, b)
        ae = a.transpose(-1, -2) if ta else a
        be = b.transpose(-1, -2) if tb else b
        ref = _to_sparse(ae @ be, lay, blk)
    elif mode == "dsd":
        sp = torch.randn(Z, int(lay.sum()), blk, blk, requires_grad=True)
        b = torch.randn(Z, H, *((D, S) if tb else (S, D)), requires_grad=True)
        a = sp
        out = mm(sp, b)
        dense = _to_dense(sp, lay, blk)
        ref = (dense.transpose(-1, -2) if ta else dense) @ (b.transpose(-1, -2) if tb else b)
    else:
        a = torch.randn(Z, H, *((S, D) if ta else (D, S)), requires_grad=True)
        sp = torch.randn(Z, int(lay.sum()), blk, blk, requires_grad=True)
        b = sp
        out = mm(a, sp)
        dense = _to_dense(sp, lay, blk)
        ref = (a.transpose(-1, -2) if ta else a) @ (dense.transpose(-1, -2) if tb else dense)
    torch.testing.assert_close(out, ref, atol=1e-4, rtol=1e-4)
    g = torch.randn_like(out)
    ga, gb = torch.autograd.grad(out, (a, b), g)
    ra, rb = torch.autograd.grad(ref, (a, b), g)
    torch.testing.assert_close(ga, ra, atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(gb, rb, atol=1e-4, rtol=1e-4)


@pytest.mark.parametrize("kpm_mode,attn_mode", [("add", "add"), ("mul", "mul")])
def test_softmax_matches_dense(kpm_mode, attn_mode):
    torch.manual_seed(0)
    blk, H, nb, Z = 16, 2, 4, 2
    S = nb * blk
    lay = _layout(H, nb, seed=3)
    x = torch.randn(Z, int(lay.sum()), blk, blk, requires_grad=True)
    rpe = torch.randn(1, H, S, S)
    kpm = (torch.rand(Z, S) > 0.2).float() if kpm_mode == "mul" else torch.randn(Z, S)
    attn = (torch.rand(S, S) > 0.3).float() if attn_mode == "mul" else torch.randn(S, S)
    attn[:, 0] = 1.0
    kpm[:, 0] = 1.0
    y = sa.Softmax(lay, blk)(x, scale=0.3, rpe=rpe, key_padding_mask=kpm, attn_mask=attn,
                             key_padding_mask_mode=kpm_mode, attn_mask_mode=attn_mode)
    dense = _to_dense(x, lay, blk) * 0.3 + rpe
    km = torch.where(kpm == 0, float("-inf"), 0.0) if kpm_mode == "mul" else kpm
    am = torch.where(attn == 0, float("-inf"), 0.0) if attn_mode == "mul" else attn
    dense = dense + km[:, None, None, :] + am
    dense = dense.masked_fill(~_mask(lay, blk), float("-inf"))
    ref = _to_sparse(torch.softmax(dense, -1).nan_to_num(0.0), lay, blk)
    torch.testing.assert_close(y, ref, atol=1e-5, rtol=1e-5)
    g = torch.randn_like(y)
    (gx,) = torch.autograd.grad(y, x, g)
    (rx,) = torch.autograd.grad(ref, x, g)
    torch.testing.assert_close(gx, rx, atol=1e-5, rtol=1e-4)


def test_sparse_self_attention_dense_layout_equals_attention():
    torch.manual_seed(0)
    cfg = sa.DenseSparsityConfig(num_heads=2, block=16)
    attn = sa.SparseSelfAttention(cfg, max_seq_length=64)
    q, k, v = (torch.randn(2, 2, 64, 32) for _ in range(3))
    out = attn(q, k, v)
    ref = torch.softmax(q @ k.transpose(-1, -2) / 32 ** 0.5, -1) @ v
    torch.testing.assert_close(out, ref, atol=1e-4, rtol=1e-4)


def test_bert_sparse_self_attention_and_utils():
    from types import SimpleNamespace
    torch.manual_seed(0)
    cfg = SimpleNamespace(hidden_size=64, num_attention_heads=4)
    layer = sa.BertSparseSelfAttention(cfg, sa.FixedSparsityConfig(num_heads=4, block=16))
    x = torch.randn(2, 48, 64)
    mask = torch.ones(2, 48)
    y = layer(x, mask)
    assert y.shape == (2, 48, 64)
    ids = torch.ones(2, 40, dtype=torch.long)
    pad, ids2, am, tt, pos, emb = sa.SparseAttentionUtils.pad_to_block_size(
        16, ids, torch.ones(2, 40), torch.zeros(2, 40, dtype=torch.long), None, None, 0, None)
    assert pad == 8 and ids2.shape == (2, 48) and am.shape == (2, 48) and bool(am[0, -1] == 0)
    assert sa.SparseAttentionUtils.unpad_sequence_output(pad, torch.zeros(2, 48, 4)).shape == (2, 40, 4)


def test_neox_sparse_attention_dense_layout_matches_dense_model():
    """GPT-NeoX with a dense 'sparse' layout must equal the dense causal model."""
    from deeperspeed_amd.models.gpt_neox import GPTNeoX, get_config
    torch.manual_seed(0)
    cfg = get_config("tiny", num_layers=2, checkpoint_activations=False)
    dense = GPTNeoX(cfg)
    cfg2 = get_config("tiny", num_layers=2, checkpoint_activations=False,
                      sparse_attention={"mode": "dense", "block": 16})
    sparse = GPTNeoX(cfg2)
    sparse.load_state_dict(dense.state_dict())
    ids = torch.randint(0, cfg.vocab_size, (2, 64))
    torch.testing.assert_close(sparse(ids), dense(ids), atol=1e-4, rtol=1e-4)
    cfg3 = get_config("tiny", num_layers=2, checkpoint_activations=False,
                      sparse_attention={"mode": "bigbird", "block": 16, "num_random_blocks": 1})
    m3 = GPTNeoX(cfg3)
    m3.load_state_dict(dense.state_dict())
    loss = m3(ids, labels=ids)
    loss.backward()
    assert torch.isfinite(loss)
    # causality: the logits at position t must not depend on tokens after t
    ids2 = ids.clone()
    ids2[:, 40:] = (ids2[:, 40:] + 1) % cfg.vocab_size
    torch.testing.assert_close(m3(ids)[:, :40], m3(ids2)[:, :40], atol=1e-5, rtol=1e-5)


def test_dsd_row_segments_cover_every_block_once():
    """The dsd row-segment LUT (long rows of layout^T split with partial slots) covers each
    non-zero block exactly once, every row appears, and split rows own contiguous slots."""
    import random
    from deeperspeed_amd.ops.sparse_attention import sparsity_config as sc
    from deeperspeed_amd.ops.sparse_attention.matmul import SparseLayout
    random.seed(0)
    lay = sc.BigBirdSparsityConfig(num_heads=2, block=16, attention="unidirectional").make_layout(1024)
    L = SparseLayout(lay, 16)
    for trans in (False, True):
        seg, fin, nslots = L.segments(trans)
        cov = torch.zeros(L.nnz, dtype=torch.long)
        rows = set()
        for r, a, b, slot in seg.tolist():
            cov[a:b] += 1
            rows.add(r)
        assert (cov == 1).all() and rows == set(range(L.H * (L.nbc if trans else L.nbr)))
        slots = sorted(sl for *_, sl in seg.tolist() if sl >= 0)
        assert slots == list(range(nslots))
        for r, s0, k, _ in fin.tolist():
            assert sorted(sl for rr, _, _, sl in seg.tolist() if rr == r) == list(range(s0, s0 + k))
        lens = (seg[:, 2] - seg[:, 1]).tolist()
        assert lens == sorted(lens, reverse=True)
    assert L.segments(True)[2] > 0  # the global key columns are split when walked transposed


def test_hf_bert_with_sparse_self_attention_matches_dense():
    """SparseAttentionUtils on the installed HuggingFace BertModel (its current attention call:
    keyword arguments, an (output, weights) pair back, a [B, 1, S, S] dtype-min padding mask):
    a layout that covers every block must equal HF's own eager attention, padding included."""
    transformers = pytest.importorskip("transformers")
    cfg = transformers.BertConfig(hidden_size=64, num_hidden_layers=2, num_attention_heads=4, intermediate_size=128,
                                  max_position_embeddings=128, vocab_size=100, attn_implementation="eager")
    torch.manual_seed(0)
    m = transformers.BertModel(cfg).eval()
    ids = torch.randint(0, 100, (2, 128))
    am = torch.ones(2, 128, dtype=torch.long)
    am[0, 96:] = 0
    ref = m(ids, attention_mask=am).last_hidden_state
    holder = type("Holder", (), {})()
    holder.bert, holder.config = m, cfg
    sa.SparseAttentionUtils.replace_model_self_attention_with_sparse_self_attention(
        holder, 128, sa.FixedSparsityConfig(num_heads=4, block=16, num_local_blocks=8, attention="bidirectional"))
    assert isinstance(m.encoder.layer[0].attention.self, sa.BertSparseSelfAttention)
    torch.testing.assert_close(m(ids, attention_mask=am).last_hidden_state, ref, atol=1e-5, rtol=1e-5)


def test_sparse_self_attention_rejects_sequences_past_its_layout():
    """A sequence longer than max_seq_length raises instead of silently using a truncated layout;
    BertSparseSelfAttention sizes its layout from the model's max_position_embeddings."""
    from types import SimpleNamespace
    attn = sa.SparseSelfAttention(sa.FixedSparsityConfig(num_heads=2, block=16), max_seq_length=64)
    with pytest.raises(RuntimeError, match="max_seq_length"):
        attn.get_layout(128)
    cfg = SimpleNamespace(hidden_size=32, num_attention_heads=2, max_position_embeddings=4096)
    layer = sa.BertSparseSelfAttention(cfg, sa.FixedSparsityConfig(num_heads=2, block=64))
    assert layer.sparse_self_attention.get_layout(4096).shape[-1] == 64
