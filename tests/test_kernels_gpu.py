"""Numerics of the HIP kernels vs plain PyTorch fp32 references (run on MI355X)."""

import pytest
import torch

pytestmark = pytest.mark.gpu


def _dev():
    return torch.device("cuda", 0)


def test_extension_is_native():
    from deeperspeed_amd.ops import native
    mod = native.hip_ops()
    assert mod.__file__.endswith(".so")


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("H", [64, 768, 2048, 6144])
def test_layernorm_fwd_bwd(dtype, H):
    from deeperspeed_amd.ops.native import layer_norm
    torch.manual_seed(0)
    x = torch.randn(37, 5, H, device=_dev(), dtype=dtype, requires_grad=True)
    w = (1 + 0.1 * torch.randn(H, device=_dev())).to(dtype).requires_grad_(True)
    b = (0.1 * torch.randn(H, device=_dev())).to(dtype).requires_grad_(True)
    y = layer_norm(x, w, b, 1e-5)
    dy = torch.randn_like(y)
    y.backward(dy)
    xr = x.detach().float().requires_grad_(True)
    wr = w.detach().float().requires_grad_(True)
    br = b.detach().float().requires_grad_(True)
    yr = torch.nn.functional.layer_norm(xr, (H,), wr, br, 1e-5)
    yr.backward(dy.float())
    tol = 2e-2 if dtype != torch.float32 else 1e-4
    assert torch.allclose(y.float(), yr, atol=tol, rtol=tol)
    assert torch.allclose(x.grad.float(), xr.grad, atol=tol * 5, rtol=tol)
    gtol = tol * 10 if dtype != torch.float32 else 1e-3
    assert torch.allclose(w.grad.float(), wr.grad, atol=gtol * 10, rtol=gtol)
    assert torch.allclose(b.grad.float(), br.grad, atol=gtol * 10, rtol=gtol)


@pytest.mark.parametrize("rows", [3, 4100, 8192])
@pytest.mark.parametrize("H", [768, 1024, 2048])
def test_layernorm_residual_wave_bwd(rows, H):
    """Wave-per-row LayerNorm backward with the fused residual-gradient add (pre-LN blocks):
    rows beyond one grid pass exercise the software-pipelined row loop and its tail."""
    from deeperspeed_amd.ops.native import layer_norm_residual
    torch.manual_seed(3)
    x = torch.randn(rows, H, device=_dev(), dtype=torch.bfloat16, requires_grad=True)
    w = (1 + 0.1 * torch.randn(H, device=_dev())).to(torch.bfloat16).requires_grad_(True)
    b = (0.1 * torch.randn(H, device=_dev())).to(torch.bfloat16).requires_grad_(True)
    y, res = layer_norm_residual(x, w, b, 1e-5)
    dy, dr = torch.randn_like(y), torch.randn_like(res)
    torch.autograd.backward((y, res), (dy, dr))
    xr = x.detach().float().requires_grad_(True)
    wr = w.detach().float().requires_grad_(True)
    br = b.detach().float().requires_grad_(True)
    yr = torch.nn.functional.layer_norm(xr, (H,), wr, br, 1e-5)
    torch.autograd.backward((yr, xr), (dy.float(), dr.float()))
    assert torch.allclose(x.grad.float(), xr.grad, atol=0.1, rtol=2e-2)
    assert torch.allclose(w.grad.float(), wr.grad, atol=2e-2 * rows ** 0.5, rtol=2e-2)
    assert torch.allclose(b.grad.float(), br.grad, atol=2e-2 * rows ** 0.5, rtol=2e-2)


@pytest.mark.parametrize("residual", [False, True])
@pytest.mark.parametrize("H", [1024, 6144])
def test_layernorm_accumulates_into_bound_param_grads(residual, H):
    """With gamma.grad / beta.grad already bound (engine gradient views), the LN backward adds
    its column sums into them in the colsum kernel (autograd gets None): same result as autograd
    adding fresh gradients."""
    from deeperspeed_amd.ops.native import FusedLayerNorm
    torch.manual_seed(5)
    ln = FusedLayerNorm(H, 1e-5, dtype=torch.bfloat16, device=_dev())
    with torch.no_grad():
        ln.weight.add_(0.1 * torch.randn_like(ln.weight))
        ln.bias.add_(0.1 * torch.randn_like(ln.bias))
    x = torch.randn(512, H, device=_dev(), dtype=torch.bfloat16, requires_grad=True)
    dy = torch.randn(512, H, device=_dev(), dtype=torch.bfloat16)

    def run():
        out = ln(x, residual_out=True)[0] if residual else ln(x)
        out.backward(dy)

    run()  # first use: fresh gradients through autograd
    g1, b1 = ln.weight.grad.clone(), ln.bias.grad.clone()
    x.grad = None
    run()  # bound gradients: accumulated in place by the kernel
    assert torch.allclose(ln.weight.grad.float(), 2 * g1.float(), rtol=2e-2, atol=2e-2)
    assert torch.allclose(ln.bias.grad.float(), 2 * b1.float(), rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("approx", [False, True])
def test_bias_gelu(dtype, approx):
    from deeperspeed_amd.ops.native import bias_gelu
    torch.manual_seed(1)
    C = 4096
    x = torch.randn(300, C, device=_dev(), dtype=dtype, requires_grad=True)
    b = torch.randn(C, device=_dev(), dtype=dtype, requires_grad=True)
    y = bias_gelu(x, b, approx)
    dy = torch.randn_like(y)
    y.backward(dy)
    xr = x.detach().float().requires_grad_(True)
    br = b.detach().float().requires_grad_(True)
    yr = torch.nn.functional.gelu(xr + br, approximate="tanh" if approx else "none")
    yr.backward(dy.float())
    tol = 2e-2 if dtype != torch.float32 else 1e-5
    assert torch.allclose(y.float(), yr, atol=tol, rtol=tol)
    assert torch.allclose(x.grad.float(), xr.grad, atol=tol * 2, rtol=tol)
    assert torch.allclose(b.grad.float(), br.grad, atol=0.5 if dtype != torch.float32 else 1e-3, rtol=2e-2)


@pytest.mark.parametrize("pdtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("adamw", [False, True])
def test_adam_flat_matches_torch(pdtype, adamw):
    from deeperspeed_amd.ops import native
    torch.manual_seed(2)
    n = 100003  # odd size exercises the tail path
    master = torch.randn(n, device=_dev())
    ref = master.clone().requires_grad_(True)
    m = torch.zeros(n, device=_dev())
    v = torch.zeros(n, device=_dev())
    out = torch.empty(n, device=_dev(), dtype=pdtype)
    cls = torch.optim.AdamW if adamw else torch.optim.Adam
    opt = cls([ref], lr=1e-2, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.1)
    for step in range(1, 4):
        g = torch.randn(n, device=_dev()).to(pdtype)
        ref.grad = g.float().clone()
        opt.step()
        native.adam_flat_(master, g, m, v, out, 1e-2, 0.9, 0.999, 1e-8, 0.1, step, True, 1.0, adamw)
    gtol = 1e-5
    assert torch.allclose(master, ref.detach(), atol=gtol, rtol=gtol)
    assert torch.allclose(out.float(), ref.detach(), atol=2e-2, rtol=1e-2)


def test_sumsq_and_colsum():
    from deeperspeed_amd.ops import native
    x = torch.randn(1 << 20, device=_dev(), dtype=torch.bfloat16)
    out = torch.zeros(1, device=_dev())
    native.sumsq_accumulate(x, out)
    native.sumsq_accumulate(x, out)
    ref = 2 * x.float().pow(2).sum()
    assert torch.allclose(out[0], ref, rtol=1e-4)
    y = torch.randn(513, 1024, device=_dev(), dtype=torch.bfloat16)
    assert torch.allclose(native.colsum(y).float(), y.float().sum(0), atol=0.2, rtol=2e-2)


@pytest.mark.parametrize("hd,rot", [(96, 24), (128, 32), (64, 64), (96, 96), (32, 8), (64, 16), (128, 128), (80, 20)])
# 41 x 5: the last chunk-kernel block is partial; 48 x 8: the LDS-tiled kernels (S % 16, NH % 4)
@pytest.mark.parametrize("S,NH", [(40, 4), (41, 5), (48, 8)])
def test_rotary_split_matches_reference(hd, rot, S, NH):
    from deeperspeed_amd.ops import attention as A
    torch.manual_seed(3)
    B = 2
    qkv = torch.randn(B, S, NH * 3 * hd, device=_dev(), dtype=torch.bfloat16, requires_grad=True)
    q, k, v = A.rotary_split(qkv, NH, hd, rot, qscale=0.5)
    g = [torch.randn_like(t) for t in (q, k, v)]
    torch.autograd.backward([q, k, v], g)
    x = qkv.detach().cpu().float().requires_grad_(True)
    qr, kr, vr = A.rotary_split(x, NH, hd, rot, qscale=0.5)
    torch.autograd.backward([qr, kr, vr], [t.cpu().float() for t in g])
    for a, b in ((q, qr), (k, kr), (v, vr)):
        assert torch.allclose(a.float().cpu(), b, atol=3e-2, rtol=2e-2)
    assert torch.allclose(qkv.grad.float().cpu(), x.grad, atol=3e-2, rtol=2e-2)


@pytest.mark.parametrize("causal", [True, False])
@pytest.mark.parametrize("S", [64, 200, 2048])
def test_masked_softmax(causal, S):
    from deeperspeed_amd.ops.attention import masked_softmax
    torch.manual_seed(4)
    C = (S + 7) // 8 * 8
    x = torch.randn(3, 5, S, C, device=_dev(), dtype=torch.bfloat16, requires_grad=True)
    y = masked_softmax(x, None, 0.7, causal, 5)
    dy = torch.randn_like(y)
    y.backward(dy)
    xr = x.detach().float().requires_grad_(True)
    s = xr * 0.7
    if causal:
        m = torch.ones(S, C, dtype=torch.bool, device=_dev()).triu(C - S + 1)
        s = s.masked_fill(m, float("-inf"))
    yr = torch.softmax(s, -1)
    yr.backward(dy.float())
    assert torch.allclose(y.float(), yr, atol=1e-2, rtol=2e-2)
    assert torch.allclose(x.grad.float(), xr.grad, atol=2e-2, rtol=5e-2)


def test_attention_matches_sdpa_math():
    from deeperspeed_amd.ops.attention import attention
    torch.manual_seed(5)
    B, NH, S, HD = 2, 4, 256, 96
    q = torch.randn(B, NH, S, HD, device=_dev(), dtype=torch.bfloat16, requires_grad=True)
    k = torch.randn_like(q, requires_grad=True)
    v = torch.randn_like(q, requires_grad=True)
    scale = HD ** -0.5
    o = attention(q, k, v, causal=True, softmax_scale=scale)
    do = torch.randn_like(o)
    o.backward(do)
    qr, kr, vr = (t.detach().float().requires_grad_(True) for t in (q, k, v))
    s = (qr @ kr.transpose(-1, -2)) * scale
    s = s.masked_fill(torch.ones(S, S, dtype=torch.bool, device=_dev()).triu(1), float("-inf"))
    orf = torch.softmax(s, -1) @ vr
    orf.backward(do.float())
    assert torch.allclose(o.float(), orf, atol=3e-2, rtol=3e-2)
    for a, b in ((q, qr), (k, kr), (v, vr)):
        assert torch.allclose(a.grad.float(), b.grad, atol=6e-2, rtol=6e-2)


def _attn_ref(q, k, v, causal, scale):
    s = (q.float() @ k.float().transpose(-1, -2)) * scale
    if causal:
        S = q.shape[-2]
        s = s.masked_fill(torch.ones(S, S, dtype=torch.bool, device=q.device).triu(1), float("-inf"))
    return torch.softmax(s, -1) @ v.float()


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("D", [64, 96, 128])
@pytest.mark.parametrize("S,causal", [(128, True), (200, True), (96, False), (333, False)])
def test_flash_attention_fwd_bwd(dtype, D, S, causal):
    from deeperspeed_amd.ops import native
    torch.manual_seed(0)
    B, H = 2, 3
    scale = D ** -0.5
    q = torch.randn(B, H, S, D, device=_dev(), dtype=dtype, requires_grad=True)
    k = torch.randn(B, H, S, D, device=_dev(), dtype=dtype, requires_grad=True)
    v = torch.randn(B, H, S, D, device=_dev(), dtype=dtype, requires_grad=True)
    assert native.has_flash_attention(q)
    o = native.flash_attention(q, k, v, causal, scale)
    do = torch.randn_like(o)
    o.backward(do)
    qr, kr, vr = (t.detach().float().requires_grad_(True) for t in (q, k, v))
    ref = _attn_ref(qr, kr, vr, causal, scale)
    ref.backward(do.float())
    tol = 2e-2 if dtype == torch.bfloat16 else 5e-3
    torch.testing.assert_close(o.float(), ref, atol=tol, rtol=tol)
    for got, want in ((q.grad, qr.grad), (k.grad, kr.grad), (v.grad, vr.grad)):
        err = (got.float() - want).abs().max().item()
        assert err <= 4 * tol * max(1.0, want.abs().max().item()), err


def test_flash_attention_lse_and_large_logits():
    """Large score magnitudes exercise the online-softmax rescale path."""
    from deeperspeed_amd.ops import native
    torch.manual_seed(1)
    q = (8 * torch.randn(1, 2, 256, 128, device=_dev())).to(torch.bfloat16)
    k = torch.randn(1, 2, 256, 128, device=_dev()).to(torch.bfloat16)
    v = torch.randn(1, 2, 256, 128, device=_dev()).to(torch.bfloat16)
    o, lse = native.hip_ops().flash_attn_fwd(q.contiguous(), k.contiguous(), v.contiguous(), True, 0.125, False)
    s = (q.float() @ k.float().transpose(-1, -2)) * 0.125
    s = s.masked_fill(torch.ones(256, 256, dtype=torch.bool, device=_dev()).triu(1), float("-inf"))
    torch.testing.assert_close(lse, torch.logsumexp(s, -1), atol=2e-2, rtol=1e-3)
    torch.testing.assert_close(o.float(), torch.softmax(s, -1) @ v.float(), atol=3e-2, rtol=3e-2)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("V", [512, 50432, 1000])
def test_fused_cross_entropy(dtype, V):
    from deeperspeed_amd.ops import native
    torch.manual_seed(0)
    x = (3 * torch.randn(2, 37, V, device=_dev())).to(dtype).requires_grad_(True)
    lab = torch.randint(0, V, (2, 37), device=_dev())
    lab[0, :5] = -100  # ignored rows
    loss = native.cross_entropy(x, lab)
    loss.backward()
    xr = x.detach().float().requires_grad_(True)
    ref = torch.nn.functional.cross_entropy(xr.view(-1, V), lab.view(-1), ignore_index=-100)
    ref.backward()
    torch.testing.assert_close(loss, ref, atol=2e-4, rtol=2e-4)
    torch.testing.assert_close(x.grad.float(), xr.grad, atol=1e-4, rtol=2e-2)


def test_adam_compact_matches_fp32_master():
    """Compact master (bf16 hi + int16 residual) must track the fp32 master bit for bit."""
    from deeperspeed_amd.ops import native
    from deeperspeed_amd.runtime.zero import compact_master as cm
    torch.manual_seed(0)
    n = 1 << 20 | 3
    w = torch.randn(n, device=_dev())
    hi, res = cm.encode(w)
    m1, v1, m2, v2 = (torch.zeros(n, device=_dev()) for _ in range(4))
    for step in range(1, 6):
        g = torch.randn(n, device=_dev()).to(torch.bfloat16)
        native.adam_flat_(w, g, m1, v1, None, 1e-3, 0.9, 0.95, 1e-8, 0.01, step, True, 0.7, True)
        native.adam_compact_(hi, res, g, m2, v2, 1e-3, 0.9, 0.95, 1e-8, 0.01, step, True, 0.7, True)
    assert torch.equal(cm.decode(hi, res).view(torch.int32), w.view(torch.int32))
    assert torch.equal(m1, m2) and torch.equal(v1, v2)


@pytest.mark.parametrize("gdt", [torch.float32, torch.bfloat16])
def test_lamb_kernel_matches_cpu(gdt):
    from deeperspeed_amd.ops import native
    torch.manual_seed(0)
    n = 100003
    w = torch.randn(n)
    wg = w.to(_dev())
    m, v = torch.zeros(n), torch.zeros(n)
    mg, vg = m.to(_dev()), v.to(_dev())
    out = torch.empty(n, dtype=torch.bfloat16, device=_dev())
    for step in range(1, 4):
        g = torch.randn(n).to(gdt)
        c1 = native.lamb_(w, g, m, v, None, 1e-2, 0.9, 0.999, 1e-8, 0.01, step, True, 0.5, 10.0, 0.01)
        c2 = native.lamb_(wg, g.to(_dev()), mg, vg, out, 1e-2, 0.9, 0.999, 1e-8, 0.01, step, True, 0.5, 10.0, 0.01)
        assert abs(float(c1) - float(c2)) < 1e-4 * abs(float(c1))
    torch.testing.assert_close(wg.cpu(), w, atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(out.float().cpu(), w, atol=1e-2, rtol=1e-2)


def test_onebit_kernels_match_cpu_reference():
    from deeperspeed_amd.ops import native
    torch.manual_seed(0)
    P, nb = 4, 1000
    n = P * nb * 8
    m = torch.randn(n)
    err = 0.1 * torch.randn(n)
    pk_c, sc_c = native.onebit_worker_compress(m, err_c := err.clone())
    pk_g, sc_g = native.onebit_worker_compress(m.to(_dev()), err_g := err.to(_dev()))
    assert torch.equal(pk_g.cpu(), pk_c)
    torch.testing.assert_close(sc_g.cpu(), sc_c, rtol=1e-5, atol=0)
    torch.testing.assert_close(err_g.cpu(), err_c, rtol=1e-5, atol=1e-6)
    signs = torch.randint(0, 256, (P * nb,), dtype=torch.uint8)
    scales = torch.rand(P)
    serr = 0.05 * torch.randn(nb * 8)
    sp_c, ss_c = native.onebit_server_compress(signs, scales, serr_c := serr.clone())
    sp_g, ss_g = native.onebit_server_compress(signs.to(_dev()), scales.to(_dev()), serr_g := serr.to(_dev()))
    assert (sp_g.cpu() != sp_c).sum() <= 2  # sign of values within fp rounding of 0 may differ
    torch.testing.assert_close(ss_g.cpu(), ss_c, rtol=1e-5, atol=0)
    out_c = native.onebit_unpack(signs, scales, torch.empty(n))
    out_g = native.onebit_unpack(signs.to(_dev()), scales.to(_dev()), torch.empty(n, device=_dev()))
    assert torch.equal(out_g.cpu(), out_c)


def _sp_layout(H, nb, seed):
    g = torch.Generator().manual_seed(seed)
    lay = (torch.rand(H, nb, nb, generator=g) < 0.4).long()
    lay[:, torch.arange(nb), torch.arange(nb)] = 1
    return lay


_SP_MODES = [("sdd", ta, tb) for ta in (False, True) for tb in (False, True)] + \
    [(m, ta, tb) for m in ("dsd", "dds") for ta, tb in ((False, False), (True, False), (False, True), (True, True))]


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("blk", [16, 32, 64, 128])
@pytest.mark.parametrize("mode,ta,tb", _SP_MODES)
def test_block_sparse_matmul_hip_vs_cpu(dtype, blk, mode, ta, tb):
    """Every mode x transpose on the LDS-staged kernels: transposed operands are read in place
    (no copies), the dense width 40 exercises partial K stages / output column tiles."""
    if dtype == torch.float16 and blk in (32, 128):
        pytest.skip("fp16 covered at blocks 16/64")
    import deeperspeed_amd.ops.sparse_attention as sa
    torch.manual_seed(0)
    H, nb, Z, D = 3, 6 if blk < 128 else 3, 2, 40
    S = nb * blk
    lay = _sp_layout(H, nb, blk)
    nnz = int(lay.sum())
    mm = sa.MatMul(lay, blk, mode, trans_a=ta, trans_b=tb)
    if mode == "sdd":
        a = torch.randn(Z, H, *((D, S) if ta else (S, D)))
        b = torch.randn(Z, H, *((S, D) if tb else (D, S)))
    elif mode == "dsd":
        a = torch.randn(Z, nnz, blk, blk) * 0.2
        b = torch.randn(Z, H, *((D, S) if tb else (S, D)))
    else:
        a = torch.randn(Z, H, *((S, D) if ta else (D, S)))
        b = torch.randn(Z, nnz, blk, blk) * 0.2
    a, b = a.to(dtype), b.to(dtype)
    ref = mm(a.float(), b.float())
    ag, bg = a.to(_dev()).requires_grad_(True), b.to(_dev()).requires_grad_(True)
    out = mm(ag, bg)
    tol = 5e-2 if dtype == torch.bfloat16 else 1e-2
    torch.testing.assert_close(out.float().cpu(), ref, atol=tol * 4, rtol=tol)
    g = torch.randn_like(ref)
    ga, gb = torch.autograd.grad(out, (ag, bg), g.to(dtype).to(_dev()))
    ar, br = a.float().requires_grad_(True), b.float().requires_grad_(True)
    ra, rb = torch.autograd.grad(mm(ar, br), (ar, br), g.to(dtype).float())
    torch.testing.assert_close(ga.float().cpu(), ra, atol=tol * 8, rtol=tol)
    torch.testing.assert_close(gb.float().cpu(), rb, atol=tol * 8, rtol=tol)


def test_block_sparse_matmul_strided_views():
    """Operands that are transposed or sliced views go to the kernels as they are."""
    import deeperspeed_amd.ops.sparse_attention as sa
    torch.manual_seed(1)
    H, nb, Z, blk = 2, 4, 2, 32
    S = nb * blk
    lay = _sp_layout(H, nb, 3)
    mm = sa.MatMul(lay, blk, "sdd", trans_a=False, trans_b=True)
    big = torch.randn(Z, H, S, 128, dtype=torch.bfloat16)
    a, b = big[..., :64], big[..., 64:]  # row stride 128, unit k stride
    ref = mm(a.float(), b.float())
    out = mm(a.to(_dev()), b.to(_dev()))
    torch.testing.assert_close(out.float().cpu(), ref, atol=0.2, rtol=5e-2)
    dd = sa.MatMul(lay, blk, "dsd")
    s = torch.randn(Z, int(lay.sum()), blk, blk, dtype=torch.bfloat16) * 0.2
    d = torch.randn(Z, H, 64, S, dtype=torch.bfloat16).transpose(-1, -2)  # [Z,H,S,64], k unit-stride
    torch.testing.assert_close(dd(s.to(_dev()), d.to(_dev())).float().cpu(), dd(s.float(), d.float()),
                               atol=0.2, rtol=5e-2)


@pytest.mark.parametrize("blk,nb,dense", [(16, 8, False), (64, 20, False), (64, 80, True)])
def test_block_sparse_softmax_row_lengths(blk, nb, dense):
    """Rows held in registers (<= 4096 elements) and the online two-pass path (longer rows)."""
    import deeperspeed_amd.ops.sparse_attention as sa
    torch.manual_seed(2)
    H, Z = 1, 1
    S = nb * blk
    lay = torch.ones(H, nb, nb, dtype=torch.long) if dense else _sp_layout(H, nb, 5)
    x = (torch.randn(Z, int(lay.sum()), blk, blk) * 3).to(torch.bfloat16)
    kpm = torch.randn(Z, S).to(torch.bfloat16)
    sm = sa.Softmax(lay, blk)
    ref = sm(x.float(), scale=0.7, key_padding_mask=kpm.float())
    xg = x.to(_dev()).requires_grad_(True)
    y = sm(xg, scale=0.7, key_padding_mask=kpm.to(_dev()))
    torch.testing.assert_close(y.float().cpu(), ref, atol=1e-2, rtol=2e-2)
    g = torch.randn_like(ref).to(torch.bfloat16)
    (gx,) = torch.autograd.grad(y, xg, g.to(_dev()))
    xr = x.float().requires_grad_(True)
    (rx,) = torch.autograd.grad(sm(xr, scale=0.7, key_padding_mask=kpm.float()), xr, g.float())
    torch.testing.assert_close(gx.float().cpu(), rx, atol=2e-2, rtol=3e-2)


@pytest.mark.parametrize("blk", [16, 64])
def test_block_sparse_softmax_and_attention_hip(blk):
    import deeperspeed_amd.ops.sparse_attention as sa
    torch.manual_seed(0)
    H, nb, Z = 2, 4, 2
    S = nb * blk
    lay = _sp_layout(H, nb, 7)
    x = torch.randn(Z, int(lay.sum()), blk, blk).to(torch.bfloat16)
    rpe = torch.randn(1, H, S, S).to(torch.bfloat16)
    kpm = (torch.rand(Z, S) > 0.2).to(torch.bfloat16)
    kpm[:, 0] = 1
    sm = sa.Softmax(lay, blk)
    ref = sm(x.float(), scale=0.5, rpe=rpe.float(), key_padding_mask=kpm.float(), key_padding_mask_mode="mul")
    xg = x.to(_dev()).requires_grad_(True)
    y = sm(xg, scale=0.5, rpe=rpe.to(_dev()), key_padding_mask=kpm.to(_dev()), key_padding_mask_mode="mul")
    torch.testing.assert_close(y.float().cpu(), ref, atol=2e-2, rtol=2e-2)
    g = torch.randn_like(ref).to(torch.bfloat16)
    (gx,) = torch.autograd.grad(y, xg, g.to(_dev()))
    xr = x.float().requires_grad_(True)
    (rx,) = torch.autograd.grad(sm(xr, scale=0.5, rpe=rpe.float(), key_padding_mask=kpm.float(),
                                   key_padding_mask_mode="mul"), xr, g.float())
    torch.testing.assert_close(gx.float().cpu(), rx, atol=3e-2, rtol=3e-2)
    # full module on a Fixed layout, bf16 HIP vs fp32 CPU
    cfg = sa.FixedSparsityConfig(num_heads=4, block=blk, num_local_blocks=2)
    att = sa.SparseSelfAttention(cfg, max_seq_length=S * 2)
    q, k, v = (torch.randn(2, 4, S * 2, 64) for _ in range(3))
    ref = att(q, k, v)
    out = att(*(t.to(torch.bfloat16).to(_dev()) for t in (q, k, v)))
    torch.testing.assert_close(out.float().cpu(), ref, atol=5e-2, rtol=5e-2)


def test_dropout_kernels():
    from deeperspeed_amd.ops import native
    torch.manual_seed(0)
    x = torch.randn(4096, 1024, device=_dev(), dtype=torch.bfloat16)
    y, mask = native.hip_ops().dropout_fwd(x, 0.25, 1234, 0)
    keep = mask.float().mean().item()
    assert abs(keep - 0.75) < 0.01
    torch.testing.assert_close(y.float(), (x.float() * mask / 0.75), atol=1e-2, rtol=1e-2)
    y2, mask2 = native.hip_ops().dropout_fwd(x, 0.25, 1234, 0)
    assert torch.equal(mask, mask2)  # counter-based: reproducible from (seed, offset)
    _, mask3 = native.hip_ops().dropout_fwd(x, 0.25, 1235, 0)
    assert not torch.equal(mask, mask3)
    b = torch.randn(1024, device=_dev(), dtype=torch.bfloat16)
    r = torch.randn_like(x)
    z, m = native.hip_ops().bias_dropout_residual(x, b, r, 0.1, 99, 0)
    torch.testing.assert_close(z.float(), r.float() + (x.float() + b.float()) * m / 0.9, atol=3e-2, rtol=2e-2)
    dx = native.hip_ops().dropout_bwd(y, mask, 0.25)
    torch.testing.assert_close(dx.float(), y.float() * mask / 0.75, atol=1e-2, rtol=1e-2)


@pytest.mark.parametrize("preln", [True, False])
def test_deepspeed_transformer_layer_gpu_vs_cpu(preln):
    import copy
    from deeperspeed_amd.ops.transformer import DeepSpeedTransformerConfig, DeepSpeedTransformerLayer
    torch.manual_seed(0)
    cfg = DeepSpeedTransformerConfig(batch_size=4, hidden_size=256, heads=4, attn_dropout_ratio=0.1,
                                     hidden_dropout_ratio=0.1, num_hidden_layers=4, initializer_range=0.02,
                                     pre_layer_norm=preln, training=False)
    cpu = DeepSpeedTransformerLayer(cfg).eval()
    gpu = copy.deepcopy(cpu).to(_dev()).to(torch.bfloat16)
    x = torch.randn(4, 128, 256)
    m = torch.zeros(4, 1, 1, 128)
    m[1, ..., -20:] = -10000.0
    ref = cpu(x, m)
    xg = x.to(_dev()).to(torch.bfloat16).requires_grad_(True)
    out = gpu(xg, m.to(_dev()).to(torch.bfloat16))
    torch.testing.assert_close(out.float().cpu(), ref, atol=6e-2, rtol=6e-2)
    out.float().sum().backward()
    assert torch.isfinite(xg.grad).all() and gpu.attn_qkvw.grad is not None
    gpu.train()
    y1 = gpu(xg.detach(), m.to(_dev()).to(torch.bfloat16))
    assert torch.isfinite(y1).all()


@pytest.mark.parametrize("D", [64, 96, 128])
@pytest.mark.parametrize("S,causal", [(256, True), (200, False)])
def test_flash_attention_bshd_output(D, S, causal):
    """Token-major output layout ([B,S,H,D], written by the kernel) matches the head-major
    result transposed, forward and backward (dO read token-major)."""
    from deeperspeed_amd.ops import native
    torch.manual_seed(1)
    B, H = 2, 5
    qkv = [torch.randn(B, H, S, D, device=_dev(), dtype=torch.bfloat16) for _ in range(3)]
    a = [t.clone().requires_grad_(True) for t in qkv]
    b = [t.clone().requires_grad_(True) for t in qkv]
    o1 = native.flash_attention(*a, causal, D ** -0.5)
    o2 = native.flash_attention(*b, causal, D ** -0.5, out_layout="bshd")
    assert o2.shape == (B, S, H, D) and o2.is_contiguous()
    torch.testing.assert_close(o2, o1.transpose(1, 2), atol=0, rtol=0)
    do = torch.randn(B, S, H, D, device=_dev(), dtype=torch.bfloat16)
    o1.backward(do.transpose(1, 2))
    o2.backward(do)
    for x, y in zip(a, b):
        torch.testing.assert_close(y.grad, x.grad, atol=0, rtol=0)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("R,C,pad", [(128, 64, 0), (256, 192, 0), (1024, 640, 64), (8192, 512, 0)])
def test_transpose2d_and_fused_colsum(dtype, R, C, pad):
    """HIP transpose (tr-read LDS tiles) is exact; its fused column sum matches fp32 and
    accumulates into an existing bias gradient."""
    from deeperspeed_amd.ops import native
    torch.manual_seed(2)
    base = torch.randn(R, C + pad, device=_dev(), dtype=dtype)
    x = base[:, :C]  # row stride C + pad
    assert native.transpose_supported(x)
    y = native.transpose2d(x)
    assert y.shape == (C, R) and y.is_contiguous()
    torch.testing.assert_close(y, x.t(), atol=0, rtol=0)
    out = torch.randn(C, device=_dev(), dtype=dtype)
    ref = out.float() + x.float().sum(0)
    y2 = native.transpose2d(x, out, accum=True)
    torch.testing.assert_close(y2, y, atol=0, rtol=0)
    torch.testing.assert_close(out.float(), ref, atol=2e-2 * (R ** 0.5), rtol=1e-2)
    out2 = torch.empty(C, device=_dev(), dtype=dtype)
    native.transpose2d(x, out2, accum=False)
    torch.testing.assert_close(out2.float(), x.float().sum(0), atol=2e-2 * (R ** 0.5), rtol=1e-2)


@pytest.mark.parametrize("bound", [True, False])
def test_linear_wgrad_transposed_operands(bound):
    """dW / db / dx from the reduction-contiguous (transposed) operands match the token-major
    formulation and an fp32 reference, in place (bound grad) and through autograd."""
    from deeperspeed_amd.ops import linear as lin
    torch.manual_seed(3)
    old = lin.WGRAD_NT_MIN_NUMEL
    lin.WGRAD_NT_MIN_NUMEL = 0
    try:
        M, fin, fout = 1024, 384, 640
        x0 = torch.randn(2, M // 2, fin, device=_dev(), dtype=torch.bfloat16)
        g = torch.randn(2, M // 2, fout, device=_dev(), dtype=torch.bfloat16)
        res = {}
        for nt in (False, True):
            lin.WGRAD_NT = lin.DGRAD_NT = nt
            layer = lin.Linear(fin, fout, device=_dev(), dtype=torch.bfloat16)
            torch.manual_seed(4)
            with torch.no_grad():
                layer.weight.normal_()
                layer.bias.normal_()
            if bound:
                layer.weight.grad = torch.zeros_like(layer.weight)
                layer.bias.grad = torch.zeros_like(layer.bias)
            x = x0.clone().requires_grad_(True)
            n0 = lin.nt_wgrad_count()
            layer(x).backward(g)
            assert (lin.nt_wgrad_count() > n0) == nt
            res[nt] = (layer.weight.grad.float(), layer.bias.grad.float(), x.grad.float(), layer.weight.float())
        ref_w = g.reshape(M, fout).float().t() @ x0.reshape(M, fin).float()
        ref_b = g.reshape(M, fout).float().sum(0)
        for nt in (False, True):
            ref_x = g.float() @ res[nt][3]
            torch.testing.assert_close(res[nt][0], ref_w, atol=0.5, rtol=2e-2)
            torch.testing.assert_close(res[nt][1], ref_b, atol=0.5, rtol=2e-2)
            torch.testing.assert_close(res[nt][2], ref_x, atol=0.5, rtol=2e-2)
    finally:
        lin.WGRAD_NT = lin.DGRAD_NT = True
        lin.WGRAD_NT_MIN_NUMEL = old


@pytest.mark.parametrize("gdt", [torch.float32, torch.bfloat16])
def test_multi_tensor_lamb_matches_per_tensor(gdt):
    """FusedLamb's multi-tensor launches (per-chunk partial norms, per-tensor trust ratio)
    equal the per-tensor kernels: weights, moments, bf16 output copies and coefficients."""
    from deeperspeed_amd.ops.lamb import FusedLamb
    torch.manual_seed(5)
    shapes = [(1000,), (300, 257), (65536 * 2 + 5,), (7,), (1024, 64)]
    res = {}
    for multi in (False, True):
        torch.manual_seed(5)
        ps = [torch.randn(*s, device=_dev()).requires_grad_(True) for s in shapes]
        opt = FusedLamb(ps, lr=1e-2, weight_decay=0.01, max_coeff=10.0, min_coeff=0.01)
        opt.multi_tensor = multi
        outs = [torch.empty(p.shape, device=_dev(), dtype=torch.bfloat16) for p in ps]
        for it in range(3):
            grads = [torch.randn_like(p).to(gdt) for p in ps]
            opt.step(grads=[grads], output_params=[outs], scale=2.0)
        res[multi] = ([p.detach().clone() for p in ps], [o.clone() for o in outs],
                      [opt.state[p]["exp_avg_sq"].clone() for p in ps], opt.get_lamb_coeffs())
    for a, b in zip(res[False][0], res[True][0]):
        torch.testing.assert_close(b, a, atol=1e-6, rtol=1e-5)
    for a, b in zip(res[False][1], res[True][1]):
        torch.testing.assert_close(b.float(), a.float(), atol=1e-2, rtol=1e-2)
    for a, b in zip(res[False][2], res[True][2]):
        torch.testing.assert_close(b, a, atol=1e-7, rtol=1e-5)
    assert len(res[True][3]) == len(shapes)
    torch.testing.assert_close(torch.tensor(res[True][3]), torch.tensor(res[False][3]), atol=1e-5, rtol=1e-4)


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_bert_head_layout_kernels(dt):
    """heads_split / heads_merge / swap12 equal the torch permute copies exactly (fwd and bwd)."""
    from deeperspeed_amd.ops import native
    torch.manual_seed(6)
    B, S, nh, hd = 3, 40, 4, 64
    qkv = torch.randn(B, S, 3 * nh * hd, device=_dev(), dtype=dt)
    q, k, v = native.hip_ops().heads_split(qkv, nh)
    ref = qkv.view(B, S, 3, nh, hd).permute(2, 0, 3, 1, 4)
    for i, t in enumerate((q, k, v)):
        torch.testing.assert_close(t, ref[i].contiguous(), atol=0, rtol=0)
    back = native.hip_ops().heads_merge(q, k, v)
    torch.testing.assert_close(back, qkv, atol=0, rtol=0)
    x = torch.randn(B, nh, S, hd, device=_dev(), dtype=dt)
    torch.testing.assert_close(native.hip_ops().swap12(x), x.transpose(1, 2).contiguous(), atol=0, rtol=0)


def test_transformer_layer_head_kernels_match_permute_path(monkeypatch):
    """DeepSpeedTransformerLayer with the HIP head-layout kernels matches the torch permute path
    (forward output and every gradient) on bf16 with a padding mask and dropout off."""
    from deeperspeed_amd.ops.transformer import DeepSpeedTransformerConfig, DeepSpeedTransformerLayer
    from deeperspeed_amd.ops.transformer import transformer as tmod
    torch.manual_seed(7)
    cfg = DeepSpeedTransformerConfig(batch_size=2, hidden_size=256, intermediate_size=1024, heads=4,
                                     attn_dropout_ratio=0.0, hidden_dropout_ratio=0.0, num_hidden_layers=2,
                                     initializer_range=0.02, pre_layer_norm=True, bf16=True)
    layer = DeepSpeedTransformerLayer(cfg).to(_dev())
    x = torch.randn(2, 64, 256, device=_dev(), dtype=torch.bfloat16)
    mask = torch.zeros(2, 1, 1, 64, device=_dev(), dtype=torch.bfloat16)
    mask[1, ..., 48:] = -10000.0
    res = {}
    for fast in (True, False):
        monkeypatch.setattr(tmod, "_use_head_kernels", lambda t, hd, _f=fast: _f)
        layer.zero_grad(set_to_none=True)
        xi = x.clone().requires_grad_(True)
        out = layer(xi, mask)
        out.float().pow(2).sum().backward()
        res[fast] = [out.detach().float(), xi.grad.float()] + [p.grad.float() for p in layer.parameters()]
    # the fast path also takes the fused encoder attention: bf16 round-off differs from the
    # materialised softmax path, so compare against each tensor's magnitude
    for a, b in zip(res[True], res[False]):
        assert (a - b).abs().max().item() <= 3e-2 * max(1.0, b.abs().max().item())


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16, torch.float32])
def test_add3_matches_reference(dtype):
    from deeperspeed_amd.ops import native
    torch.manual_seed(0)
    dev = torch.device("cuda")
    a, b, c = (torch.randn(4, 512, 768, device=dev, dtype=dtype) for _ in range(3))
    ref = a.float() + b.float() + c.float()
    # one rounding of the fp32 sum: error within half an ulp of the result's magnitude
    half_ulp = {torch.bfloat16: 2.0 ** -8, torch.float16: 2.0 ** -11, torch.float32: 2.0 ** -23}[dtype]
    err = (native.hip_ops().add3(a, b, c).float() - ref).abs()
    assert bool((err <= half_ulp * ref.abs() * 1.01 + 1e-6).all())
    ref2 = a.float() + b.float()
    err2 = (native.hip_ops().add3(a, b).float() - ref2).abs()
    assert bool((err2 <= half_ulp * ref2.abs() * 1.01 + 1e-6).all())
    xs = [t.clone().requires_grad_(True) for t in (a, b, c)]
    native.add3(*xs).float().sum().backward()
    assert all(torch.equal(x.grad, torch.ones_like(x)) for x in xs)


def _enc_reference(q, k, v, bias, scale, keep, p):
    s = (q.float() @ k.float().transpose(-1, -2)) * scale
    if bias is not None:
        s = s + bias.float()[:, None, None, :]
    pr = torch.softmax(s, -1)
    if keep is not None:
        pr = pr * keep.float() / (1.0 - p)
    return pr @ v.float()


@pytest.mark.parametrize("D", [64, 128])
@pytest.mark.parametrize("S,p", [(128, 0.0), (128, 0.1), (96, 0.1), (64, 0.0), (200, 0.1), (512, 0.25)])
def test_encoder_flash_bias_dropout(D, S, p):
    """Encoder flash (non-causal, key-padding bias, in-kernel dropout) against an fp32 reference
    that applies the kernel's own keep mask (native.flash_dropout_keep_mask)."""
    from deeperspeed_amd.ops import native
    torch.manual_seed(0)
    dev = torch.device("cuda")
    B, H = 2, 3
    q, k, v = (torch.randn(B, H, S, D, device=dev, dtype=torch.bfloat16) for _ in range(3))
    bias = torch.zeros(B, S, device=dev)
    bias[0, -7:] = -10000.0
    bias[1, : S // 3] = -10000.0
    scale = D ** -0.5
    seed = 1234567
    keep = native.flash_dropout_keep_mask(B, H, S, p, seed, device=dev) if p > 0 else None
    qs, ks, vs = (t.clone().requires_grad_(True) for t in (q, k, v))
    seed_fn = native._draw_seed
    try:
        native._draw_seed = lambda generator=None: seed
        o = native.flash_attention_encoder(qs, ks, vs, bias, scale, p, True, out_layout="bshd")
    finally:
        native._draw_seed = seed_fn
    g = torch.randn(B, S, H, D, device=dev)
    (o.float() * g).sum().backward()
    qr, kr, vr = (t.float().clone().requires_grad_(True) for t in (q, k, v))
    ref = _enc_reference(qr, kr, vr, bias, scale, keep, p)
    (ref * g.transpose(1, 2)).sum().backward()
    assert (o.float().transpose(1, 2) - ref).abs().max().item() < 3e-2
    for a, b in ((qs.grad, qr.grad), (ks.grad, kr.grad), (vs.grad, vr.grad)):
        err = (a.float() - b).abs().max().item()
        assert err < 5e-2 * max(1.0, b.abs().max().item()), err
    if p > 0:
        rate = 1.0 - keep.float().mean().item()
        assert abs(rate - p) < 0.01


def test_encoder_flash_dropout_only_and_eval():
    """Dropout without a bias; in eval mode the call is plain non-causal flash attention."""
    from deeperspeed_amd.ops import native
    torch.manual_seed(1)
    dev = torch.device("cuda")
    q, k, v = (torch.randn(2, 4, 256, 64, device=dev, dtype=torch.bfloat16) for _ in range(3))
    ref = _enc_reference(q, k, v, None, 0.125, None, 0.0)
    o = native.flash_attention_encoder(q, k, v, None, 0.125, 0.1, training=False)
    assert (o.float() - ref).abs().max().item() < 3e-2
    gen = torch.Generator().manual_seed(3)
    o1 = native.flash_attention_encoder(q, k, v, None, 0.125, 0.1, True, generator=gen)
    gen = torch.Generator().manual_seed(3)
    o2 = native.flash_attention_encoder(q, k, v, None, 0.125, 0.1, True, generator=gen)
    assert torch.equal(o1, o2)  # same generator state -> same keep mask
    assert (o1.float() - ref).abs().max().item() > 1e-2  # dropout was applied


@pytest.mark.parametrize("out_f32", [False, True])
@pytest.mark.parametrize("accumulate", [False, True])
def test_sum_slices_and_colsum_accumulate(out_f32, accumulate):
    """Split-K fold (sum of bf16 partial slices, fp32 accumulation) and column sums into /
    onto an existing output."""
    from deeperspeed_amd.ops import native
    torch.manual_seed(0)
    dev = _dev()
    part = torch.randn(4, 384, 1024, device=dev, dtype=torch.bfloat16)
    out = torch.randn(384, 1024, device=dev, dtype=torch.float32 if out_f32 else torch.bfloat16)
    ref = part.float().sum(0) + (out.float() if accumulate else 0.0)
    native.hip_ops().sum_slices(part, out, accumulate)
    tol = 1e-5 if out_f32 else 2e-2
    assert (out.float() - ref).abs().max().item() <= tol * max(1.0, ref.abs().max().item())
    x = torch.randn(3000, 1024, device=dev, dtype=torch.bfloat16)
    acc = torch.randn(1024, device=dev, dtype=torch.bfloat16)
    want = x.float().sum(0) + (acc.float() if accumulate else 0.0)
    got = native.colsum(x, acc, accumulate=accumulate)
    assert got.data_ptr() == acc.data_ptr()
    assert (got.float() - want).abs().max().item() <= 2e-2 * want.abs().max().item()


@pytest.mark.parametrize("S", [128, 256, 512])
@pytest.mark.parametrize("p", [0.0, 0.1])
def test_qkv_layout_flash_matches_head_major(p, S):
    """Encoder flash attention reading q, k, v straight from the fused QKV output (and writing
    dqkv in that layout) equals the head-major path bit for bit (same kernels, same keep mask)."""
    from deeperspeed_amd.ops import native
    torch.manual_seed(2)
    dev = _dev()
    B, H, D = 3, 4, 64
    qkv = torch.randn(B, S, 3 * H * D, device=dev, dtype=torch.bfloat16)
    bias = torch.zeros(B, S, device=dev)
    bias[1, -40:] = -10000.0
    g = torch.randn(B, S, H * D, device=dev, dtype=torch.bfloat16)
    seed_fn = native._draw_seed
    try:
        native._draw_seed = lambda generator=None: 987654321
        a = qkv.clone().requires_grad_(True)
        oa = native.flash_attention_qkv(a, H, bias, D ** -0.5, p, True)
        (oa.float() * g.float()).sum().backward()
        b = qkv.clone().requires_grad_(True)
        q, k, v = b.view(B, S, 3, H, D).permute(2, 0, 3, 1, 4)
        ob = native.flash_attention_encoder(q, k, v, bias, D ** -0.5, p, True, out_layout="bshd").reshape(B, S, H * D)
        (ob.float() * g.float()).sum().backward()
    finally:
        native._draw_seed = seed_fn
    assert torch.equal(oa, ob)
    assert torch.equal(a.grad, b.grad)


@pytest.mark.parametrize("C", [1024, 4096, 264])
def test_dropout_bwd_with_bias_grad(C):
    """Dropout backward fused with the bias-gradient column sums equals mask * dy / (1-p) and
    its column sums."""
    from deeperspeed_amd.ops import native
    torch.manual_seed(1)
    dev = _dev()
    dy = torch.randn(2000, C, device=dev, dtype=torch.bfloat16)
    mask = (torch.rand(2000, C, device=dev) >= 0.1).to(torch.uint8)
    dx, db = native.hip_ops().dropout_bwd_db(dy, mask, 0.1)
    ref = dy.float() * mask.float() / 0.9
    assert (dx.float() - ref).abs().max().item() < 2e-2 * ref.abs().max().item()
    want = ref.sum(0)
    assert (db.float() - want).abs().max().item() < 2e-2 * want.abs().max().item()


def test_cross_entropy_inplace_grad():
    """inplace_grad: dlogits written over the (internal) logits give the same input gradients,
    and a second backward through the graph fails loudly instead of reading gradients."""
    from deeperspeed_amd.ops import native
    torch.manual_seed(5)
    V = 50432
    h = torch.randn(64, 256, device=_dev(), dtype=torch.bfloat16, requires_grad=True)
    w = (0.05 * torch.randn(V, 256, device=_dev())).to(torch.bfloat16).requires_grad_(True)
    lab = torch.randint(0, V, (64,), device=_dev())
    grads = []
    for inplace in (False, True):
        h.grad = w.grad = None
        loss = native.cross_entropy(h @ w.t(), lab, inplace_grad=inplace)
        loss.backward()
        grads.append((float(loss), h.grad.clone(), w.grad.clone()))
    assert grads[0][0] == grads[1][0]
    torch.testing.assert_close(grads[0][1], grads[1][1], atol=0, rtol=0)
    torch.testing.assert_close(grads[0][2], grads[1][2], atol=0, rtol=0)
    loss = native.cross_entropy(h @ w.t(), lab, inplace_grad=True)
    loss.backward(retain_graph=True)
    with pytest.raises(RuntimeError):
        loss.backward()


@pytest.mark.parametrize("V,pattern", [(50432, "random"), (30528, "padding-heavy"), (2, "token-type"),
                                       (512, "positions")])
@pytest.mark.parametrize("padding_idx", [None, 0])
def test_embedding_backward_sync_free(V, pattern, padding_idx):
    """Sorted-run embedding backward (embedding.hip): equals the fp32 scatter-sum of the output
    gradient rows, including runs that span many chunks (padding / token types), padding_idx,
    and accumulation into an already bound weight gradient; bit-stable across calls."""
    from deeperspeed_amd.ops.native import Embedding
    torch.manual_seed(11)
    H, n = 1024, 8192
    if pattern == "random":
        ids = torch.randint(0, V, (n,), device=_dev())
    elif pattern == "padding-heavy":  # half the tokens are id 0, the rest random
        ids = torch.randint(0, V, (n,), device=_dev())
        ids[torch.rand(n, device=_dev()) < 0.5] = 0
    elif pattern == "token-type":
        ids = (torch.arange(n, device=_dev()) % 128 >= 64).long()
    else:
        ids = torch.arange(n, device=_dev()) % V
    ids = ids.view(64, n // 64)
    emb = Embedding(V, H, padding_idx=padding_idx, device=_dev(), dtype=torch.bfloat16)
    dy = torch.randn(64, n // 64, H, device=_dev(), dtype=torch.bfloat16)
    ref = torch.zeros(V, H, device=_dev(), dtype=torch.float32)
    ref.index_add_(0, ids.reshape(-1), dy.reshape(-1, H).float())
    if padding_idx is not None:
        ref[padding_idx] = 0
    emb(ids).backward(dy)
    g1 = emb.weight.grad.clone()
    assert torch.allclose(g1.float(), ref, atol=3e-2, rtol=1e-2)
    emb(ids).backward(dy)  # bound gradient: accumulated in place
    assert torch.allclose(emb.weight.grad.float(), 2 * ref, atol=6e-2, rtol=2e-2)
    emb.weight.grad = None
    emb(ids).backward(dy)
    assert torch.equal(emb.weight.grad, g1)  # deterministic


def test_embedding_backward_int32_ids():
    """nn.Embedding accepts int32 ids; the HIP backward (int64 sorted ids) widens them first
    (ADVICE r3): same gradient as int64 ids."""
    from deeperspeed_amd.ops.native import Embedding
    torch.manual_seed(3)
    V, H = 4096, 256
    ids = torch.randint(0, V, (8, 512), device=_dev())
    dy = torch.randn(8, 512, H, device=_dev(), dtype=torch.bfloat16)
    grads = []
    for dt in (torch.int64, torch.int32):
        emb = Embedding(V, H, device=_dev(), dtype=torch.bfloat16)
        emb(ids.to(dt)).backward(dy)
        grads.append(emb.weight.grad.clone())
    assert torch.equal(grads[0], grads[1])
