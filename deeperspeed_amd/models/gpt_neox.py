"""GPT-NeoX family (flagship model of the framework).

Architecture as trained with DeeperSpeed by GPT-NeoX: pre-LayerNorm blocks with *parallel*
attention + MLP residual (`x + attn(ln1(x)) + mlp(ln2(x))`), partial rotary position
embedding (rotary_pct of each head), GeLU MLP of width 4h, untied input/output
embeddings, final LayerNorm.  Presets include GPT-NeoX-20B (the north-star config of
BASELINE.json), 1.3B and GPT-3-6.7B-shaped models.

Hot ops run on the framework's HIP kernels (LayerNorm, bias+GeLU, fused rotary/QKV split,
fused attention softmax or flash attention); GEMMs use hipBLASLt through torch.
Layers are plain modules so the same blocks serve `DeepSpeedEngine` (ZeRO-1/2/3) and the
pipeline engine (`to_pipeline()` builds a PipelineModule of LayerSpecs).
"""

from __future__ import annotations

import math
from dataclasses import dataclass, field, asdict
from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops import native
from ..ops.linear import Linear, grad_only_linear, linear, nt_wgrad_planned, zero_placeholder
from ..ops.attention import attention, rotary_split
from ..runtime.activation_checkpointing import checkpointing as ds_ckpt


@dataclass
class GPTNeoXConfig:
    vocab_size: int = 50432
    hidden_size: int = 6144
    num_layers: int = 44
    num_heads: int = 64
    intermediate_size: Optional[int] = None
    rotary_pct: float = 0.25
    rotary_base: float = 10000.0
    max_seq_len: int = 2048
    layernorm_eps: float = 1e-5
    use_parallel_residual: bool = True
    gelu_approximate: bool = False
    checkpoint_activations: bool = True
    init_std: float = 0.02
    hidden_dropout: float = 0.0
    attention_dropout: float = 0.0
    # block-sparse attention (GPT-NeoX `attention_config` sparse types), e.g.
    # {"mode": "bigbird", "block": 64, "num_random_blocks": 1, "num_sliding_window_blocks": 3}
    sparse_attention: Optional[dict] = None

    def __post_init__(self):
        if self.intermediate_size is None:
            self.intermediate_size = 4 * self.hidden_size
        assert self.hidden_size % self.num_heads == 0
        rot = int(self.head_dim * self.rotary_pct)
        self.rotary_dim = rot - rot % 2

    @property
    def head_dim(self):
        return self.hidden_size // self.num_heads

    def num_params(self, include_embeddings=True):
        h, i, L, V = self.hidden_size, self.intermediate_size, self.num_layers, self.vocab_size
        per_layer = 3 * h * h + 3 * h + h * h + h + 2 * h * i + i + h + 4 * h
        n = L * per_layer + 2 * h
        if include_embeddings:
            n += 2 * V * h
        return n

    def flops_per_token(self, seq_len=None, recompute=True):
        """Model FLOPs per trained token (fwd+bwd[+recompute]) incl. attention.  With block-sparse
        attention only the layout's active score elements are counted (attention_density)."""
        s = seq_len or self.max_seq_len
        n = self.num_params(include_embeddings=False) + self.vocab_size * self.hidden_size  # output proj GEMM
        attn = 2 * self.num_layers * s * self.hidden_size  # QK^T + PV per token (causal halves, x2 fwd terms)
        attn *= self.attention_density(s)
        mult = 8 if recompute else 6
        return mult * n + (mult // 2) * attn

    def attention_density(self, seq_len=None) -> float:
        """Fraction of the causal score triangle (s^2/2 elements) the attention computes: 1.0
        dense; for a block-sparse layout the active blocks, diagonal blocks counted half."""
        if not self.sparse_attention:
            return 1.0
        s = seq_len or self.max_seq_len
        sc = make_sparsity_config(self)
        lay = sc.make_layout(s).bool()
        nb = lay.shape[-1]
        lower = torch.tril(torch.ones(nb, nb, dtype=torch.bool), diagonal=-1)
        diag = torch.eye(nb, dtype=torch.bool)
        active = (lay & lower).sum().item() + 0.5 * (lay & diag).sum().item()
        return float(active / lay.shape[0] * sc.block ** 2 / (s * s / 2.0))


PRESETS = {
    "gpt-neox-20b": dict(vocab_size=50432, hidden_size=6144, num_layers=44, num_heads=64, rotary_pct=0.25),
    "gpt-neox-1.3b": dict(vocab_size=50304, hidden_size=2048, num_layers=24, num_heads=16, rotary_pct=0.25),
    "gpt-neox-125m": dict(vocab_size=50304, hidden_size=768, num_layers=12, num_heads=12, rotary_pct=0.25),
    "gpt3-6.7b": dict(vocab_size=50304, hidden_size=4096, num_layers=32, num_heads=32, rotary_pct=1.0),
    "tiny": dict(vocab_size=512, hidden_size=128, num_layers=2, num_heads=4, rotary_pct=0.25, max_seq_len=64),
}


def get_config(name: str, **overrides) -> GPTNeoXConfig:
    d = dict(PRESETS[name])
    d.update(overrides)
    return GPTNeoXConfig(**d)


class LinearBiasGeLU(nn.Linear):
    """dense_h_to_4h: GEMM without bias, then the fused bias+GeLU HIP kernel.  Keeping the
    whole op inside this module's forward matters for ZeRO-3: a module's parameters are
    gathered by its own forward hooks, so they must not be touched from a parent's forward."""

    def __init__(self, in_features, out_features, approximate=False, device=None, dtype=None):
        super().__init__(in_features, out_features, device=device, dtype=dtype)
        self.approximate = approximate
        # set by NeoXMLP when the consumer is a gradient-only linear during recompute: the
        # activation is then produced transposed (its only reader is that linear's weight
        # gradient, which wants it reduction-contiguous)
        self.colmajor_in_recompute = False
        self.keep_u = False  # MLP stash: hand the GEMM output to the caller (kept_u) on this forward
        self.kept_u = None
        self.stashed_u = None  # MLP stash: the next forward reuses this GEMM output (gradient-only GEMM)

    def forward(self, x):
        if self.stashed_u is not None:
            u_st, self.stashed_u = self.stashed_u, None
            u = _StashInject.apply(grad_only_linear(x, self.weight), u_st)
        else:
            u = linear(x, self.weight)
            if self.keep_u:
                self.kept_u = u
        if (self.colmajor_in_recompute and _SKIP_OUTPUTS and torch.is_grad_enabled() and COLMAJOR_GELU
                and native.bias_gelu_t_supported(u)):
            return native.bias_gelu_colmajor(u, self.bias, self.approximate)
        # the backward also writes du^T when this layer's own weight gradient will read it
        offer = u.is_cuda and nt_wgrad_planned(u.numel() // self.out_features, self.out_features, self.in_features,
                                               u.element_size(), g_ready=True)
        return native.bias_gelu(u, self.bias, self.approximate, offer_t=offer)




# the recompute writes the GeLU output column-major for fc2's weight gradient (False: row-major,
# fc2's wgrad transposes it; tests' A/B)
COLMAJOR_GELU = True

_SKIP_OUTPUTS = 0


class skip_unread_outputs:
    """Context for the recompute of ONE checkpointed block whose result is the checkpoint's
    own output: inside it, OutputLinear layers flagged `skip_in_recompute` produce gradients
    only.  (Never set for multi-block checkpoint segments, where block i's output is block
    i+1's input.)"""

    def __enter__(self):
        global _SKIP_OUTPUTS
        _SKIP_OUTPUTS += 1

    def __exit__(self, *exc):
        global _SKIP_OUTPUTS
        _SKIP_OUTPUTS -= 1


class _GradOnlySum(torch.autograd.Function):
    """Residual sum whose value is never read (the recomputed block output): no kernel in
    forward, the incoming gradient passed to every summand in backward."""

    @staticmethod
    def forward(ctx, *xs):
        ctx.n = len(xs)
        return zero_placeholder(xs[0], xs[0].shape)

    @staticmethod
    def backward(ctx, g):
        return (g,) * ctx.n


def residual_sum(*xs):
    """x + branch outputs; inside skip_unread_outputs() (the recompute of a checkpointed block,
    whose output only seeds backward) the two full-tensor adds are skipped."""
    if _SKIP_OUTPUTS and torch.is_grad_enabled():
        return _GradOnlySum.apply(*xs)
    if len(xs) <= 3:
        return native.add3(*xs)  # one fused HIP pass on the GPU
    out = xs[0] + xs[1]
    for x in xs[2:]:
        out = out + x
    return out


class _StashInject(torch.autograd.Function):
    """Value of `stashed`, gradient routed to `placeholder` (a gradient-only GEMM whose output
    the first forward already computed and kept)."""

    @staticmethod
    def forward(ctx, placeholder, stashed):
        return stashed.view(stashed.shape)

    @staticmethod
    def backward(ctx, g):
        return g, None


class OutputLinear(nn.Linear):
    """Final projection of a residual branch (attention `dense` with parallel residual, MLP
    `dense_4h_to_h`).

    Its output only enters the block's residual sum, which no backward reads.  During the
    block's activation recompute (inside backward) the GEMM is therefore skipped and only
    gradients are formed: that removes ~20 % of the recomputed forward FLOPs of a GPT-NeoX
    block."""

    skip_in_recompute = True
    # parallel residual: attention `dense` and MLP `dense_4h_to_h` receive the same output
    # gradient; the first weight gradient's transpose of it is reused by the second.
    # share_partner = the other projection's (out, in), set by the layer.
    share_partner = None

    def _share(self, x):
        if self.share_partner is None or not x.is_cuda:
            return False
        M = x.numel() // x.shape[-1]
        return all(nt_wgrad_planned(M, o, i, x.element_size())
                   for o, i in ((self.out_features, self.in_features), self.share_partner))

    def forward(self, x):
        if _SKIP_OUTPUTS and self.skip_in_recompute and torch.is_grad_enabled():
            return grad_only_linear(x, self.weight, self.bias, self._share(x))
        return linear(x, self.weight, self.bias, self._share(x))


def make_sparsity_config(cfg: GPTNeoXConfig):
    """Causal (unidirectional) SparsityConfig from cfg.sparse_attention."""
    from ..ops import sparse_attention as sa
    d = dict(cfg.sparse_attention)
    mode = d.pop("mode", "bigbird").lower()
    classes = {"fixed": sa.FixedSparsityConfig, "variable": sa.VariableSparsityConfig,
               "bigbird": sa.BigBirdSparsityConfig, "bslongformer": sa.BSLongformerSparsityConfig,
               "local": sa.LocalSlidingWindowSparsityConfig, "dense": sa.DenseSparsityConfig}
    cls = classes[mode]
    if mode != "dense":
        d.setdefault("attention", "unidirectional")
    return cls(num_heads=cfg.num_heads, **d)


class NeoXAttention(nn.Module):
    def __init__(self, cfg: GPTNeoXConfig, device=None, dtype=None, layer_number: int = 0):
        super().__init__()
        h = cfg.hidden_size
        self.cfg = cfg
        self.layer_number = layer_number
        self._sparsity = make_sparsity_config(cfg) if cfg.sparse_attention else None
        self._sp_ops = {}
        self.query_key_value = Linear(h, 3 * h, device=device, dtype=dtype)
        self.dense = OutputLinear(h, h, device=device, dtype=dtype)
        # with a sequential residual the attention output feeds post_attention_layernorm
        self.dense.skip_in_recompute = cfg.use_parallel_residual
        # Selective recompute (set per layer by the trainer when HBM allows): the first forward
        # of a checkpointed block keeps q, k, v and the attention output + LSE (4 s*b*h + LSE),
        # and the recompute in backward reuses them, skipping the QKV GEMM, the rotary split and
        # the flash forward (~1.8 ms per 20B layer and micro-batch of 4x2048 on MI355X).
        # Stashes are keyed by the checkpointed block's input (its storage is held by the
        # checkpoint until that block's backward, and the recompute sees a detached view of the
        # same storage), so several forwards in flight before their backwards (pipeline 1F1B,
        # forward-forward-backward loops) each recompute with their own tensors.
        self.stash_outputs = False
        # stash_offload: the stash is parked in pinned host memory between the forward and the
        # recompute (runtime/activation_checkpointing/host_stash.py) -- for layers beyond the
        # HBM budget; the recompute of the layer above prefetches it back
        self.stash_offload = False
        self._stash = {}
        self._stash_key = None  # set by the enclosing layer around each block call
        self.__dict__["_below"] = []  # attention modules of the next layers in backward order

    _STASH_LIMIT = 16  # in-flight checkpointed forwards per layer (pipeline depth bound)

    def forward(self, x):
        cfg = self.cfg
        B, S, H = x.shape
        qs = 1.0 / math.sqrt(cfg.head_dim)
        key = self._stash_key
        stash = self._stash.pop(key, None) if (key is not None and self._stash and torch.is_grad_enabled()
                                               and ds_ckpt.is_recomputing()) else None
        if stash is not None:
            from ..runtime.activation_checkpointing.host_stash import StashEntry, host_stash
            if isinstance(stash, StashEntry):
                stash = host_stash().fetch(stash)
            for below in self.__dict__["_below"]:  # start bringing the next layers' stashes back
                for e in below._stash.values():
                    if isinstance(e, StashEntry):
                        host_stash().prefetch(e)
            self.query_key_value.grad_only_next = True  # gradient handle only: q, k, v are kept
            qkv = self.query_key_value(x)
            q, k, v = rotary_split(qkv, cfg.num_heads, cfg.head_dim, cfg.rotary_dim, cfg.rotary_base, qscale=qs,
                                   stash=stash[:3])
            if self._sparsity is not None:
                from ..ops.sparse_attention import flash as sflash
                ctx = sflash.sparse_flash_attention(q, k, v, self._sparse_ops(S)[3], 1.0, out_bshd=True,
                                                    stash=stash[3:])
            else:
                ctx = native.flash_attention(q, k, v, True, 1.0, out_layout="bshd", stash=stash[3:])
            return self.dense(ctx.reshape(B, S, H))
        qkv = self.query_key_value(x)
        q, k, v = rotary_split(qkv, cfg.num_heads, cfg.head_dim, cfg.rotary_dim, cfg.rotary_base, qscale=qs)
        if self._sparsity is not None:
            ctx = self._sparse_attention(q, k, v, key)
            if ctx.shape[1] == S:  # fused kernel wrote the token-major [B, S, H, D] layout
                return self.dense(ctx.reshape(B, S, H))
        else:
            if (self.stash_outputs and ds_ckpt.is_checkpoint_forward() and cfg.attention_dropout == 0.0
                    and native.has_flash_attention(q)):
                ctx, lse = native.flash_attention_fwd_lse(q, k, v, True, 1.0, out_layout="bshd")
                if key is not None:
                    if key in self._stash or len(self._stash) >= self._STASH_LIMIT:
                        raise RuntimeError(f"layer {self.layer_number}: selective-recompute stash for this input "
                                           f"was never consumed (forward without backward?)")
                    if self.stash_offload:
                        from ..runtime.activation_checkpointing.host_stash import host_stash
                        self._stash[key] = host_stash().park(id(self), (q, k, v, ctx, lse))
                    else:
                        self._stash[key] = (q, k, v, ctx, lse)
            else:
                ctx = attention(q, k, v, causal=True, softmax_scale=1.0, dropout_p=cfg.attention_dropout,
                                training=self.training, out_layout="bshd")
            return self.dense(ctx.reshape(B, S, H))  # [B,S,NH,HD] written by the kernel: free view
        ctx = ctx.transpose(1, 2).reshape(B, S, H)
        return self.dense(ctx)


    def _sparse_ops(self, S):
        if S not in self._sp_ops:
            import random
            from ..ops.sparse_attention import MatMul, Softmax
            state = random.getstate()
            random.seed(1234 + self.layer_number)  # identical random blocks on every rank
            layout = self._sparsity.make_layout(S)
            random.setstate(state)
            blk = self._sparsity.block
            from ..ops.sparse_attention.flash import SparseFlashLUT
            try:  # fused LUT-walk kernel (ops/sparse_attention/flash.py); else SDD / softmax / DSD
                lut = SparseFlashLUT(layout, blk, causal=True)
            except ValueError:
                lut = None
            self._sp_ops[S] = (MatMul(layout, blk, "sdd", trans_b=True), MatMul(layout, blk, "dsd"),
                               Softmax(layout, blk), lut)
        return self._sp_ops[S]

    def _sparse_attention(self, q, k, v, key=None):
        """Block-sparse causal attention (q is pre-scaled).  On the GPU one fused kernel walks the
        layout's active tiles and returns [B, S, H, D]; otherwise SDD -> causal sparse softmax ->
        DSD returns [B, H, S, D].  With stash_outputs, the checkpointed first forward keeps q, k,
        v, the output and the LSE for the recompute (as the dense path does)."""
        sdd, dsd, softmax, lut = self._sparse_ops(q.shape[2])
        from ..ops.sparse_attention import flash as sflash
        if self.cfg.attention_dropout == 0.0 and sflash.supported(q, lut):
            if self.stash_outputs and ds_ckpt.is_checkpoint_forward() and key is not None:
                ctx, lse = sflash.sparse_flash_fwd_lse(q, k, v, lut, 1.0, out_bshd=True)
                if key in self._stash or len(self._stash) >= self._STASH_LIMIT:
                    raise RuntimeError(f"layer {self.layer_number}: selective-recompute stash for this input "
                                       f"was never consumed (forward without backward?)")
                if self.stash_offload:
                    from ..runtime.activation_checkpointing.host_stash import host_stash
                    self._stash[key] = host_stash().park(id(self), (q, k, v, ctx, lse))
                else:
                    self._stash[key] = (q, k, v, ctx, lse)
                return ctx
            return sflash.sparse_flash_attention(q, k, v, lut, 1.0, out_bshd=True)
        w = softmax(sdd(q, k), scale=1.0, causal=True)
        return dsd(w, v)


class NeoXMLP(nn.Module):
    def __init__(self, cfg: GPTNeoXConfig, device=None, dtype=None):
        super().__init__()
        self.cfg = cfg
        self.dense_h_to_4h = LinearBiasGeLU(cfg.hidden_size, cfg.intermediate_size, cfg.gelu_approximate,
                                            device=device, dtype=dtype)
        self.dense_4h_to_h = OutputLinear(cfg.intermediate_size, cfg.hidden_size, device=device, dtype=dtype)
        self.dense_h_to_4h.colmajor_in_recompute = self.dense_4h_to_h.skip_in_recompute
        # Selective MLP recompute (set per layer by the trainer when HBM allows, after the
        # attention stash): the first forward of a checkpointed block keeps the fc1 GEMM output
        # u [tokens, 4h]; the recompute takes it instead of re-running the GEMM (the bias + GeLU
        # and fc1's gradients run as usual).  Keyed like NeoXAttention's stash.  stash_offload:
        # u is parked in pinned host memory between the forward and the recompute (the copy
        # engines move it while the later layers compute; the recompute of the layers above
        # prefetches it back) -- for the FIRST layers, whose u is written earliest in the forward
        # and read latest in the backward.
        self.stash_outputs = False
        self.stash_offload = False
        self._stash = {}
        self._stash_key = None
        self.__dict__["_below"] = []  # MLP modules of the next layers in backward order

    def forward(self, x):
        key, fc1 = self._stash_key, self.dense_h_to_4h
        if self.stash_outputs and key is not None:
            if ds_ckpt.is_recomputing() and torch.is_grad_enabled():
                u = self._stash.pop(key, None)
                from ..runtime.activation_checkpointing.host_stash import StashEntry, host_stash
                for below in self.__dict__["_below"]:  # start bringing the next layers' u back
                    for e in below._stash.values():
                        if isinstance(e, StashEntry):
                            host_stash().prefetch(e)
                if isinstance(u, StashEntry):
                    u = host_stash().fetch(u)[0]
                if u is not None:
                    fc1.stashed_u = u
            elif ds_ckpt.is_checkpoint_forward():
                if key in self._stash or len(self._stash) >= NeoXAttention._STASH_LIMIT:
                    raise RuntimeError("MLP selective-recompute stash for this input was never consumed")
                fc1.keep_u = True
                try:
                    h = fc1(x)
                finally:
                    fc1.keep_u = False
                if self.stash_offload:
                    from ..runtime.activation_checkpointing.host_stash import host_stash
                    self._stash[key] = host_stash().park(id(self), (fc1.kept_u,))
                else:
                    self._stash[key] = fc1.kept_u
                fc1.kept_u = None
                return self.dense_4h_to_h(h)
        return self.dense_4h_to_h(fc1(x))


STASH_PREFETCH_DEPTH = 2  # layers whose host-parked stash a recompute starts bringing back


def link_stash_prefetch(mods):
    """Each attention (or MLP) module learns the modules recomputed right after it in backward
    (the layers below), whose host-parked stashes its own recompute prefetches."""
    for i, a in enumerate(mods):
        a.__dict__["_below"] = [mods[j] for j in range(i - 1, max(-1, i - 1 - STASH_PREFETCH_DEPTH), -1)]


class NeoXTransformerLayer(nn.Module):
    """One GPT-NeoX block. Class name matches DeeperSpeed's `layers_to_hook` pattern."""

    def __init__(self, cfg: GPTNeoXConfig, layer_number: int = 0, device=None, dtype=None):
        super().__init__()
        self.cfg = cfg
        self.layer_number = layer_number
        self.input_layernorm = native.FusedLayerNorm(cfg.hidden_size, cfg.layernorm_eps, device=device, dtype=dtype)
        self.post_attention_layernorm = native.FusedLayerNorm(cfg.hidden_size, cfg.layernorm_eps, device=device,
                                                              dtype=dtype)
        self.attention = NeoXAttention(cfg, device, dtype, layer_number)
        self.mlp = NeoXMLP(cfg, device, dtype)
        if cfg.use_parallel_residual:
            d, f = self.attention.dense, self.mlp.dense_4h_to_h
            d.share_partner, f.share_partner = (f.out_features, f.in_features), (d.out_features, d.in_features)

    def _block(self, x):
        # each LayerNorm hands its input on as a second output, so the gradients of the residual
        # stream are summed inside the LN-backward kernels instead of by separate adds
        h1, x = self.input_layernorm(x, residual_out=True)
        a = self.attention(h1)
        if self.cfg.use_parallel_residual:
            h2, x = self.post_attention_layernorm(x, residual_out=True)
            return residual_sum(x, a, self.mlp(h2))
        x = x + a
        h2, x = self.post_attention_layernorm(x, residual_out=True)
        return residual_sum(x, self.mlp(h2))

    def _block_ckpt(self, x):
        key = (x.untyped_storage().data_ptr(), x.storage_offset(), tuple(x.shape))
        self.attention._stash_key = self.mlp._stash_key = key
        try:
            if ds_ckpt.is_recomputing():
                with skip_unread_outputs():
                    return self._block(x)
            return self._block(x)
        finally:
            self.attention._stash_key = self.mlp._stash_key = None

    def forward(self, x):
        if self.cfg.checkpoint_activations and self.training and torch.is_grad_enabled():
            return ds_ckpt.checkpoint(self._block_ckpt, x)
        return self._block(x)


class GPTNeoX(nn.Module):
    """Causal LM; `forward(input_ids, labels=None)` returns logits or the mean token loss."""

    def __init__(self, cfg: GPTNeoXConfig, device=None, dtype=None):
        super().__init__()
        self.cfg = cfg
        self.embed_in = native.Embedding(cfg.vocab_size, cfg.hidden_size, device=device, dtype=dtype)
        self.layers = nn.ModuleList([NeoXTransformerLayer(cfg, i, device, dtype) for i in range(cfg.num_layers)])
        link_stash_prefetch([l.attention for l in self.layers])
        link_stash_prefetch([l.mlp for l in self.layers])
        self.final_layer_norm = native.FusedLayerNorm(cfg.hidden_size, cfg.layernorm_eps, device=device, dtype=dtype)
        self.embed_out = Linear(cfg.hidden_size, cfg.vocab_size, bias=False, device=device, dtype=dtype)
        self.reset_parameters()

    @torch.no_grad()
    def reset_parameters(self):
        std = self.cfg.init_std
        out_std = std / math.sqrt(2.0 * max(1, self.cfg.num_layers))
        for name, p in self.named_parameters():
            if p.dim() >= 2:
                p.normal_(0.0, out_std if name.endswith("dense.weight") or name.endswith("4h_to_h.weight") else std)
            elif "layernorm" in name or "layer_norm" in name:
                p.fill_(1.0 if name.endswith("weight") else 0.0)
            else:
                p.zero_()

    def forward(self, input_ids, labels=None):
        x = self.embed_in(input_ids)
        for layer in self.layers:
            x = layer(x)
        x = self.final_layer_norm(x)
        logits = self.embed_out(x)
        if labels is None:
            return logits
        return lm_loss(logits, labels, internal=True)


def lm_loss(logits, labels, internal=False):
    """Mean next-token loss (labels already aligned with logits); fused HIP kernel on GPU.
    internal: the logits never leave the model, so the backward writes dlogits over them."""
    return native.cross_entropy(logits, labels, inplace_grad=internal)


# -------------------------------------------------------------------------- pipeline form
class _EmbedPipe(nn.Module):
    def __init__(self, cfg, device=None, dtype=None):
        super().__init__()
        self.embed_in = native.Embedding(cfg.vocab_size, cfg.hidden_size, device=device, dtype=dtype)
        nn.init.normal_(self.embed_in.weight, 0.0, cfg.init_std)

    def forward(self, input_ids):
        return self.embed_in(input_ids)


class _LayerPipe(NeoXTransformerLayer):
    pass


class _FinalPipe(nn.Module):
    def __init__(self, cfg, device=None, dtype=None):
        super().__init__()
        self.final_layer_norm = native.FusedLayerNorm(cfg.hidden_size, cfg.layernorm_eps, device=device, dtype=dtype)
        self.embed_out = Linear(cfg.hidden_size, cfg.vocab_size, bias=False, device=device, dtype=dtype)
        nn.init.normal_(self.embed_out.weight, 0.0, cfg.init_std)

    def forward(self, x):
        return self.embed_out(self.final_layer_norm(x))


def to_pipeline(cfg: GPTNeoXConfig, num_stages: int, topology=None, partition_method="type:NeoXTransformerLayer",
                activation_checkpoint_interval=0, **kw):
    """GPT-NeoX as a PipelineModule (embedding, N blocks, final norm + head)."""
    from ..runtime.pipe.module import LayerSpec, PipelineModule
    # only transformer blocks are recomputed: a checkpointed embedding would see integer token
    # ids as its only input and return an output that does not require grad
    kw.setdefault("checkpointable_layers", ["NeoXTransformerLayer"])
    specs = [LayerSpec(_EmbedPipe, cfg)]
    for i in range(cfg.num_layers):
        specs.append(LayerSpec(NeoXTransformerLayer, cfg, i))
    specs.append(LayerSpec(_FinalPipe, cfg))
    return PipelineModule(layers=specs, num_stages=num_stages if topology is None else None, topology=topology,
                          loss_fn=lm_loss, partition_method=partition_method,
                          activation_checkpoint_interval=activation_checkpoint_interval, **kw)
