"""GPT-2 (the reference's Megatron-GPT2 test model family, tests/model/Megatron_GPT2) on the
framework's MI355X kernels: learned absolute position embeddings, pre-LayerNorm blocks,
tanh-GeLU MLP with the bias fused into the HIP GeLU kernel, fused causal flash attention, and an
LM head tied to the token embedding.

ZeRO-3: the tied head uses the embedding weight outside the embedding module, so it declares
it with `register_external_parameter` (reference partition_parameters.py usage pattern)."""

from __future__ import annotations

import math
from dataclasses import dataclass

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops import native
from ..ops.linear import Linear
from ..ops.attention import attention
from ..runtime.activation_checkpointing import checkpointing as ds_ckpt
from ..runtime.zero.partition_parameters import register_external_parameter
from .gpt_neox import LinearBiasGeLU, OutputLinear, lm_loss, skip_unread_outputs


@dataclass
class GPT2Config:
    vocab_size: int = 50304  # 50257 padded to a multiple of 64
    n_positions: int = 1024
    hidden_size: int = 768
    num_layers: int = 12
    num_heads: int = 12
    layernorm_eps: float = 1e-5
    init_std: float = 0.02
    checkpoint_activations: bool = False

    @property
    def head_dim(self):
        return self.hidden_size // self.num_heads

    def num_params(self):
        h, L, V = self.hidden_size, self.num_layers, self.vocab_size
        return V * h + self.n_positions * h + L * (12 * h * h + 13 * h) + 2 * h

    def flops_per_token(self, seq_len, recompute=False):
        mult = 8 if recompute else 6
        return mult * (self.num_params() - self.n_positions * self.hidden_size) + \
            (mult // 2) * 2 * self.num_layers * seq_len * self.hidden_size


GPT2_PRESETS = {
    "gpt2-125m": dict(hidden_size=768, num_layers=12, num_heads=12),
    "gpt2-350m": dict(hidden_size=1024, num_layers=24, num_heads=16),
    "gpt2-774m": dict(hidden_size=1280, num_layers=36, num_heads=20),
    "gpt2-1.5b": dict(hidden_size=1600, num_layers=48, num_heads=25),
    "gpt2-tiny": dict(hidden_size=128, num_layers=2, num_heads=4, vocab_size=512, n_positions=128),
}


def get_gpt2_config(name="gpt2-125m", **overrides) -> GPT2Config:
    d = dict(GPT2_PRESETS[name])
    d.update(overrides)
    return GPT2Config(**d)


class GPT2Attention(nn.Module):
    def __init__(self, cfg: GPT2Config, device=None, dtype=None):
        super().__init__()
        self.cfg = cfg
        self.c_attn = Linear(cfg.hidden_size, 3 * cfg.hidden_size, device=device, dtype=dtype)
        self.c_proj = Linear(cfg.hidden_size, cfg.hidden_size, device=device, dtype=dtype)

    def forward(self, x):
        B, S, H = x.shape
        nh, hd = self.cfg.num_heads, self.cfg.head_dim
        q, k, v = self.c_attn(x).view(B, S, 3, nh, hd).permute(2, 0, 3, 1, 4).unbind(0)
        ctx = attention(q.contiguous(), k.contiguous(), v.contiguous(), causal=True, softmax_scale=1.0 / math.sqrt(hd),
                        out_layout="bshd")
        return self.c_proj(ctx.reshape(B, S, H))


class GPT2Block(nn.Module):
    def __init__(self, cfg: GPT2Config, device=None, dtype=None):
        super().__init__()
        self.cfg = cfg
        self.ln_1 = native.FusedLayerNorm(cfg.hidden_size, cfg.layernorm_eps, device=device, dtype=dtype)
        self.attn = GPT2Attention(cfg, device, dtype)
        self.ln_2 = native.FusedLayerNorm(cfg.hidden_size, cfg.layernorm_eps, device=device, dtype=dtype)
        self.c_fc = LinearBiasGeLU(cfg.hidden_size, 4 * cfg.hidden_size, approximate=True, device=device, dtype=dtype)
        # feeds only the block's final residual sum: skipped during recompute
        self.c_proj = OutputLinear(4 * cfg.hidden_size, cfg.hidden_size, device=device, dtype=dtype)

    def _block_ckpt(self, x):
        if ds_ckpt.is_recomputing():
            with skip_unread_outputs():
                return self._block(x)
        return self._block(x)

    def _block(self, x):
        x = x + self.attn(self.ln_1(x))
        return x + self.c_proj(self.c_fc(self.ln_2(x)))

    def forward(self, x):
        if self.cfg.checkpoint_activations and self.training and torch.is_grad_enabled():
            return ds_ckpt.checkpoint(self._block_ckpt, x)
        return self._block(x)


class GPT2LMHead(nn.Module):
    """Final LayerNorm + projection onto the (tied) token embedding."""

    def __init__(self, cfg: GPT2Config, wte: nn.Embedding, device=None, dtype=None):
        super().__init__()
        self.ln_f = native.FusedLayerNorm(cfg.hidden_size, cfg.layernorm_eps, device=device, dtype=dtype)
        self._wte = [wte]  # not a submodule: the parameter is owned by the embedding
        register_external_parameter(self, wte.weight)

    def forward(self, x):
        return F.linear(self.ln_f(x), self._wte[0].weight)


class GPT2(nn.Module):
    def __init__(self, cfg: GPT2Config, device=None, dtype=None):
        super().__init__()
        self.cfg = cfg
        self.wte = native.Embedding(cfg.vocab_size, cfg.hidden_size, device=device, dtype=dtype)
        self.wpe = native.Embedding(cfg.n_positions, cfg.hidden_size, device=device, dtype=dtype)
        self.h = nn.ModuleList([GPT2Block(cfg, device, dtype) for _ in range(cfg.num_layers)])
        self.head = GPT2LMHead(cfg, self.wte, device, dtype)
        self.reset_parameters()

    @torch.no_grad()
    def reset_parameters(self):
        std = self.cfg.init_std
        proj_std = std / math.sqrt(2.0 * self.cfg.num_layers)
        for name, p in self.named_parameters():
            if p.dim() >= 2:
                p.normal_(0.0, proj_std if name.endswith("c_proj.weight") else std)
            elif "ln" in name and name.endswith("weight"):
                p.fill_(1.0)
            else:
                p.zero_()

    def forward(self, input_ids, labels=None):
        S = input_ids.shape[1]
        pos = torch.arange(S, device=input_ids.device)
        x = self.wte(input_ids) + self.wpe(pos)[None]
        for blk in self.h:
            x = blk(x)
        logits = self.head(x)
        if labels is None:
            return logits
        return lm_loss(logits, labels)
