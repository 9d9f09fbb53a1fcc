"""BERT pre-training model built on DeepSpeedTransformerLayer (the reference's BERT path).

Reference parity: the BingBertSquad / "fastest BERT training" model the reference benchmarks its
transformer kernel with (docs/_posts/2020-05-28-fastest-bert-training.md; test model
tests/unit/modeling.py `BertForPreTraining` with `DeepSpeedTransformerLayer` encoder layers,
pre-LayerNorm, masked-LM head over the masked positions only, next-sentence head).

Encoder layers are `ops.transformer.DeepSpeedTransformerLayer` (HIP LayerNorm, bias+GeLU,
masked softmax, Philox dropout, bias+dropout+residual kernels, hipBLASLt GEMMs).  The MLM decoder
is tied to the word embedding and evaluated only on the gathered masked positions; its
cross-entropy is the fused HIP kernel.

Progressive layer dropping (PLD, reference: deepspeed/runtime/progressive_layer_drop.py and the
engine's forward kwargs, deepspeed/runtime/engine.py `progressive_layer_drop` / `pld_theta`): the
engine passes `progressive_layer_drop=True, pld_theta=theta(t)`; in training, encoder layer i
(1-based) of L runs with keep probability 1 - i / L * (1 - theta) and is an identity otherwise
(pre-LN layers are residual blocks, so a dropped layer passes its input through).  The draws come
from a host generator seeded by the config, so every data-parallel rank skips the same layers
(their gradient buckets stay aligned) without a collective.
"""

from __future__ import annotations

import math
from dataclasses import dataclass

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops import native
from ..ops.linear import Linear
from ..ops.transformer import DeepSpeedTransformerConfig, DeepSpeedTransformerLayer
from ..ops.transformer.transformer import chain_layer_norms, take_chained_norm


@dataclass
class BertConfig:
    vocab_size: int = 30528  # 30522 padded to a multiple of 64
    hidden_size: int = 1024
    num_layers: int = 24
    num_heads: int = 16
    intermediate_size: int = 4096
    max_position: int = 512
    type_vocab_size: int = 2
    hidden_dropout: float = 0.1
    attn_dropout: float = 0.1
    layer_norm_eps: float = 1e-12
    init_range: float = 0.02
    pre_layer_norm: bool = True
    seed: int = 42

    def flops_per_sample(self, seq: int, masked: int) -> float:
        """Training FLOPs (3x forward) of one sequence: encoder GEMMs 24*S*H^2 per layer,
        attention 4*S^2*H per layer, MLM transform + decoder over the masked positions."""
        H, L = self.hidden_size, self.num_layers
        enc = L * (24 * seq * H * H + 4 * seq * seq * H)
        head = 2 * masked * H * (H + self.vocab_size)
        return 3.0 * (enc + head)


PRESETS = {
    "bert-large": dict(hidden_size=1024, num_layers=24, num_heads=16, intermediate_size=4096),
    "bert-base": dict(hidden_size=768, num_layers=12, num_heads=12, intermediate_size=3072),
    "tiny": dict(vocab_size=512, hidden_size=128, num_layers=2, num_heads=4, intermediate_size=512, max_position=128),
}


def get_config(name: str, **overrides) -> BertConfig:
    d = dict(PRESETS[name])
    d.update(overrides)
    return BertConfig(**d)


class BertForPreTraining(nn.Module):
    """forward(input_ids, token_type_ids, attention_mask, masked_positions, masked_labels,
    next_sentence_labels) -> scalar loss (MLM + NSP)."""

    def __init__(self, cfg: BertConfig, device=None, dtype=None):
        super().__init__()
        self.cfg = cfg
        H = cfg.hidden_size
        self.word_embeddings = native.Embedding(cfg.vocab_size, H)
        self.position_embeddings = native.Embedding(cfg.max_position, H)
        self.token_type_embeddings = native.Embedding(cfg.type_vocab_size, H)
        self.embeddings_ln = native.FusedLayerNorm(H, cfg.layer_norm_eps)
        lcfg = DeepSpeedTransformerConfig(batch_size=-1, hidden_size=H, intermediate_size=cfg.intermediate_size,
                                          heads=cfg.num_heads, attn_dropout_ratio=cfg.attn_dropout,
                                          hidden_dropout_ratio=cfg.hidden_dropout, num_hidden_layers=cfg.num_layers,
                                          initializer_range=cfg.init_range, layer_norm_eps=cfg.layer_norm_eps,
                                          seed=cfg.seed, pre_layer_norm=cfg.pre_layer_norm,
                                          bf16=dtype == torch.bfloat16, fp16=dtype == torch.float16)
        self.layers = nn.ModuleList()
        for _ in range(cfg.num_layers):
            import copy
            self.layers.append(DeepSpeedTransformerLayer(copy.copy(lcfg)))
        self.final_ln = native.FusedLayerNorm(H, cfg.layer_norm_eps) if cfg.pre_layer_norm else None
        self.mlm_dense = Linear(H, H)
        self.mlm_ln = native.FusedLayerNorm(H, cfg.layer_norm_eps)
        self.mlm_bias = nn.Parameter(torch.zeros(cfg.vocab_size))
        self.pooler = Linear(H, H)
        self.nsp = Linear(H, 2)
        for m in (self.word_embeddings, self.position_embeddings, self.token_type_embeddings):
            nn.init.normal_(m.weight, 0.0, cfg.init_range)
        for m in (self.mlm_dense, self.pooler, self.nsp):
            nn.init.normal_(m.weight, 0.0, cfg.init_range)
            nn.init.zeros_(m.bias)
        self.to(device=device, dtype=dtype)
        self._pld_gen = torch.Generator().manual_seed(cfg.seed)
        # each encoder layer's output pass applies the next LayerNorm (ops/transformer chain_layer_norms)
        self.chain_norms = True
        self.pld_kept = []  # layers run by the last PLD forward (tests / diagnostics)

    def _pld_keep(self, theta: float):
        """Bernoulli keep mask over the encoder layers for one PLD forward."""
        L = len(self.layers)
        u = torch.rand(L, generator=self._pld_gen).tolist()
        return [u[i] < 1.0 - (i + 1) / L * (1.0 - theta) for i in range(L)]

    def enable_device_rng(self, seed: int = 1234):
        """Every dropout of the model draws from device [seed, step] counters that kernels inside
        the forward advance (the embeddings' here, each encoder layer its own), so a HIP graph
        captured around a whole training step gets fresh masks on every replay
        (`scripts/bench_bert.py --hip-graphs step`).  The masks differ from host-seeded ones."""
        self._emb_rng = torch.tensor([int(seed), 0], dtype=torch.int64, device=self.word_embeddings.weight.device)
        for i, layer in enumerate(self.layers):
            layer.enable_device_rng(seed + 7919 * (i + 1))

    def encode(self, input_ids, token_type_ids=None, attention_mask=None, progressive_layer_drop=False,
               pld_theta=1.0):
        B, S = input_ids.shape
        pos = torch.arange(S, device=input_ids.device)
        x = self.word_embeddings(input_ids) + self.position_embeddings(pos)[None]
        if token_type_ids is not None:
            x = x + self.token_type_embeddings(token_type_ids)
        x = self.embeddings_ln(x)
        rng = getattr(self, "_emb_rng", None)
        if rng is not None and self.training and torch.is_grad_enabled():
            rng[1:].add_(1)
        x = native.dropout(x, self.cfg.hidden_dropout, self.training, rng=rng)
        ext = None
        if attention_mask is not None:
            ext = ((1.0 - attention_mask.to(x.dtype)) * -10000.0)[:, None, None, :]
        keep = self._pld_keep(pld_theta) if progressive_layer_drop and self.training else None
        if keep is not None:
            self.pld_kept = [i for i, k in enumerate(keep) if k]
        run = [layer for i, layer in enumerate(self.layers) if keep is None or keep[i]]
        # each layer's output pass also applies the LayerNorm that reads it next
        chain_layer_norms(run, self.final_ln, enabled=self.chain_norms)
        for layer in run:
            x = layer(x, ext)
        if self.final_ln is not None:
            y = take_chained_norm(x, self.final_ln)
            x = self.final_ln(x) if y is None else y
        return x

    def forward(self, input_ids, token_type_ids=None, attention_mask=None, masked_positions=None, masked_labels=None,
                next_sentence_labels=None, progressive_layer_drop=False, pld_theta=1.0):
        x = self.encode(input_ids, token_type_ids, attention_mask, progressive_layer_drop, pld_theta)
        B, S, H = x.shape
        if masked_positions is None:
            masked_positions = torch.arange(S, device=x.device)[None].expand(B, S)
        flat = (masked_positions + S * torch.arange(B, device=x.device)[:, None]).reshape(-1)
        h = x.reshape(B * S, H).index_select(0, flat)
        h = self.mlm_ln(native.bias_gelu(F.linear(h, self.mlm_dense.weight), self.mlm_dense.bias, approximate=True))
        logits = F.linear(h, self.word_embeddings.weight, self.mlm_bias)
        if masked_labels is None:
            return logits
        loss = native.cross_entropy(logits, masked_labels.reshape(-1))
        if next_sentence_labels is not None:
            pooled = torch.tanh(self.pooler(x[:, 0]))
            loss = loss + F.cross_entropy(self.nsp(pooled).float(), next_sentence_labels)
        return loss
