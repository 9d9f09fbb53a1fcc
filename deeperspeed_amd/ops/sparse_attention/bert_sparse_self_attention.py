"""BERT self-attention with block-sparse attention (reference parity:
deepspeed/ops/sparse_attention/bert_sparse_self_attention.py:10-78)."""

import torch.nn as nn

from .sparse_self_attention import SparseSelfAttention
from .sparsity_config import FixedSparsityConfig


class BertSparseSelfAttention(nn.Module):
    def __init__(self, config, sparsity_config=FixedSparsityConfig(num_heads=4)):
        super().__init__()
        if config.hidden_size % config.num_attention_heads != 0:
            raise ValueError(f"The hidden size ({config.hidden_size}) is not a multiple of the number of attention "
                             f"heads ({config.num_attention_heads})")
        self.num_attention_heads = config.num_attention_heads
        self.attention_head_size = int(config.hidden_size / config.num_attention_heads)
        self.all_head_size = self.num_attention_heads * self.attention_head_size
        self.query = nn.Linear(config.hidden_size, self.all_head_size)
        self.key = nn.Linear(config.hidden_size, self.all_head_size)
        self.value = nn.Linear(config.hidden_size, self.all_head_size)
        # layouts sized for the model's positions (the reference keeps SparseSelfAttention's
        # 2048 default here, which caps BERT at 2048 tokens)
        self.sparse_self_attention = SparseSelfAttention(
            sparsity_config, max_seq_length=max(2048, int(getattr(config, "max_position_embeddings", 2048) or 2048)))

    def transpose_for_scores(self, x):
        x = x.view(*x.size()[:-1], self.num_attention_heads, self.attention_head_size)
        return x.permute(0, 2, 1, 3)

    def forward(self, hidden_states, attention_mask=None, *args, **kwargs):
        """attention_mask: additive key-padding mask ([B, S] or HF's extended [B, 1, 1, S]).

        Called the way current HuggingFace BertAttention calls its self-attention (keyword
        arguments such as encoder_hidden_states / past_key_values, an (output, weights) pair
        expected back) it returns (context, None); called as the reference's
        layer(hidden_states, attention_mask) it returns the context tensor."""
        if kwargs.get("encoder_hidden_states") is not None:
            raise NotImplementedError("block-sparse attention is self-attention only")
        q = self.transpose_for_scores(self.query(hidden_states))
        k = self.transpose_for_scores(self.key(hidden_states))
        v = self.transpose_for_scores(self.value(hidden_states))
        if attention_mask is not None and attention_mask.dim() == 4 and attention_mask.size(-2) > 1:
            # current HF passes the padding mask expanded over the query rows ([B, 1, S, S]); for
            # an encoder every row is the same key-padding row
            attention_mask = attention_mask[:, :, :1, :]
        if attention_mask is not None and attention_mask.is_floating_point():
            # HF fills masked keys with the dtype's minimum; the reference convention is -10000
            # (finite after the log2(e) scaling inside the kernels)
            attention_mask = attention_mask.clamp(min=-10000.0)
        ctx = self.sparse_self_attention(q, k, v, key_padding_mask=attention_mask)
        ctx = ctx.permute(0, 2, 1, 3).contiguous()
        ctx = ctx.view(*ctx.size()[:-2], self.all_head_size)
        return (ctx, None) if (args or kwargs) else ctx
