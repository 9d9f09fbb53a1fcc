"""Swap BERT-style layers for DeepSpeedTransformerLayer and back.

Reference parity: deepspeed/module_inject/{inject.py:1-122, replace_module.py:1-193}
(`module_inject`, `replace_transformer_layer`, `revert_transformer_layer`, `replace_module`).
HuggingFace post-LN BertLayer attribute paths by default; `preln=True` uses the NVIDIA
pre-LN names (PreAttentionLayerNorm / PostAttentionLayerNorm / intermediate.dense_act).
Weights are copied (not aliased) so the original model is untouched.
"""

import copy

import torch

from ..ops.transformer import DeepSpeedTransformerConfig, DeepSpeedTransformerLayer


def _attn_ln(child, preln):
    return child.PostAttentionLayerNorm if preln else child.attention.output.LayerNorm


def _inter(child, preln):
    return child.intermediate.dense_act if preln else child.intermediate.dense


def _out_ln(child, preln):
    return child.PreAttentionLayerNorm if preln else child.output.LayerNorm


def _ds_config(bert_config, micro_batch_size, seed, preln, fp16, training, huggingface, local_rank=-1):
    return DeepSpeedTransformerConfig(batch_size=micro_batch_size, hidden_size=bert_config.hidden_size,
                                      intermediate_size=getattr(bert_config, "intermediate_size", -1),
                                      heads=bert_config.num_attention_heads,
                                      attn_dropout_ratio=bert_config.attention_probs_dropout_prob,
                                      hidden_dropout_ratio=bert_config.hidden_dropout_prob,
                                      num_hidden_layers=bert_config.num_hidden_layers,
                                      initializer_range=bert_config.initializer_range,
                                      layer_norm_eps=getattr(bert_config, "layer_norm_eps", 1e-12), seed=seed,
                                      fp16=fp16, pre_layer_norm=preln, huggingface=huggingface, training=training,
                                      local_rank=local_rank)


@torch.no_grad()
def _to_ds_layer(child, cfg, preln):
    new = DeepSpeedTransformerLayer(cfg)
    att = child.attention.self
    dt = new.attn_qkvw.dtype
    cp = lambda dst, src: dst.data.copy_(src.data.to(dst.device, dt))  # noqa: E731
    cp(new.attn_qkvw, torch.cat([att.query.weight, att.key.weight, att.value.weight], 0))
    cp(new.attn_qkvb, torch.cat([att.query.bias, att.key.bias, att.value.bias], 0))
    cp(new.attn_ow, child.attention.output.dense.weight)
    cp(new.attn_ob, child.attention.output.dense.bias)
    cp(new.attn_nw, _attn_ln(child, preln).weight)
    cp(new.attn_nb, _attn_ln(child, preln).bias)
    cp(new.inter_w, _inter(child, preln).weight)
    cp(new.inter_b, _inter(child, preln).bias)
    cp(new.output_w, child.output.dense.weight)
    cp(new.output_b, child.output.dense.bias)
    cp(new.norm_w, _out_ln(child, preln).weight)
    cp(new.norm_b, _out_ln(child, preln).bias)
    return new.to(child.output.dense.weight.device)


@torch.no_grad()
def _from_ds_layer(ds, orig_layer_impl, bert_config, preln):
    orig = orig_layer_impl(bert_config)
    H = ds.config.hidden_size
    att = orig.attention.self
    cp = lambda dst, src: dst.data.copy_(src.data.to(dst.dtype))  # noqa: E731
    q, k, v = ds.attn_qkvw.split(H, 0)
    qb, kb, vb = ds.attn_qkvb.split(H, 0)
    cp(att.query.weight, q), cp(att.key.weight, k), cp(att.value.weight, v)
    cp(att.query.bias, qb), cp(att.key.bias, kb), cp(att.value.bias, vb)
    cp(orig.attention.output.dense.weight, ds.attn_ow)
    cp(orig.attention.output.dense.bias, ds.attn_ob)
    cp(_attn_ln(orig, preln).weight, ds.attn_nw)
    cp(_attn_ln(orig, preln).bias, ds.attn_nb)
    cp(_inter(orig, preln).weight, ds.inter_w)
    cp(_inter(orig, preln).bias, ds.inter_b)
    cp(orig.output.dense.weight, ds.output_w)
    cp(orig.output.dense.bias, ds.output_b)
    cp(_out_ln(orig, preln).weight, ds.norm_w)
    cp(_out_ln(orig, preln).bias, ds.norm_b)
    return orig.to(ds.attn_qkvw.device)


def replace_module(model, orig_class, replace_fn):
    """Replace every `orig_class` submodule with `replace_fn(child)` (recursive)."""
    for name, child in model.named_children():
        if isinstance(child, orig_class):
            setattr(model, name, replace_fn(child))
        else:
            replace_module(child, orig_class, replace_fn)
    return model


def replace_transformer_layer(orig_layer_impl, model, micro_batch_size, bert_config, seed, preln=False, fp16=True,
                              training=True, huggingface=False, local_rank=-1):
    cfg = _ds_config(bert_config, micro_batch_size, seed, preln, fp16, training, huggingface, local_rank)
    return replace_module(model, orig_layer_impl, lambda child: _to_ds_layer(child, copy.deepcopy(cfg), preln))


def revert_transformer_layer(orig_layer_impl, model, bert_config, preln=False):
    return replace_module(model, DeepSpeedTransformerLayer,
                          lambda child: _from_ds_layer(child, orig_layer_impl, bert_config, preln))


def module_inject(layer_obj, model, config, micro_batch_size, max_seq_length, seed, preln, fp16=True):
    """Reference inject.py entry point (max_seq_length is informational here)."""
    return replace_transformer_layer(layer_obj, model, micro_batch_size, config, seed, preln=preln, fp16=fp16)
