"""DeepSpeed BERT transformer layer for MI355X.

Reference parity: deepspeed/ops/transformer/transformer.py:39-614 (`DeepSpeedTransformerConfig`,
`DeepSpeedTransformerFunction`, `DeepSpeedTransformerLayer`) and the layer dataflow of
csrc/transformer/ds_transformer_cuda.cpp:147-292 (same parameter names and shapes, pre-LN and
post-LN, tanh GeLU, additive attention mask [B,1,1,S], attention-prob and hidden dropout).

Built from the framework's HIP kernels + hipBLASLt GEMMs instead of one monolithic C++
layer: fused LayerNorm, bias+tanh-GeLU, row softmax with a broadcast additive mask, Philox
dropout, and bias+dropout+residual fusion, composed under autograd (so ZeRO-3 hooks,
activation checkpointing and mixed precision work unchanged).  Memory flags (reference
ds_transformer_cuda.cpp:185-193): `gelu_checkpoint` is inherent (the GeLU kernel keeps only its
input); `attn_dropout_checkpoint` keeps the softmax output + the 1-byte dropout mask and
re-applies the mask in backward instead of holding the dropped probabilities
(native.dropout_matmul); `normalize_invertible` keeps LayerNorm outputs only and recovers the
normalised input from them in backward (native.layer_norm_invertible).  `stochastic_mode` is
accepted for config compatibility: the kernels here are deterministic and already take the
reference's fast path.
"""

import json
import math

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import native
from ..attention import masked_softmax
from ..linear import linear as _linear


class TransformerConfig:
    def __init__(self, batch_size, hidden_size, intermediate_size, heads, attn_dropout_ratio, hidden_dropout_ratio,
                 num_hidden_layers, initializer_range):
        self.layer_id = -1
        self.batch_size = batch_size
        self.hidden_size = hidden_size
        self.intermediate_size = intermediate_size
        self.heads = heads
        self.attn_dropout_ratio = attn_dropout_ratio
        self.hidden_dropout_ratio = hidden_dropout_ratio
        self.num_hidden_layers = num_hidden_layers
        self.initializer_range = initializer_range


class DeepSpeedTransformerConfig(TransformerConfig):
    def __init__(self, batch_size=-1, hidden_size=-1, intermediate_size=-1, heads=-1, attn_dropout_ratio=-1,
                 hidden_dropout_ratio=-1, num_hidden_layers=-1, initializer_range=-1, layer_norm_eps=1e-12,
                 local_rank=-1, seed=-1, fp16=False, pre_layer_norm=True, normalize_invertible=False,
                 gelu_checkpoint=False, adjust_init_range=True, attn_dropout_checkpoint=False, stochastic_mode=False,
                 huggingface=False, training=True, bf16=False):
        super().__init__(batch_size, hidden_size, intermediate_size if intermediate_size > 0 else 4 * hidden_size,
                         heads, attn_dropout_ratio, hidden_dropout_ratio, num_hidden_layers, initializer_range)
        self.fp16 = fp16
        self.bf16 = bf16
        self.pre_layer_norm = pre_layer_norm
        self.local_rank = local_rank
        self.seed = seed
        self.normalize_invertible = normalize_invertible
        self.gelu_checkpoint = gelu_checkpoint
        self.adjust_init_range = adjust_init_range
        self.test_gemm = False
        self.layer_norm_eps = layer_norm_eps
        self.training = training
        self.is_grad_enabled = True
        self.attn_dropout_checkpoint = attn_dropout_checkpoint
        self.stochastic_mode = stochastic_mode
        self.huggingface = huggingface

    @classmethod
    def from_dict(cls, json_object):
        config = DeepSpeedTransformerConfig()
        for k, v in json_object.items():
            config.__dict__[k] = v
        return config

    @classmethod
    def from_json_file(cls, json_file):
        with open(json_file, "r", encoding="utf-16") as reader:
            return cls.from_dict(json.loads(reader.read()))


class _SplitHeads(torch.autograd.Function):
    """qkv [B,S,3H] -> contiguous q,k,v [B,nh,S,hd] in one HIP pass (reference
    bias_add_transform_0213); backward merges dq,dk,dv back into dqkv in one pass."""

    @staticmethod
    def forward(ctx, qkv, nh):
        q, k, v = native.hip_ops().heads_split(qkv.contiguous(), nh)
        return q, k, v

    @staticmethod
    def backward(ctx, dq, dk, dv):
        return native.hip_ops().heads_merge(dq.contiguous(), dk.contiguous(), dv.contiguous()), None


class _MergeHeads(torch.autograd.Function):
    """ctx [B,nh,S,hd] -> [B,S,nh*hd] (reference transform4d_0213) and back."""

    @staticmethod
    def forward(ctx, x):
        B, nh, S, hd = x.shape
        ctx.nh, ctx.hd = nh, hd
        return native.hip_ops().swap12(x.contiguous()).view(B, S, nh * hd)

    @staticmethod
    def backward(ctx, g):
        B, S, _ = g.shape
        return native.hip_ops().swap12(g.contiguous().view(B, S, ctx.nh, ctx.hd))


# flash attention for the encoder (False: the materialised scores -> softmax -> dropout -> P V path)
_ENCODER_FLASH = True


def _use_head_kernels(x, hd):
    return x.is_cuda and x.dtype in (torch.bfloat16, torch.float16) and hd % 8 == 0


class DeepSpeedTransformerFunction:
    """Functional form of the layer (reference exposes an autograd.Function with this name)."""

    @staticmethod
    def apply(input, input_mask, layer, grads, layer_id, attn_qkvw, attn_qkvb, attn_ow, attn_ob, attn_nw, attn_nb,
              inter_w, inter_b, output_w, output_b, norm_w, norm_b, config):
        cfg = config
        training = cfg.training
        B, S, Hd = input.shape
        nh = cfg.heads
        hd = Hd // nh
        gen = layer._generator if layer is not None else None
        eps = cfg.layer_norm_eps
        x = input
        invertible = getattr(cfg, "normalize_invertible", False)
        ln = native.layer_norm_invertible if invertible else native.layer_norm
        # pre-LN: the block input feeds both the LayerNorm and the residual add; the fused form
        # returns it as a second output so the LN backward adds the residual gradient in-kernel
        fuse_res = cfg.pre_layer_norm and not invertible
        # layer slots of the stacked activation / gradient buffers of ops/wgrad_batch (the weight
        # gradients of all layers then run as batched GEMMs); set by chain_layer_norms
        si, sn = (getattr(layer, "_dsa_slab_index", None), getattr(layer, "_dsa_slab_count", 0)) \
            if (layer is not None and torch.is_grad_enabled()) else (None, 0)

        def slab(kind, idx=None):
            return None if si is None else (kind, si if idx is None else idx, sn)

        pre = getattr(x, "_dsa_next_ln", None)
        if fuse_res and pre is not None and pre[0] is layer:
            inp = pre[1]  # the previous layer's output pass already normalised x with this layer's LN
        elif fuse_res:
            inp, x = native.layer_norm_residual(x, norm_w, norm_b, eps, y_slab=slab("qkv_x"))
        else:
            inp = ln(x, norm_w, norm_b, eps) if cfg.pre_layer_norm else x
        qkv = _linear(inp, attn_qkvw, attn_qkvb)
        fast = _use_head_kernels(qkv, hd)
        mask = None
        if input_mask is not None:
            mask = input_mask
            if mask.dim() == 2:
                mask = mask[:, None, None, :]
            mask = mask.reshape(B, 1, -1, S)
        rng = getattr(layer, "_rng", None) if (layer is not None and training) else None
        if (fast and _ENCODER_FLASH and native.qkv_flash_supported(qkv, nh)
                and (mask is None or mask.shape[2] == 1)):
            # one fused kernel per direction reading q, k, v straight out of the QKV projection:
            # scores, key-padding bias, softmax, dropout and P V stay on chip, the context is
            # written token-major [B, S, nh * hd] for the output projection, dqkv in qkv's layout
            ctx = native.flash_attention_qkv(qkv, nh, None if mask is None else mask.reshape(B, S),
                                             1.0 / math.sqrt(hd), cfg.attn_dropout_ratio, training, gen, rng=rng, site=1,
                                             slabs=(slab("ao_x"), slab("qkv_dy")))
        else:
            if fast:
                q, k, v = _SplitHeads.apply(qkv, nh)  # contiguous [B, nh, S, hd]: batched GEMMs without copies
            else:
                q, k, v = qkv.view(B, S, 3, nh, hd).permute(2, 0, 3, 1, 4).unbind(0)  # [B, nh, S, hd]
            scores = torch.matmul(q, k.transpose(-1, -2))
            if mask is not None:
                mask = mask.to(scores.dtype).contiguous()
            probs = masked_softmax(scores, mask, 1.0 / math.sqrt(hd), False, nh)
            if getattr(cfg, "attn_dropout_checkpoint", False):
                ctx = native.dropout_matmul(probs, v, cfg.attn_dropout_ratio, training, gen)
            else:
                probs = native.dropout(probs, cfg.attn_dropout_ratio, training, gen)
                ctx = torch.matmul(probs, v)
            ctx = _MergeHeads.apply(ctx) if fast else ctx.transpose(1, 2).reshape(B, S, Hd)
        attn_out = _linear(ctx, attn_ow)
        if fuse_res:
            # residual sum + the MLP's LayerNorm in one pass (native.bias_dropout_residual_ln)
            ff1_inp, add_res = native.bias_dropout_residual_ln(attn_out, attn_ob, x, attn_nw, attn_nb, eps,
                                                               cfg.hidden_dropout_ratio, training, gen, rng=rng, site=2,
                                                               slabs=(slab("fc1_x"), slab("ao_dy")))
        else:
            add_res = native.bias_dropout_residual(attn_out, attn_ob, x, cfg.hidden_dropout_ratio, training, gen,
                                                   rng=rng, site=2)
            ff1_inp = ln(add_res, attn_nw, attn_nb, eps)
        inter = native.bias_gelu(_linear(ff1_inp, inter_w), inter_b, approximate=True,
                                 slabs=(slab("fc2_x"), slab("fc1_dy")))
        out = _linear(inter, output_w)
        nxt = getattr(layer, "_dsa_next_norm", None) if layer is not None else None
        if cfg.pre_layer_norm and fuse_res and nxt is not None:
            # the block output is the next layer's (or the final) LayerNorm input: normalise it in
            # the same pass and hand the result over on the output tensor (consumed by that owner)
            owner, nw, nb, neps = nxt
            nidx = getattr(owner, "_dsa_slab_index", None) if isinstance(owner, DeepSpeedTransformerLayer) else None
            y_next, out = native.bias_dropout_residual_ln(out, output_b, add_res, nw, nb, neps,
                                                          cfg.hidden_dropout_ratio, training, gen, rng=rng, site=3,
                                                          slabs=(None if nidx is None else slab("qkv_x", nidx),
                                                                 slab("fc2_dy")))
            out._dsa_next_ln = (owner, y_next)
        elif cfg.pre_layer_norm:
            out = native.bias_dropout_residual(out, output_b, add_res, cfg.hidden_dropout_ratio, training, gen, rng=rng,
                                               site=3)
        else:
            out = native.bias_dropout_residual(out, output_b, ff1_inp, cfg.hidden_dropout_ratio, training, gen, rng=rng,
                                               site=3)
            out = ln(out, norm_w, norm_b, eps)
        if grads is not None:  # reference test hook: collect gradients of the intermediates
            for t in (out, add_res, ff1_inp):
                if t.requires_grad:
                    t.register_hook(lambda g, _l=grads: _l.append(g))
        return out


class DeepSpeedTransformerLayer(nn.Module):
    layer_id = 0
    _stochastic_warned = False

    def __init__(self, config, initial_weights=None, initial_biases=None):
        super().__init__()
        self.config = config
        self.config.layer_id = DeepSpeedTransformerLayer.layer_id
        DeepSpeedTransformerLayer.layer_id += 1
        if getattr(config, "stochastic_mode", False) and not DeepSpeedTransformerLayer._stochastic_warned:
            # reference: a separate -D__STOCHASTIC_MODE__ build that drops block barriers in the
            # LayerNorm reductions and does dropout in half2 math (csrc/transformer/
            # normalize_kernels.cu:64-191, dropout_kernels.cu:68-187).  Nothing here has a racy
            # fast variant to switch to: the LayerNorms reduce within one wave (no barrier) and
            # dropout is already 16-byte vectorised, so the deterministic kernels run.
            import warnings
            warnings.warn("DeepSpeedTransformerConfig.stochastic_mode=True: no separate stochastic kernels on "
                          "MI355X; the deterministic kernels (already barrier-free per row) are used", stacklevel=2)
            DeepSpeedTransformerLayer._stochastic_warned = True
        if self.config.local_rank >= 0 and torch.cuda.is_available():
            torch.cuda.set_device(self.config.local_rank)
        H, I = config.hidden_size, config.intermediate_size
        self._generator = None
        if config.seed >= 0:
            self._generator = torch.Generator().manual_seed(config.seed + config.layer_id)
        if initial_weights is None and initial_biases is None:
            self.attn_qkvw = nn.Parameter(torch.empty(3 * H, H))
            self.attn_qkvb = nn.Parameter(torch.empty(3 * H))
            self.attn_ow = nn.Parameter(torch.empty(H, H))
            self.attn_ob = nn.Parameter(torch.empty(H))
            self.attn_nw = nn.Parameter(torch.empty(H))
            self.attn_nb = nn.Parameter(torch.empty(H))
            self.inter_w = nn.Parameter(torch.empty(I, H))
            self.inter_b = nn.Parameter(torch.empty(I))
            self.output_w = nn.Parameter(torch.empty(H, I))
            self.output_b = nn.Parameter(torch.empty(H))
            self.norm_w = nn.Parameter(torch.empty(H))
            self.norm_b = nn.Parameter(torch.empty(H))
            self.init_transformer_weights(config.adjust_init_range)
        else:  # unit-test path: weights supplied as [q, k, v, o, attn_norm, inter, output, norm]
            self.attn_qkvw = nn.Parameter(torch.cat([w.detach() for w in initial_weights[:3]], 0).clone())
            self.attn_qkvb = nn.Parameter(torch.zeros(3 * H))
            self.attn_ow, self.attn_ob = initial_weights[3], initial_biases[3]
            self.attn_nw, self.attn_nb = initial_weights[4], initial_biases[4]
            self.inter_w, self.inter_b = initial_weights[5], initial_biases[5]
            self.output_w, self.output_b = initial_weights[6], initial_biases[6]
            self.norm_w, self.norm_b = initial_weights[7], initial_biases[7]
        dtype = torch.float16 if config.fp16 else (torch.bfloat16 if getattr(config, "bf16", False) else None)
        if dtype is not None:
            self.to(dtype)

    @torch.no_grad()
    def init_transformer_weights(self, adjust_init_range=False):
        std = self.config.initializer_range
        out_std = std / math.sqrt(2.0 * self.config.num_hidden_layers) if adjust_init_range else std
        self.attn_qkvw.normal_(0.0, std)
        self.attn_qkvb.zero_()
        self.attn_ow.normal_(0.0, out_std)
        self.attn_ob.zero_()
        self.attn_nw.fill_(1.0)
        self.attn_nb.zero_()
        self.inter_w.normal_(0.0, std)
        self.inter_b.zero_()
        self.output_w.normal_(0.0, out_std)
        self.output_b.zero_()
        self.norm_w.fill_(1.0)
        self.norm_b.zero_()

    def enable_device_rng(self, seed: int, device=None):
        """Dropout seeds from a device int64 [seed, step] that the layer's forward advances with
        a kernel: a HIP graph captured around the layer then draws fresh masks on every replay
        (host-drawn seeds would be frozen into the graph).  Needed for graphed training
        (`make_graphed_encoder`); the eager masks differ from the host-seeded ones."""
        dev = device or self.attn_qkvw.device
        self._rng = torch.tensor([int(seed), 0], dtype=torch.int64, device=dev)

    def forward(self, hidden_states, attention_mask=None, head_mask=None, encoder_hidden_states=None,
                encoder_attention_mask=None, output_attentions=False, grads=None):
        rng = getattr(self, "_rng", None)
        if rng is not None and self.training:
            from ...runtime.activation_checkpointing import checkpointing as ds_ckpt
            # a new training forward draws new masks -- including the first (no_grad) forward of
            # an activation checkpoint; its recompute inside backward must redraw the same masks,
            # so it does not advance (the recompute follows its own forward before the next
            # forward of this layer, as in gradient accumulation)
            if (torch.is_grad_enabled() or ds_ckpt.is_checkpoint_forward()) and not ds_ckpt.is_recomputing():
                rng[1:].add_(1)
        self.config.training = self.training
        self.config.is_grad_enabled = torch.is_grad_enabled()
        out = DeepSpeedTransformerFunction.apply(hidden_states, attention_mask, self, grads, self.config.layer_id,
                                                 self.attn_qkvw, self.attn_qkvb, self.attn_ow, self.attn_ob,
                                                 self.attn_nw, self.attn_nb, self.inter_w, self.inter_b,
                                                 self.output_w, self.output_b, self.norm_w, self.norm_b, self.config)
        return (out,) if self.config.huggingface else out


def chain_layer_norms(layers, final_norm=None, enabled: bool = True):
    """Let each pre-LN layer of `layers` (the ones that run, in order) normalise its output with
    the LayerNorm that reads it next -- the following layer's input LayerNorm, or `final_norm`
    (a FusedLayerNorm / nn.LayerNorm) after the last layer -- in the pass that forms the output
    (native.bias_dropout_residual_ln), so that LayerNorm is not a separate launch that re-reads the
    residual stream.  The result travels on the output tensor and is taken only by that owner; any
    other consumer recomputes the LayerNorm (same values).  Call before every forward whose set of
    layers can change (progressive layer drop); layers captured as HIP graphs are left unchained,
    and enabled=False unchains every layer."""
    def ln_of(mod):
        if isinstance(mod, DeepSpeedTransformerLayer):
            c = mod.config
            if c.pre_layer_norm and not getattr(c, "normalize_invertible", False) and not getattr(mod, "_dsa_graphed", False):
                return (mod, mod.norm_w, mod.norm_b, c.layer_norm_eps)
            return None
        if mod is not None and getattr(mod, "weight", None) is not None and hasattr(mod, "eps"):
            return (mod, mod.weight, getattr(mod, "bias", None), mod.eps)
        return None

    layers = list(layers)
    ours = [l for l in layers if isinstance(l, DeepSpeedTransformerLayer) and not getattr(l, "_dsa_graphed", False)]
    for i, layer in enumerate(ours):  # slots of the layer-stacked buffers (ops/wgrad_batch.py)
        object.__setattr__(layer, "_dsa_slab_index", i if enabled else None)
        object.__setattr__(layer, "_dsa_slab_count", len(ours))
    for i, layer in enumerate(layers):
        if not isinstance(layer, DeepSpeedTransformerLayer):
            continue
        nxt = None
        if enabled and native.BDR_LN and not getattr(layer, "_dsa_graphed", False):
            nxt = ln_of(layers[i + 1] if i + 1 < len(layers) else final_norm)
        object.__setattr__(layer, "_dsa_next_norm", nxt)


def take_chained_norm(x, owner):
    """The LayerNorm output chain_layer_norms' previous layer left on x for `owner`, or None."""
    pre = getattr(x, "_dsa_next_ln", None)
    return pre[1] if pre is not None and pre[0] is owner else None


def make_graphed_encoder(layers, sample_hidden, sample_mask=None, seed: int = 1234, warmup: int = 3,
                         persistent_grads: bool = True):
    """Capture every DeepSpeedTransformerLayer of `layers` (an nn.ModuleList, replaced in place)
    as HIP graphs -- one forward and one backward graph per layer (torch.cuda.make_graphed_callables)
    -- so a training step replays 2 x num_layers graphs instead of launching ~30 kernels per
    layer and direction from Python.  The layers' dropout then draws from device RNG state
    (`enable_device_rng`), advanced by a kernel inside the forward graph, so every replay gets
    fresh masks.  Shapes (batch, sequence) and the attention-mask layout are fixed by the
    samples; parameters keep receiving ordinary .grad tensors.

    The reference has no graph capture (CUDA graphs postdate DeepSpeed v0.3.15); the BERT layer it
    benchmarks is its ds_transformer_cuda op (csrc/transformer/ds_transformer_cuda.cpp)."""
    for i, layer in enumerate(layers):
        if not isinstance(layer, DeepSpeedTransformerLayer):
            raise TypeError("make_graphed_encoder: every layer must be a DeepSpeedTransformerLayer")
        # a graph replays its captured outputs only: no LayerNorm hand-over between layers
        object.__setattr__(layer, "_dsa_graphed", True)
        object.__setattr__(layer, "_dsa_next_norm", None)
        layer.enable_device_rng(seed + 7919 * i)
        for p in layer.parameters():  # the graphs hold these addresses: never rebound later
            p._dsa_graph_captured = True
        if persistent_grads:
            # the backward graphs accumulate weight / bias / LayerNorm gradients straight into these
            # buffers (ops/linear.py, native LayerNorm): no static gradient outputs to copy into .grad
            # after every replay; the optimizer zeroes them in place (FP16_UnfusedOptimizer.zero_grad)
            for p in layer.parameters():
                p.grad = torch.zeros_like(p)
                p._dsa_persistent_grad = True
    args = []
    for _ in layers:
        h = sample_hidden.detach().clone().requires_grad_(True)
        args.append((h,) if sample_mask is None else (h, sample_mask.detach()))
    graphed = torch.cuda.make_graphed_callables(tuple(layers), tuple(args), num_warmup_iters=warmup,
                                                allow_unused_input=persistent_grads)
    for i, g in enumerate(graphed):
        layers[i] = g
    if persistent_grads:  # the warmup iterations accumulated into the persistent buffers
        torch._foreach_zero_([p.grad for layer in layers for p in layer.parameters()])
    return layers
