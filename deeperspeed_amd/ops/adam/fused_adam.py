"""FusedAdam on the CDNA4 HIP kernel.

Reference parity: deepspeed/ops/adam/fused_adam.py:15-182 (same constructor, L2 vs decoupled
weight decay via ``adam_w_mode``, bias correction, multi-tensor launch).  MI355X design:
one multi-tensor launch per (param dtype, grad dtype) class with the tensor table held in a
small device buffer (no 36-tensor kernel-argument limit), and a flat entry point
(``update_flat``) used by the ZeRO wrappers which updates an fp32 master shard and writes
the bf16/fp16 model copy in the same memory pass.
"""

import torch

from .. import native

_CHUNK = 65536


class FusedAdam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, bias_correction=True, betas=(0.9, 0.999), eps=1e-8, adam_w_mode=True,
                 weight_decay=0.0, amsgrad=False, set_grad_none=True):
        if amsgrad:
            raise RuntimeError("FusedAdam does not support the AMSGrad variant.")
        defaults = dict(lr=lr, bias_correction=bias_correction, betas=betas, eps=eps, weight_decay=weight_decay)
        super().__init__(params, defaults)
        self.adam_w_mode = 1 if adam_w_mode else 0
        self.set_grad_none = set_grad_none
        self._meta_cache = {}

    def zero_grad(self, set_to_none=None):
        if set_to_none is None:
            set_to_none = self.set_grad_none
        super().zero_grad(set_to_none=set_to_none)

    # ------------------------------------------------------------------ flat path (ZeRO)
    def state_for(self, p: torch.Tensor):
        st = self.state[p]
        if len(st) == 0:
            st["step"] = 0
            st["exp_avg"] = torch.zeros_like(p, dtype=torch.float32)
            st["exp_avg_sq"] = torch.zeros_like(p, dtype=torch.float32)
        return st

    def update_flat(self, group, state_key, w, g, out=None, grad_scale=1.0, lo=0, hi=None, step=None):
        """Update w[lo:hi] (fp32 master, or the param itself) from g[lo:hi]; moments live in
        self.state[state_key]. `out` (already sliced) receives the low-precision copy."""
        st = self.state_for(state_key)
        hi = w.numel() if hi is None else hi
        b1, b2 = group["betas"]
        if w.dtype == torch.int16:  # compact master: w holds the residual, `out` the bf16 high half
            native.adam_compact_(out, w[lo:hi], g[lo:hi], st["exp_avg"][lo:hi], st["exp_avg_sq"][lo:hi],
                                 group["lr"], b1, b2, group["eps"], group["weight_decay"],
                                 step if step is not None else st["step"], group["bias_correction"], grad_scale,
                                 bool(self.adam_w_mode))
            return
        native.adam_flat_(w[lo:hi], g[lo:hi], st["exp_avg"][lo:hi], st["exp_avg_sq"][lo:hi], out, group["lr"], b1, b2,
                          group["eps"], group["weight_decay"], step if step is not None else st["step"],
                          group["bias_correction"], grad_scale, bool(self.adam_w_mode))

    # ------------------------------------------------------------------ multi-tensor path
    def _meta(self, device, ws, gs, ms, vs, outs):
        key = tuple(t.data_ptr() for t in ws) + tuple(t.data_ptr() for t in gs)
        meta = self._meta_cache.get(key)
        if meta is None:
            T = len(ws)
            numels = [t.numel() for t in ws]
            chunks = [(n + _CHUNK - 1) // _CHUNK for n in numels]
            pref = [0]
            for c in chunks:
                pref.append(pref[-1] + c)
            rows = ([t.data_ptr() for t in ws] + [t.data_ptr() for t in gs] + [t.data_ptr() for t in ms] +
                    [t.data_ptr() for t in vs] + [(o.data_ptr() if o is not None else 0) for o in outs] + numels + pref)
            host = torch.tensor(rows, dtype=torch.int64).pin_memory() if torch.cuda.is_available() else \
                torch.tensor(rows, dtype=torch.int64)
            meta = (host.to(device, non_blocking=True), T, pref[-1])
            if len(self._meta_cache) > 64:
                self._meta_cache.clear()
            self._meta_cache[key] = meta
        return meta

    @torch.no_grad()
    def step(self, closure=None, grads=None, output_params=None, scale=1.0, grad_norms=None):
        loss = closure() if closure is not None else None
        for group in self.param_groups:
            buckets = {}
            for p in group["params"]:
                if p.grad is None:
                    continue
                if p.grad.is_sparse:
                    raise RuntimeError("FusedAdam does not support sparse gradients")
                st = self.state_for(p)
                st["step"] += 1
                key = (p.device, p.dtype, p.grad.dtype, st["step"])
                buckets.setdefault(key, []).append(p)
            for (dev, pdt, gdt, step), plist in buckets.items():
                if dev.type != "cuda":
                    for p in plist:
                        st = self.state[p]
                        native.adam_flat_(p.data, p.grad, st["exp_avg"], st["exp_avg_sq"], None, group["lr"],
                                          group["betas"][0], group["betas"][1], group["eps"], group["weight_decay"],
                                          step, group["bias_correction"], 1.0 / scale, bool(self.adam_w_mode))
                    continue
                ws = [p.data for p in plist]
                gs = [p.grad.contiguous() for p in plist]
                ms = [self.state[p]["exp_avg"] for p in plist]
                vs = [self.state[p]["exp_avg_sq"] for p in plist]
                outs = [None] * len(plist)
                meta, T, total = self._meta(dev, ws, gs, ms, vs, outs)
                b1, b2 = group["betas"]
                bc1 = 1 - b1 ** step if group["bias_correction"] else 1.0
                bc2 = 1 - b2 ** step if group["bias_correction"] else 1.0
                code = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2}
                native.hip_ops().adam_multi(meta, T, total, _CHUNK, code[pdt], code[gdt], 1, group["lr"], b1, b2,
                                            group["eps"], group["weight_decay"], bc1, bc2, 1.0 / scale,
                                            bool(self.adam_w_mode))
        return loss
