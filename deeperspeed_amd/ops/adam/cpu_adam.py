"""DeepSpeedCPUAdam: Adam/AdamW on host-resident fp32 parameters (ZeRO-Offload).

Reference parity: deepspeed/ops/adam/cpu_adam.py:12-176 (constructor, `step(closure,
fp16_param_groups)` that also refreshes low-precision device copies) backed by the native
AVX-512/AVX2 kernel in `_cpu_ops` (ops/csrc/cpu/cpu_adam.cpp).  The device copy is written
by the kernel into a pinned bf16/fp16 staging buffer and moved with a non-blocking H2D copy.
"""

from __future__ import annotations

import math

import torch

from .. import builder

_ops = None


def cpu_ops():
    global _ops
    if _ops is None:
        _ops = builder.load("_cpu_ops")
    return _ops


class _Staging:
    """Pinned staging buffers for host->device low-precision copies, double-buffered."""

    def __init__(self):
        self.bufs = {}
        self.events = {}
        self.flip = 0

    def get(self, n, dtype):
        self.flip ^= 1
        key = (dtype, self.flip)
        buf = self.bufs.get(key)
        ev = self.events.get(key)
        if ev is not None:
            ev.synchronize()
        if buf is None or buf.numel() < n:
            buf = torch.empty(max(n, 1 << 20), dtype=dtype, pin_memory=torch.cuda.is_available())
            self.bufs[key] = buf
        return key, buf[:n]

    def mark(self, key):
        if torch.cuda.is_available():
            ev = torch.cuda.Event()
            ev.record()
            self.events[key] = ev


_STAGING = _Staging()


def cpu_adam_update_flat(master, grad, exp_avg, exp_avg_sq, group, step, grad_scale, adamw, out_device=None):
    """Update host fp32 `master` in place; optionally refresh a device low-precision copy."""
    b1, b2 = group["betas"]
    if grad.device.type != "cpu":
        grad = grad.to("cpu")
    if grad.dtype not in (torch.float32, torch.bfloat16):  # the kernel widens bf16 itself
        grad = grad.float()
    out_host = None
    key = None
    if out_device is not None and out_device.device.type == "cuda":
        key, out_host = _STAGING.get(master.numel(), out_device.dtype)
    cpu_ops().adam_update(master, grad.contiguous(), exp_avg, exp_avg_sq, group["lr"], b1, b2, group["eps"],
                          group["weight_decay"], int(step), bool(group.get("bias_correction", True)),
                          float(grad_scale), bool(adamw), out_host)
    if out_device is not None:
        if out_host is not None:
            out_device.copy_(out_host, non_blocking=True)
            _STAGING.mark(key)
        else:
            out_device.copy_(master)


class DeepSpeedCPUAdam(torch.optim.Optimizer):
    optimizer_id = 0
    supports_flat_update = True

    def __init__(self, model_params, lr=1e-3, bias_correction=True, betas=(0.9, 0.999), eps=1e-8, weight_decay=0,
                 amsgrad=False, adamw_mode=True):
        if amsgrad:
            raise RuntimeError("DeepSpeedCPUAdam does not support the AMSGrad variant.")
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, bias_correction=bias_correction,
                        amsgrad=amsgrad)
        super().__init__(model_params, defaults)
        self.opt_id = DeepSpeedCPUAdam.optimizer_id
        DeepSpeedCPUAdam.optimizer_id += 1
        self.adam_w_mode = adamw_mode
        self.adamw_mode = adamw_mode

    def update_flat(self, group, state_key, w, g, out=None, grad_scale=1.0, lo=0, hi=None, step=None):
        st = self.state[state_key]
        hi = w.numel() if hi is None else hi
        cpu_adam_update_flat(w[lo:hi], g[lo:hi], st["exp_avg"][lo:hi], st["exp_avg_sq"][lo:hi], group,
                             step if step is not None else st["step"], grad_scale, self.adamw_mode, out)

    def state_for(self, p):
        st = self.state[p]
        if len(st) == 0:
            st["step"] = 0
            st["exp_avg"] = torch.zeros_like(p, dtype=torch.float32, device="cpu")
            st["exp_avg_sq"] = torch.zeros_like(p, dtype=torch.float32, device="cpu")
        return st

    @torch.no_grad()
    def step(self, closure=None, fp16_param_groups=None):
        loss = closure() if closure is not None else None
        for gi, group in enumerate(self.param_groups):
            for pi, p in enumerate(group["params"]):
                if p.grad is None:
                    continue
                assert p.device.type == "cpu", "DeepSpeedCPUAdam requires host parameters"
                st = self.state_for(p)
                st["step"] += 1
                out = None
                if fp16_param_groups is not None:
                    out = fp16_param_groups[gi][pi]
                cpu_adam_update_flat(p.data.view(-1), p.grad.view(-1), st["exp_avg"].view(-1),
                                     st["exp_avg_sq"].view(-1), group, st["step"], 1.0, self.adamw_mode,
                                     out.data.view(-1) if out is not None else None)
        return loss
