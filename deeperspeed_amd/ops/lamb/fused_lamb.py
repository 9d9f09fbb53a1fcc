"""FusedLamb: LAMB on the HIP kernels (ops/csrc/kernels/optim.hip lamb_*).

Reference parity: deepspeed/ops/lamb/fused_lamb.py:12-189 (per-parameter launch, trust ratio
clamped to [min_coeff, max_coeff], `get_lamb_coeffs`).  On the GPU the whole parameter list is
updated by three multi-tensor launches (per-chunk moments + partial norms, per-tensor trust
ratios, apply) instead of the reference's kernel per tensor; coefficients stay on the device,
so a step has no host synchronisation and `get_lamb_coeffs()` syncs only when called.
"""

import torch

from .. import native

_CHUNK = 65536  # elements per block of the multi-tensor kernels


class FusedLamb(torch.optim.Optimizer):
    """LAMB (https://arxiv.org/abs/1904.00962).

    Args: params, lr=1e-3, bias_correction=True, betas=(0.9, 0.999), eps=1e-8,
    eps_inside_sqrt=False, weight_decay=0., max_grad_norm=0., max_coeff=10.0,
    min_coeff=0.01, amsgrad=False (unsupported).
    """

    def __init__(self, params, lr=1e-3, bias_correction=True, betas=(0.9, 0.999), eps=1e-8, eps_inside_sqrt=False,
                 weight_decay=0., max_grad_norm=0., max_coeff=10.0, min_coeff=0.01, amsgrad=False):
        if amsgrad:
            raise RuntimeError("FusedLamb does not support the AMSGrad variant.")
        defaults = dict(lr=lr, bias_correction=bias_correction, betas=betas, eps=eps, weight_decay=weight_decay,
                        max_grad_norm=max_grad_norm, max_coeff=max_coeff, min_coeff=min_coeff)
        super().__init__(params, defaults)
        self.eps_mode = 0 if eps_inside_sqrt else 1
        self.lamb_coeffs = []
        self.requires_per_param_masters = True  # trust ratio is per tensor: never flatten
        self.multi_tensor = True  # GPU: one multi-tensor launch set per (dtype, step) bucket
        self._meta_cache = {}
        self._dev_step = None  # param group -> device step counter (enable_device_step)

    supports_fused_lp_step = True  # FP16_UnfusedOptimizer passes low-precision grads/outputs

    @property
    def supports_device_scale(self):
        """step(scale_tensor=...) is honoured (the multi-tensor GPU kernels read it)."""
        return self.multi_tensor

    def enable_device_step(self):
        """Keep each param group's step counter on the GPU and form the bias-corrected step size
        lr * sqrt(1 - b2^t) / (1 - b1^t) there (a few scalar kernels per group and step), so a HIP
        graph captured around a whole training step (`scripts/bench_bert.py --hip-graphs step`)
        advances it on every replay.  The host-side state["step"] only advances on eager steps;
        `device_step(gi)` holds the true count."""
        if self._dev_step is None:
            self._dev_step = {}

    def device_step(self, gi=0):
        return None if self._dev_step is None else self._dev_step.get(gi)

    def _device_lr(self, gi, group, dev):
        t = self._dev_step.get(gi)
        if t is None:
            steps = [self.state[p]["step"] for p in group["params"] if len(self.state[p])]
            t = self._dev_step[gi] = torch.tensor(float(steps[0] if steps else 0), dtype=torch.float64, device=dev)
        t.add_(1)
        b1, b2 = group["betas"]
        if not group["bias_correction"]:
            return torch.full((1,), group["lr"], dtype=torch.float32, device=dev)
        return (group["lr"] * torch.sqrt(1.0 - torch.pow(b2, t)) / (1.0 - torch.pow(b1, t))).float().reshape(1)

    @torch.no_grad()
    def step(self, closure=None, grads=None, output_params=None, scale=1.0, grad_norms=None, scale_tensor=None):
        """`grads`/`output_params`/`scale` follow the reference's legacy fused interface:
        optional explicit gradient lists, low-precision output copies and a loss scale the
        gradients are divided by.  GPU tensors of one (dtype, step) bucket are updated by the
        multi-tensor kernels: three launches for the whole bucket (per-chunk partial norms,
        per-tensor trust ratios, apply)."""
        loss = closure() if closure is not None else None
        self.lamb_coeffs = []
        for gi, group in enumerate(self.param_groups):
            b1, b2 = group["betas"]
            g_list = grads[gi] if grads is not None else [None] * len(group["params"])
            o_list = output_params[gi] if output_params is not None else [None] * len(group["params"])
            buckets = {}
            for p, g, o in zip(group["params"], g_list, o_list):
                g = p.grad if g is None else g
                if g is None:
                    continue
                if g.is_sparse:
                    raise RuntimeError("FusedLamb does not support sparse gradients")
                if o is not None and o.data_ptr() == p.data_ptr():
                    o = None
                st = self.state[p]
                if len(st) == 0:
                    st["step"] = 0
                    st["exp_avg"] = torch.zeros(p.numel(), dtype=torch.float32, device=p.device)
                    st["exp_avg_sq"] = torch.zeros(p.numel(), dtype=torch.float32, device=p.device)
                st["step"] += 1
                if scale_tensor is not None and not (p.is_cuda and self.multi_tensor):
                    raise RuntimeError("FusedLamb: scale_tensor needs the multi-tensor GPU path")
                if p.is_cuda and self.multi_tensor:
                    key = (p.device, p.dtype, g.dtype, o.dtype if o is not None else None, st["step"])
                    buckets.setdefault(key, []).append((p, g.contiguous(), o))
                    continue
                c = native.lamb_(p.data.view(-1), g.contiguous().view(-1), st["exp_avg"], st["exp_avg_sq"],
                                 o.view(-1) if o is not None else None, group["lr"], b1, b2, group["eps"],
                                 group["weight_decay"], st["step"], group["bias_correction"], 1.0 / scale,
                                 group["max_coeff"], group["min_coeff"], self.eps_mode == 1)
                self.lamb_coeffs.append(c)
            lr_dev = None
            if buckets and self._dev_step is not None:
                lr_dev = self._device_lr(gi, group, next(iter(buckets))[0])
            for (dev, pdt, gdt, odt, step), items in buckets.items():
                self.lamb_coeffs.append(self._multi_step(dev, pdt, gdt, odt, step, items, group, 1.0 / scale,
                                                         scale_tensor, lr_dev))
        return loss

    @torch.no_grad()
    def step_subset(self, gi, idxs, grads, output_params=None, scale_tensor=None):
        """Update only parameters `idxs` of param group `gi` (one bucket of an overlapped step,
        runtime/overlap_step.py).  grads / output_params: lists aligned with those indices.
        scale_tensor: one fp32 on the device multiplied into the gradients (unscale x clip formed
        on the GPU); a non-finite value makes the kernels skip the update.  Returns the trust
        ratios of the bucket (device tensors)."""
        group = self.param_groups[gi]
        buckets = {}
        for i, g, o in zip(idxs, grads, output_params or [None] * len(idxs)):
            p = group["params"][i]
            if g is None:
                continue
            if o is not None and o.data_ptr() == p.data_ptr():
                o = None
            st = self.state[p]
            if len(st) == 0:
                st["step"] = 0
                st["exp_avg"] = torch.zeros(p.numel(), dtype=torch.float32, device=p.device)
                st["exp_avg_sq"] = torch.zeros(p.numel(), dtype=torch.float32, device=p.device)
            st["step"] += 1
            key = (p.device, p.dtype, g.dtype, o.dtype if o is not None else None, st["step"])
            buckets.setdefault(key, []).append((p, g.contiguous(), o))
        return [self._multi_step(dev, pdt, gdt, odt, step, items, group, 1.0, scale_tensor)
                for (dev, pdt, gdt, odt, step), items in buckets.items()]

    def _multi_step(self, dev, pdt, gdt, odt, step, items, group, grad_scale, scale_tensor=None, lr_dev=None):
        import math
        ws = [p.data for p, _, _ in items]
        gs = [g for _, g, _ in items]
        ms = [self.state[p]["exp_avg"] for p, _, _ in items]
        vs = [self.state[p]["exp_avg_sq"] for p, _, _ in items]
        outs = [o for _, _, o in items]
        key = tuple(t.data_ptr() for t in ws + gs) + tuple(o.data_ptr() if o is not None else 0 for o in outs)
        hit = self._meta_cache.get(key)
        if hit is None and dev.type == "cuda" and torch.cuda.is_current_stream_capturing():
            raise RuntimeError("FusedLamb: new parameter / gradient addresses while a HIP graph is being captured; "
                               "give the parameters persistent gradients first (runtime/step_graph.persistent_grads)")
        if hit is None:
            numels = [t.numel() for t in ws]
            pref = [0]
            for n in numels:
                pref.append(pref[-1] + (n + _CHUNK - 1) // _CHUNK)
            rows = ([t.data_ptr() for t in ws] + [t.data_ptr() for t in gs] + [t.data_ptr() for t in ms] +
                    [t.data_ptr() for t in vs] + [(o.data_ptr() if o is not None else 0) for o in outs] + numels
                    + pref)
            # pinned staging + async copy: a pageable H2D copy would wait for the whole stream
            # (the gradients are new tensors every step, so this runs every step).  The pinned
            # table stays referenced: a graph that captured the copy re-reads it on every replay.
            host = torch.tensor(rows, dtype=torch.int64).pin_memory()
            meta = host.to(dev, non_blocking=True)
            hit = (meta, len(ws), pref[-1], torch.empty(2 * pref[-1], dtype=torch.float32, device=dev), host)
            if len(self._meta_cache) > 64:
                self._meta_cache.clear()
            self._meta_cache[key] = hit
        meta, T, total, partial, _ = hit
        b1, b2 = group["betas"]
        bc1 = 1.0 - b1 ** step if group["bias_correction"] else 1.0
        bc2 = 1.0 - b2 ** step if group["bias_correction"] else 1.0
        code = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2}
        coeff = torch.empty(T, dtype=torch.float32, device=dev)
        native.hip_ops().lamb_multi(meta, T, total, _CHUNK, code[pdt], code[gdt], code[odt or pdt],
                                    group["lr"] * math.sqrt(bc2) / bc1, b1, b2, group["eps"], group["weight_decay"],
                                    bc1, bc2, grad_scale, group["max_coeff"], group["min_coeff"],
                                    self.eps_mode == 1, partial, coeff, scale_tensor, lr_dev)
        return coeff

    def get_lamb_coeffs(self):
        return [float(x) for c in self.lamb_coeffs for x in c.reshape(-1).tolist()]
