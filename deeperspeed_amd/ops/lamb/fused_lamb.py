"""FusedLamb: LAMB on the HIP kernels (ops/csrc/kernels/optim.hip lamb_*).

Reference parity: deepspeed/ops/lamb/fused_lamb.py:12-189 (per-parameter launch, trust ratio
clamped to [min_coeff, max_coeff], `get_lamb_coeffs`).  Three launches per tensor (moments +
partial norms, norm finish, apply) with the coefficient kept on the device, so a step has no
host synchronisation; `get_lamb_coeffs()` syncs only when called.
"""

import torch

from .. import native


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

    supports_fused_lp_step = True  # FP16_UnfusedOptimizer passes low-precision grads/outputs

    @torch.no_grad()
    def step(self, closure=None, grads=None, output_params=None, scale=1.0, grad_norms=None):
        """`grads`/`output_params`/`scale` follow the reference's legacy fused interface:
        optional explicit gradient lists, low-precision output copies and a loss scale the
        gradients are divided by."""
        loss = closure() if closure is not None else None
        self.lamb_coeffs = []
        for gi, group in enumerate(self.param_groups):
            b1, b2 = group["betas"]
            g_list = grads[gi] if grads is not None else [None] * len(group["params"])
            o_list = output_params[gi] if output_params is not None else [None] * len(group["params"])
            for p, g, o in zip(group["params"], g_list, o_list):
                g = p.grad if g is None else g
                if g is None:
                    continue
                if o is not None and o.data_ptr() == p.data_ptr():
                    o = None
                if g.is_sparse:
                    raise RuntimeError("FusedLamb does not support sparse gradients")
                st = self.state[p]
                if len(st) == 0:
                    st["step"] = 0
                    st["exp_avg"] = torch.zeros(p.numel(), dtype=torch.float32, device=p.device)
                    st["exp_avg_sq"] = torch.zeros(p.numel(), dtype=torch.float32, device=p.device)
                st["step"] += 1
                w = p.data.view(-1)
                c = native.lamb_(w, g.contiguous().view(-1), st["exp_avg"], st["exp_avg_sq"],
                                 o.view(-1) if o is not None else None, group["lr"], b1, b2, group["eps"],
                                 group["weight_decay"], st["step"], group["bias_correction"], 1.0 / scale,
                                 group["max_coeff"], group["min_coeff"], self.eps_mode == 1)
                self.lamb_coeffs.append(c)
        return loss

    def get_lamb_coeffs(self):
        return [float(c) for c in self.lamb_coeffs]
