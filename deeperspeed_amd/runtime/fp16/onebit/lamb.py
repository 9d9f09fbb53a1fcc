"""1-bit LAMB (https://arxiv.org/abs/2104.06069).

Reference parity: deepspeed/runtime/fp16/onebit/lamb.py:14-471.
* warm-up: LAMB with per-tensor trust ratio; an EMA of the coefficient (`coeff_beta`) is kept;
* at freeze: per-tensor `scaling_coeff` = mean momentum scale / own scale (so all momenta share
  one compression scale), momenta fused into one flat buffer compressed-all-reduced per step;
* compression stage: variance frozen, a fresh variance is tracked from the reconstructed
  gradient, and the coefficient = frozen coefficient * a bounded, rate-limited factor
  (`factor_max`, `factor_min`, `factor_threshold`).
No CuPy warm-up call (see OnebitAdam).
"""

import numpy as np
import torch
from torch._utils import _flatten_dense_tensors, _unflatten_dense_tensors

from ....utils.logging import logger


class OnebitLamb(torch.optim.Optimizer):
    def __init__(self, params, deepspeed=None, lr=1e-3, freeze_step=100000, bias_correction=True, betas=(0.9, 0.999),
                 eps=1e-8, eps_inside_sqrt=False, weight_decay=0., max_grad_norm=0., max_coeff=10.0, min_coeff=0.01,
                 amsgrad=False, cuda_aware=False, comm_backend_name="nccl", coeff_beta=0.9, factor_max=4.0,
                 factor_min=0.5, factor_threshold=0.1):
        if amsgrad:
            raise RuntimeError("1-bit Lamb does not support the AMSGrad variant.")
        defaults = dict(lr=lr, bias_correction=bias_correction, betas=betas, eps=eps, weight_decay=weight_decay,
                        max_grad_norm=max_grad_norm, max_coeff=max_coeff, min_coeff=min_coeff)
        super().__init__(params, defaults)
        self.eps_mode = 0 if eps_inside_sqrt else 1
        self.deepspeed = deepspeed
        self.lamb_freeze_key = False
        self.freeze_step = freeze_step
        self.coeff_beta, self.factor_max, self.factor_min = coeff_beta, factor_max, factor_min
        self.factor_threshold = factor_threshold
        self.using_pipeline = bool(deepspeed is not None and hasattr(deepspeed, "pipeline_enable_backward_allreduce"))
        self.requires_per_param_masters = True
        mpu = getattr(deepspeed, "mpu", None) if deepspeed is not None else None
        if comm_backend_name == "nccl":
            from ...comm.nccl import NcclBackend
            self.comm_backend_handle = NcclBackend(mpu)
        elif comm_backend_name == "mpi":
            from ...comm.mpi import MpiBackend
            self.comm_backend_handle = MpiBackend(cuda_aware)
        else:
            raise ValueError(f"unknown comm backend {comm_backend_name}")
        self.size = self.comm_backend_handle.size
        self.divider = int(self.size * 8 / np.gcd(self.size, 8))
        self.exp_avg_flat, self.dummy_exp_avg = [], {}
        self.corrected_tensor_sizes, self.server_chunk_sizes = [], []
        self.worker_errors, self.server_errors = [], []
        self.lamb_coeffs = []

    def _set_backward_allreduce(self, enabled):
        if self.deepspeed is None:
            return
        if self.using_pipeline:
            self.deepspeed.pipeline_enable_backward_allreduce = enabled
        else:
            self.deepspeed.enable_backward_allreduce = enabled

    def _params(self):
        return [p for g in self.param_groups for p in g["params"]]

    def _denom(self, v, eps):
        return v.sqrt().add(eps) if self.eps_mode == 1 else (v + eps).sqrt()

    def _fuse_momenta(self):
        moms, size = [], 0
        for p in self._params():
            moms.append(self.state[p]["exp_avg"])
            size += p.numel()
        q = self.size * self.divider
        corrected = (size + q - 1) // q * q
        if corrected != size:
            self.dummy_exp_avg[0] = torch.zeros(corrected - size, device=moms[0].device)
            moms.append(self.dummy_exp_avg[0])
        self.corrected_tensor_sizes = [corrected]
        self.server_chunk_sizes = [corrected // self.size]
        flat = _flatten_dense_tensors([m.detach().clone() for m in moms])
        for m, q_ in zip(moms, _unflatten_dense_tensors(flat, moms)):
            m.data = q_.data  # momenta become views of the fused buffer
        self.exp_avg_flat = [flat]

    @torch.no_grad()
    def step(self, closure=None, grads=None):
        loss = closure() if closure is not None else None
        self.lamb_coeffs = []
        params = [p for p in self._params() if p.grad is not None]
        if self.lamb_freeze_key:
            last = {p: self.state[p]["exp_avg"].detach().clone() for p in params}
            if "scaling_coeff" not in self.state[params[0]]:
                scales = {p: (self.state[p]["exp_avg"].norm() / np.sqrt(p.numel())).item() for p in params}
                united = sum(scales.values()) / len(scales)
                for p in params:
                    self.state[p]["scaling_coeff"] = united / scales[p] if scales[p] > 0 else 1.0
        for group in self.param_groups:
            b1, b2 = group["betas"]
            for p in group["params"]:
                if p.grad is None:
                    continue
                grad = p.grad.data
                st = self.state[p]
                if "step" not in st:
                    st["step"] = 0
                    st["lamb_coeff_freeze"] = 0.0
                    st["last_factor"] = 1.0
                    st["exp_avg"] = torch.zeros_like(p.data)
                    st["exp_avg_sq"] = torch.zeros_like(p.data)
                    st["exp_avg_sq_fresh"] = torch.zeros_like(p.data)
                exp_avg, exp_avg_sq = st["exp_avg"], st["exp_avg_sq"]
                st["step"] += 1
                if not self.lamb_freeze_key:
                    exp_avg.mul_(b1).add_(grad, alpha=1 - b1)
                    exp_avg_sq.mul_(b2).addcmul_(grad, grad, value=1 - b2)
                    if st["step"] == self.freeze_step:
                        st["exp_avg_sq_fresh"].data = exp_avg_sq.detach().clone()
                    wn = p.data.float().norm()
                    update = exp_avg / self._denom(exp_avg_sq, group["eps"])
                    if group["weight_decay"] > 0.0:
                        update = update + group["weight_decay"] * p.data
                    un = update.norm()
                    c = 1.0
                    if wn != 0 and un != 0:
                        c = min(max((wn / un).item(), group["min_coeff"]), group["max_coeff"])
                    if c != 1.0:
                        st["lamb_coeff_freeze"] = self.coeff_beta * st["lamb_coeff_freeze"] + (1 - self.coeff_beta) * c
                    self.lamb_coeffs.append(c)
                    p.data.add_(update, alpha=-group["lr"] * c)
                else:
                    exp_avg.mul_(b1).add_(grad, alpha=1 - b1)
                    exp_avg.mul_(st["scaling_coeff"])
        if self.lamb_freeze_key:
            if not self.exp_avg_flat:
                self._fuse_momenta()
            if not self.worker_errors:
                self.worker_errors = [torch.zeros(self.corrected_tensor_sizes[0], device=self.exp_avg_flat[0].device)]
                self.server_errors = [torch.zeros(self.server_chunk_sizes[0], device=self.exp_avg_flat[0].device)]
            if self.size > 1:
                self.comm_backend_handle.compressed_allreduce(self.exp_avg_flat[0], self.worker_errors[0],
                                                              self.server_errors[0],
                                                              getattr(self.deepspeed, "local_rank", 0))
            for group in self.param_groups:
                b1, b2 = group["betas"]
                for p in group["params"]:
                    if p.grad is None:
                        continue
                    st = self.state[p]
                    exp_avg, exp_avg_sq, fresh = st["exp_avg"], st["exp_avg_sq"], st["exp_avg_sq_fresh"]
                    exp_avg.div_(st["scaling_coeff"])
                    if "exp_avg_mask" in group:
                        exp_avg.mul_(group["exp_avg_mask"].to(exp_avg.device))
                    g_rec = (exp_avg - last[p] * b1) / (1 - b1)
                    fresh.mul_(b2).addcmul_(g_rec, g_rec, value=1 - b2)
                    denom = self._denom(exp_avg_sq, group["eps"])
                    prelim = exp_avg / denom
                    update = prelim + group["weight_decay"] * p.data if group["weight_decay"] > 0.0 else prelim
                    un = update.norm()
                    factor = (denom / self._denom(fresh, group["eps"])).max().item()
                    if group["weight_decay"] > 0.0:
                        ratio = min(1.0, (prelim.norm() / un).item()) if un > 0 else 1.0
                        factor = factor * ratio + (1.0 - ratio)
                    factor = min(max(factor, self.factor_min), self.factor_max)
                    factor = min(factor, st["last_factor"] * (1.0 + self.factor_threshold))
                    factor = max(factor, st["last_factor"] * (1.0 - self.factor_threshold))
                    st["last_factor"] = factor
                    c = st["lamb_coeff_freeze"] * factor
                    self.lamb_coeffs.append(c)
                    p.data.add_(update, alpha=-group["lr"] * c)
        if not self.lamb_freeze_key:
            st0 = self.state[self._params()[0]]
            if st0.get("step", 0) >= self.freeze_step:
                logger.info("OnebitLamb - starting compressed communication")
                self.lamb_freeze_key = True
                self._set_backward_allreduce(False)
        return loss

    def get_lamb_coeffs(self):
        return list(self.lamb_coeffs)

    def load_state_dict(self, state_dict):
        for i, group in enumerate(self.param_groups):
            if "exp_avg_mask" in group:
                state_dict["param_groups"][i]["exp_avg_mask"] = group["exp_avg_mask"]
            elif "exp_avg_mask" in state_dict["param_groups"][i]:
                state_dict["param_groups"][i].pop("exp_avg_mask")
        super().load_state_dict(state_dict)
        self.exp_avg_flat, self.dummy_exp_avg = [], {}
        self.worker_errors, self.server_errors = [], []
        st0 = self.state[self._params()[0]]
        frozen = st0.get("step", 0) >= self.freeze_step
        self.lamb_freeze_key = frozen
        self._set_backward_allreduce(not frozen)
        for p in self._params():
            self.state[p].pop("worker_error", None)
            self.state[p].pop("server_error", None)
