"""1-bit Adam (https://arxiv.org/abs/2102.02888): error-compensated 1-bit momentum
communication after a full-precision warm-up.

Reference parity: deepspeed/runtime/fp16/onebit/adam.py:14-322.
* warm-up (step < freeze_step): plain Adam on engine-all-reduced gradients (no bias
  correction, as in the reference);
* compression stage: the engine stops all-reducing gradients (`enable_backward_allreduce`
  False); each rank folds its LOCAL gradient into the momentum, the momentum is averaged with
  `compressed_allreduce` (worker/server error feedback), the frozen variance is reused;
* `exp_avg_mask` param-group entry zeroes momentum entries that must stay exactly zero;
* checkpoints reset the compression errors (the reference does the same).
Difference: the reference's first `step()` only allocates CuPy buffers and skips the update;
there is no such warm-up call here.
"""

import numpy as np
import torch
import torch.distributed as dist

from ....utils.logging import logger


class OnebitAdam(torch.optim.Optimizer):
    def __init__(self, params, deepspeed=None, lr=1e-3, freeze_step=100000, bias_correction=True, betas=(0.9, 0.999),
                 eps=1e-8, eps_inside_sqrt=False, weight_decay=0., max_grad_norm=0., amsgrad=False, cuda_aware=False,
                 comm_backend_name="nccl"):
        if amsgrad:
            raise RuntimeError("1-bit Adam does not support the AMSGrad variant.")
        defaults = dict(lr=lr, bias_correction=bias_correction, betas=betas, eps=eps, weight_decay=weight_decay,
                        max_grad_norm=max_grad_norm)
        super().__init__(params, defaults)
        self.eps_mode = 0 if eps_inside_sqrt else 1
        self.deepspeed = deepspeed
        self.freeze_step = freeze_step
        self.adam_freeze_key = False
        self.cuda_aware = cuda_aware
        self.using_pipeline = bool(deepspeed is not None and hasattr(deepspeed, "pipeline_enable_backward_allreduce"))
        self.requires_per_param_masters = True
        self.comm_backend_name = comm_backend_name
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

    def _set_backward_allreduce(self, enabled):
        if self.deepspeed is None:
            return
        if self.using_pipeline:
            self.deepspeed.pipeline_enable_backward_allreduce = enabled
        else:
            self.deepspeed.enable_backward_allreduce = enabled

    def _init_state(self, p):
        st = self.state[p]
        st["step"] = 0
        st["exp_avg"] = torch.zeros_like(p.data)
        st["exp_avg_sq"] = torch.zeros_like(p.data)
        st["tensor_size"] = p.numel()
        q = self.size * self.divider
        st["corrected_tensor_size"] = (p.numel() + q - 1) // q * q
        st["server_chunk_size"] = st["corrected_tensor_size"] // self.size

    @torch.no_grad()
    def step(self, closure=None, grads=None):
        loss = closure() if closure is not None else None
        for group in self.param_groups:
            b1, b2 = group["betas"]
            for p in group["params"]:
                if p.grad is None:
                    continue
                grad = p.grad.data
                if grad.is_sparse:
                    raise RuntimeError("1-bit Adam does not support sparse gradients")
                st = self.state[p]
                if len(st) == 0:
                    self._init_state(p)
                if self.adam_freeze_key and "worker_error" not in st:
                    st["worker_error"] = torch.zeros(st["corrected_tensor_size"], device=p.device)
                    st["server_error"] = torch.zeros(st["server_chunk_size"], device=p.device)
                exp_avg, exp_avg_sq = st["exp_avg"], st["exp_avg_sq"]
                st["step"] += 1
                if not self.adam_freeze_key:
                    exp_avg.mul_(b1).add_(grad, alpha=1 - b1)
                    exp_avg_sq.mul_(b2).addcmul_(grad, grad, value=1 - b2)
                elif group.get("non_freeze", False):
                    dist.all_reduce(grad)
                    grad.mul_(1.0 / dist.get_world_size())
                    exp_avg.mul_(b1).add_(grad, alpha=1 - b1)
                    exp_avg_sq.mul_(b2).addcmul_(grad, grad, value=1 - b2)
                else:
                    exp_avg.mul_(b1).add_(grad, alpha=1 - b1)
                    if self.size > 1:
                        self.comm_backend_handle.compressed_allreduce(exp_avg, st["worker_error"], st["server_error"],
                                                                      getattr(self.deepspeed, "local_rank", 0))
                    if "exp_avg_mask" in group:
                        if group["exp_avg_mask"].device != exp_avg.device:
                            group["exp_avg_mask"] = group["exp_avg_mask"].to(exp_avg.device)
                        exp_avg.mul_(group["exp_avg_mask"])
                denom = exp_avg_sq.sqrt().add_(group["eps"]) if self.eps_mode == 1 else (exp_avg_sq + group["eps"]).sqrt()
                update = exp_avg / denom
                if group["weight_decay"] > 0.0:
                    update.add_(p.data, alpha=group["weight_decay"])
                p.data.add_(update, alpha=-group["lr"])
        if not self.adam_freeze_key:
            st0 = self.state[self.param_groups[0]["params"][0]]
            if st0.get("step", 0) >= self.freeze_step:
                logger.info("OnebitAdam - starting compressed communication")
                self.adam_freeze_key = True
                self._set_backward_allreduce(False)
        return loss

    def load_state_dict(self, state_dict):
        for i, group in enumerate(self.param_groups):
            if "exp_avg_mask" in group:
                state_dict["param_groups"][i]["exp_avg_mask"] = group["exp_avg_mask"]
            elif "exp_avg_mask" in state_dict["param_groups"][i]:
                state_dict["param_groups"][i].pop("exp_avg_mask")
        super().load_state_dict(state_dict)
        st0 = self.state[self.param_groups[0]["params"][0]]
        frozen = st0.get("step", 0) >= self.freeze_step
        self.adam_freeze_key = frozen
        self._set_backward_allreduce(not frozen)
        for group in self.param_groups:
            for p in group["params"]:
                self.state[p].pop("worker_error", None)
                self.state[p].pop("server_error", None)
