"""`"amp": {"enabled": true, ...}` mapped onto torch autocast (no apex on ROCm).

The reference hands the model and optimizer to apex `amp.initialize` (REF
deepspeed/runtime/engine.py:682-693), scales the loss with `amp.scale_loss` and delays the
unscale inside gradient accumulation (:1085-1093), and clips `amp.master_params`
(:1146-1155).  apex's O1/O2 keep fp32 master weights and run the matmuls in half precision.

Here the same contract is met natively:
  * the module stays fp32 -- its parameters ARE the fp32 masters -- and the engine's forward
    runs under `torch.autocast(<device>, dtype)` (bf16 by default: MFMA bf16 GEMMs on MI355X);
  * bf16 needs no loss scaling; with `"dtype": "float16"` a dynamic `torch.amp.GradScaler`
    plays apex's role (`loss_scale` = "dynamic" or a fixed number), and its unscale is delayed
    to the accumulation boundary like apex's `delay_unscale`;
  * gradient clipping runs on the unscaled fp32 parameters; an overflow skips the step and
    is counted like the fp16 optimizers' overflow;
  * the model is broadcast from the data-parallel source rank at init (apex path of the
    reference, :693-694).

Accepted keys: `dtype` ("bfloat16" | "float16"), `opt_level` ("O0" = plain fp32, "O1"/"O2"/"O3"
= autocast), `loss_scale`, `init_scale`, `growth_interval`; other apex keys
(`keep_batchnorm_fp32`, `master_weights`, `cast_model_type`, ...) are accepted and ignored
with a warning, since autocast has no equivalent switch.
"""

from __future__ import annotations

import contextlib
from typing import Optional

import torch

from ..utils.logging import logger

_DTYPES = {"bfloat16": torch.bfloat16, "bf16": torch.bfloat16, "float16": torch.float16, "fp16": torch.float16,
           "half": torch.float16}
_KNOWN = {"dtype", "opt_level", "loss_scale", "init_scale", "growth_interval"}


class AmpState:
    def __init__(self, params: Optional[dict], device: torch.device):
        params = dict(params or {})
        unknown = sorted(set(params) - _KNOWN)
        if unknown:
            logger.warning(f"amp: keys {unknown} have no autocast equivalent and are ignored")
        name = str(params.get("dtype", "bfloat16")).lower()
        if name not in _DTYPES:
            raise ValueError(f"amp.dtype must be one of {sorted(_DTYPES)}, got {params.get('dtype')!r}")
        self.dtype = _DTYPES[name]
        self.opt_level = str(params.get("opt_level", "O1")).upper()
        if self.opt_level not in ("O0", "O1", "O2", "O3"):
            raise ValueError(f"amp.opt_level must be O0..O3, got {self.opt_level!r}")
        self.enabled = self.opt_level != "O0"
        self.device_type = "cuda" if device.type == "cuda" else "cpu"
        self.scaler = None
        self.static_scale = None
        if self.enabled and self.dtype == torch.float16:
            ls = params.get("loss_scale", "dynamic")
            dynamic = ls in (None, "dynamic", 0, 0.0)
            init = float(params.get("init_scale", 2.0 ** 16)) if dynamic else float(ls)
            # a fixed loss_scale uses the scaler's default factors (torch asserts growth > 1 and
            # backoff < 1) and pins the scale back after every update
            self.static_scale = None if dynamic else init
            self.scaler = torch.amp.GradScaler(self.device_type, init_scale=init,
                                               growth_interval=int(params.get("growth_interval", 2000)))
        self.overflow = False
        self._unscaled = False

    def autocast(self):
        if not self.enabled:
            return contextlib.nullcontext()
        return torch.autocast(self.device_type, dtype=self.dtype)

    def scale(self, loss: torch.Tensor) -> torch.Tensor:
        return self.scaler.scale(loss) if self.scaler is not None else loss

    @property
    def loss_scale(self) -> float:
        return float(self.scaler.get_scale()) if self.scaler is not None else 1.0

    def unscale(self, optimizer):
        """Unscale the accumulated gradients once, at the accumulation boundary (apex's
        delay_unscale=False on the boundary micro-batch)."""
        if self.scaler is not None and not self._unscaled:
            self.scaler.unscale_(optimizer)
            self._unscaled = True

    def step(self, optimizer):
        """optimizer.step() unless the scaled gradients overflowed; returns True if stepped."""
        if self.scaler is None:
            optimizer.step()
            self.overflow = False
            return True
        self.unscale(optimizer)
        # overflow = the unscale's found-inf flags (a static scale never backs off, so comparing
        # scales before / after the update would miss its skipped steps)
        found = self.scaler._found_inf_per_device(optimizer)
        self.overflow = bool(sum(float(v.item()) for v in found.values()) > 0)
        self.scaler.step(optimizer)  # skips the update when a found-inf flag is set
        if self.static_scale is not None:
            self.scaler.update(new_scale=self.static_scale)
        else:
            self.scaler.update()
        self._unscaled = False
        return not self.overflow

    def state_dict(self):
        return {"scaler": self.scaler.state_dict() if self.scaler is not None else None}

    def load_state_dict(self, sd):
        if self.scaler is not None and sd and sd.get("scaler"):
            self.scaler.load_state_dict(sd["scaler"])
