"""Static and dynamic loss scaling (reference parity: deepspeed/runtime/fp16/loss_scaler.py:1-223).

Semantics kept: hysteresis (`delayed_shift`) before each scale decrease, growth by
`scale_factor` after `scale_window` clean iterations, error when an overflow happens at
`min_scale`.  Overflow detection itself is done on device by the optimizer wrappers
(one fused sum-of-squares over the flat gradient shard, no per-tensor host syncs).
"""

import torch


class LossScaleUnderflowError(Exception):
    """Raised when gradients overflow although the dynamic loss scale is at its minimum."""


class LossScalerBase:
    def __init__(self, cur_scale):
        self.cur_scale = cur_scale
        self.dynamic = False

    @property
    def loss_scale(self):
        return self.cur_scale

    def scale_gradient(self, module, grad_in, grad_out):
        return tuple(self.loss_scale * g for g in grad_in)

    def update_scale(self, overflow):
        pass

    def backward(self, loss, retain_graph=False):
        scaled_loss = loss * self.loss_scale
        scaled_loss.backward(retain_graph=retain_graph)

    def state_dict(self):
        return {"cur_scale": self.cur_scale, "dynamic": self.dynamic}

    def load_state_dict(self, sd):
        self.cur_scale = sd.get("cur_scale", self.cur_scale)


class LossScaler(LossScalerBase):
    """Static loss scale."""

    def __init__(self, scale=1):
        super().__init__(scale)

    def has_overflow(self, params):
        return False

    @staticmethod
    def _has_inf_or_nan(x):
        return False


class DynamicLossScaler(LossScalerBase):
    def __init__(self, init_scale=2 ** 32, scale_factor=2.0, scale_window=1000, min_scale=1, delayed_shift=1,
                 consecutive_hysteresis=False, raise_error_at_min_scale=True):
        super().__init__(init_scale)
        self.cur_iter = 0
        self.last_overflow_iter = -1
        self.scale_factor = scale_factor
        self.scale_window = scale_window
        self.min_scale = min_scale
        self.delayed_shift = delayed_shift
        self.cur_hysteresis = delayed_shift
        self.consecutive_hysteresis = consecutive_hysteresis
        self.raise_error_at_min_scale = raise_error_at_min_scale
        self.dynamic = True

    def has_overflow_serial(self, params):
        for p in params:
            if p.grad is not None and self._has_inf_or_nan(p.grad.data):
                return True
        return False

    def has_overflow(self, params):
        return self.has_overflow_serial(params)

    @staticmethod
    def _has_inf_or_nan(x):
        s = float(x.float().sum())
        return s != s or s in (float("inf"), float("-inf"))

    def update_scale(self, overflow):
        """Advance one iteration.  An overflow first spends the hysteresis budget
        (`delayed_shift - 1` tolerated overflows), then divides the scale (never below
        `min_scale`; overflowing AT the minimum is fatal when raise_error_at_min_scale).
        Every `scale_window` iterations after the last overflow the scale grows by
        `scale_factor` and the budget refills (consecutive_hysteresis refills it on every
        clean iteration)."""
        it = self.cur_iter
        self.cur_iter = it + 1
        if overflow:
            self.last_overflow_iter = it
            if self.delayed_shift > 1 and self.cur_hysteresis > 1:
                self.cur_hysteresis -= 1
                return
            if self.raise_error_at_min_scale and self.cur_scale == self.min_scale:
                raise LossScaleUnderflowError(
                    f"gradients overflow at the minimum loss scale ({self.min_scale}); the run cannot continue")
            self.cur_scale = max(self.min_scale, self.cur_scale / self.scale_factor)
            return
        grow = (it - self.last_overflow_iter) % self.scale_window == 0
        if grow or self.consecutive_hysteresis:
            self.cur_hysteresis = self.delayed_shift
        if grow:
            self.cur_scale *= self.scale_factor

    def state_dict(self):
        sd = super().state_dict()
        sd.update(cur_iter=self.cur_iter, last_overflow_iter=self.last_overflow_iter,
                  cur_hysteresis=self.cur_hysteresis)
        return sd

    def load_state_dict(self, sd):
        super().load_state_dict(sd)
        self.cur_iter = sd.get("cur_iter", self.cur_iter)
        self.last_overflow_iter = sd.get("last_overflow_iter", self.last_overflow_iter)
        self.cur_hysteresis = sd.get("cur_hysteresis", self.cur_hysteresis)


def make_loss_scaler(static_loss_scale=1.0, dynamic=False, dynamic_args=None):
    if dynamic:
        args = dict(dynamic_args or {})
        return DynamicLossScaler(**args)
    return LossScaler(scale=static_loss_scale)
