"""Batch-size warm-up schedule (reference parity: deepspeed/runtime/bs_schedules.py:5-71).

The batch grows from ceil(min_batch_size_multiplier * final_batch_size) to final_batch_size
in `num_intervals` evenly spaced steps over `warmup_num_steps` iterations and stays there.
Consecutive intervals that truncate to the same size are merged.  Like the reference, this is
a standalone helper: the client (e.g. a GPT-NeoX training loop) reads `current_batch_size`
after `step()` and slices its batches accordingly; the engine does not consume it.
"""

from __future__ import annotations

import bisect
import math

import numpy as np


class BatchSizeScheduler:
    def __init__(self, final_batch_size: int, min_batch_size_multiplier: float = 0.01,
                 warmup_num_steps: int = 1000, num_intervals: int = 4, last_batch_iteration: int = -1,
                 deepspeed=None):
        self.final_batch_size = int(final_batch_size)
        self.min_batch_size_multiplier = float(min_batch_size_multiplier)
        self.warmup_num_steps = int(warmup_num_steps)
        self.num_intervals = int(num_intervals)
        self.last_batch_iteration = int(last_batch_iteration)
        self.deepspeed = deepspeed
        self.schedule = self._build_schedule()
        self._keys = sorted(self.schedule)
        self.current_batch_size = None

    def _build_schedule(self):
        start = math.ceil(self.min_batch_size_multiplier * self.final_batch_size)
        # integer-truncated linear ramps of sizes and of the steps they start at
        sizes = np.linspace(start, self.final_batch_size, num=self.num_intervals, dtype=int)
        steps = np.linspace(0, self.warmup_num_steps, num=self.num_intervals, dtype=int)
        out, prev = {}, None
        for st, bs in zip(steps.tolist(), sizes.tolist()):
            if bs != prev:
                out[st] = bs
            prev = bs
        return out

    def get_current_batch_size(self) -> int:
        """Size of the last interval whose start step is <= the current iteration (the first
        interval before training starts)."""
        i = bisect.bisect_right(self._keys, self.last_batch_iteration) - 1
        return self.schedule[self._keys[max(i, 0)]]

    def step(self, last_batch_iteration=None):
        if last_batch_iteration is None:
            last_batch_iteration = self.last_batch_iteration + 1
        self.last_batch_iteration = int(last_batch_iteration)
        self.current_batch_size = self.get_current_batch_size()

    def state_dict(self):
        return {"last_batch_iteration": self.last_batch_iteration}

    def load_state_dict(self, sd):
        self.last_batch_iteration = sd["last_batch_iteration"]
