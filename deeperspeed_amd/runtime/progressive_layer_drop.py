"""Progressive Layer Dropping (reference parity: deepspeed/runtime/progressive_layer_drop.py:1-33).

theta(t) = (1 - theta_bar) * exp(-gamma * t) + theta_bar: the keep probability of
transformer layers decays from 1 towards `theta` over training; the engine injects
`progressive_layer_drop=True, pld_theta=theta(t)` into the model's forward kwargs.
"""

import math

from ..utils.logging import log_dist


class ProgressiveLayerDrop:
    def __init__(self, theta=0.5, gamma=0.001):
        self.theta = theta
        self.gamma = gamma
        self.current_theta = 1.0
        log_dist(f"Enabled progressive layer dropping (theta = {self.theta})", ranks=[0])

    def get_state(self):
        return {"progressive_layer_drop": True, "pld_theta": self.get_theta()}

    def get_theta(self):
        return self.current_theta

    def update_state(self, global_step):
        self.current_theta = (1.0 - self.theta) * math.exp(-self.gamma * global_step) + self.theta
