"""Progressive Layer Dropping (reference `runtime/progressive_layer_drop.py`; Zhang & He 2020): the keep
probability theta(t) = (1 - theta_bar) * exp(-gamma * t) + theta_bar decays from 1 to `theta`; the engine hands
`progressive_layer_drop=True, pld_theta=theta(t)` to the model's forward, which skips layers stochastically."""
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
