"""Progressive Layer Drop (parity: reference runtime/progressive_layer_drop.py:10).

Keep-probability schedule theta(t) = (1 - theta_bar) * exp(-gamma * t) + theta_bar; the engine
passes ``progressive_layer_drop=True, pld_theta=theta(t)`` to the model's forward, and models apply
layer i with probability 1 - i / L * (1 - theta) during training.
"""
import math


class ProgressiveLayerDrop:
    def __init__(self, theta=0.5, gamma=0.001):
        self.theta = theta
        self.gamma = gamma
        self.current_theta = 1.0

    def get_state(self):
        return {"progressive_layer_drop": True, "pld_theta": self.get_theta()}

    def get_theta(self):
        return self.current_theta

    def update_state(self, global_step):
        self.current_theta = (1.0 - self.theta) * math.exp(-self.gamma * global_step) + self.theta


def layer_keep_prob(layer_idx, num_layers, theta):
    """Stochastic-depth keep probability of layer ``layer_idx`` (0-based) under PLD."""
    return 1.0 - (layer_idx + 1) / num_layers * (1.0 - theta)
