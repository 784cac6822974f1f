"""Learning-rate persistence and schedules.

``LearningRate`` keeps the reference's JSON persistence API
(``distribute_learningrate.py:12-50``: ``{"learning_rate": x}`` at
``save_path``, loaded at construction, ``update == save``) and is also
callable so it can be passed directly as an optimizer learning rate.
Schedules are host-side callables ``f(global_step) -> float``.
"""
import json
import math
import os

from . import log as logger


class LearningRate(object):
    def __init__(self, initial_learning_rate, save_path, decay_factor=None):
        self.path = save_path
        self.decay_factor = decay_factor
        self.learning_rate = initial_learning_rate
        if save_path and os.path.exists(save_path):
            self.learning_rate = self.load()

    def save(self, current_learning_rate):
        if not os.path.exists(self.path):
            logger.info("Create Json file for learning rate.")
        try:
            tmp = self.path + ".tmp"
            with open(tmp, "w") as f:
                json.dump({'learning_rate': current_learning_rate}, f)
            os.replace(tmp, self.path)
        except IOError as err:
            raise RuntimeError("[Error]: Error happens when read/write %s: %s" % (self.path, err))
        self.learning_rate = current_learning_rate
        return current_learning_rate

    def load(self):
        if not os.path.exists(self.path):
            return self.learning_rate
        try:
            with open(self.path) as f:
                return json.load(f)["learning_rate"]
        except (IOError, ValueError, KeyError) as err:
            raise RuntimeError("[Error]: Error happens when read/write %s: %s" % (self.path, err))

    def update(self, current_learning_rate):
        return self.save(current_learning_rate)

    def decay(self):
        if self.decay_factor is not None:
            return self.update(self.learning_rate * self.decay_factor)
        return self.learning_rate

    def __call__(self, global_step=0):
        return self.learning_rate


def piecewise_constant(boundaries, values):
    def f(step):
        for b, v in zip(boundaries, values):
            if step < b:
                return v
        return values[-1]
    return f


def exponential_decay(learning_rate, decay_steps, decay_rate, staircase=False):
    def f(step):
        p = step / float(decay_steps)
        if staircase:
            p = math.floor(p)
        return learning_rate * decay_rate ** p
    return f


def warmup_linear_decay(peak, warmup_steps, total_steps, end=0.0):
    def f(step):
        if step < warmup_steps:
            return peak * (step + 1) / float(max(warmup_steps, 1))
        frac = min((step - warmup_steps) / float(max(total_steps - warmup_steps, 1)), 1.0)
        return end + (peak - end) * (1.0 - frac)
    return f


def cosine_decay(learning_rate, decay_steps, alpha=0.0, warmup_steps=0):
    def f(step):
        if step < warmup_steps:
            return learning_rate * (step + 1) / float(warmup_steps)
        s = min(step - warmup_steps, decay_steps)
        cos = 0.5 * (1 + math.cos(math.pi * s / decay_steps))
        return learning_rate * ((1 - alpha) * cos + alpha)
    return f
