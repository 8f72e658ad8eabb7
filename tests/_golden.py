"""Loader for the committed golden fixtures (produced by tests/golden/make_golden.py)."""
import json
import os

import numpy as np

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


class Golden:
    def __init__(self):
        with open(os.path.join(HERE, "golden.json")) as f:
            self.j = json.load(f)
        self.npz = np.load(os.path.join(HERE, "golden_inputs.npz"), allow_pickle=False)

    def explicit(self):
        """Yield (name, z, y, record) for every explicit-input case."""
        for name, rec in sorted(self.j["explicit"].items()):
            yield name, self.npz[f"{name}__z"], self.npz[f"{name}__y"], rec

    def arr(self, key):
        return self.npz[key]


def F(h: str) -> float:
    return float.fromhex(h)


def load_golden() -> Golden:
    return Golden()
