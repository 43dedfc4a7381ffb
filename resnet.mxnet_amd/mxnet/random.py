"""mx.random: seeding of the host RNG used by the initializers."""
import numpy as np

_rng = np.random.default_rng(2)


def seed(seed_state, ctx="all"):
    global _rng
    _rng = np.random.default_rng(seed_state)


def rng():
    return _rng
