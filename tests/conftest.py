"""pytest config: `gpu` marker + shared fixtures (oracle = test infrastructure only)."""
import gzip
import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
sys.path.insert(0, os.path.join(ROOT, "gym-chess_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")


def load_golden(name):
    path = os.path.join(GOLDEN, name)
    if name.endswith(".gz"):
        with gzip.open(path, "rb") as f:
            return json.loads(f.read())
    with open(path) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def oracle():
    import oracle as O

    O.lib()
    return O


@pytest.fixture(scope="session")
def engine():
    from gym_chess_amd.engine import Engine

    return Engine(0)


def random_positions(n, seed, weird=True):
    """Seeded random positions: sparse random piece placement; with `weird`, also boards the
    reference accepts but real chess never has (several / no kings, pawns on the back rank,
    rights set without rooks)."""
    rng = np.random.RandomState(seed)
    boards = np.zeros((n, 64), dtype=np.int8)
    metas = np.zeros((n, 8), dtype=np.uint8)
    for i in range(n):
        k = rng.randint(2, 26)
        sq = rng.choice(64, size=k, replace=False)
        ids = rng.choice([2, 3, 4, 5, 6, 6, 6, -2, -3, -4, -5, -6, -6, -6], size=k)
        b = np.zeros(64, dtype=np.int8)
        b[sq] = ids
        mode = rng.randint(10) if weird else 0
        free = [s for s in range(64) if b[s] == 0]
        if mode != 1 and free:  # white king unless mode 1
            b[free.pop(rng.randint(len(free)))] = 1
        if mode != 2 and free:
            b[free.pop(rng.randint(len(free)))] = -1
        if mode == 3 and free:  # an extra king
            b[free.pop(rng.randint(len(free)))] = rng.choice([1, -1])
        if mode in (4, 5):  # castling geometry: kings/rooks on home squares (positive ids at the top too)
            for s, v in ((60, 1), (56, 3), (63, 3), (4, 1 if mode == 5 else -1), (0, 3 if mode == 5 else -3),
                         (7, 3 if mode == 5 else -3)):
                b[b == v] = 0 if v in (1, -1) else b[b == v]
                b[s] = v
            for s in (57, 58, 59, 61, 62, 1, 2, 3, 5, 6):
                if rng.rand() < 0.7:
                    b[s] = 0
        boards[i] = b
        metas[i, 0] = rng.randint(2)
        metas[i, 1:5] = rng.randint(2, size=4)
    return boards, metas
