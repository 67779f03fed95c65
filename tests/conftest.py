import json
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "onitama-alphazero_amd"))
sys.path.insert(0, str(ROOT / "tests"))

GOLDEN = ROOT / "tests" / "golden"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; runs the HIP path through the C ABI")


@pytest.fixture(scope="session")
def kats():
    return json.loads((GOLDEN / "reference_kats.json").read_text())


@pytest.fixture(scope="session")
def nn_golden():
    g = np.load(GOLDEN / "nn_golden.npz", allow_pickle=False)
    return {k: g[k] for k in g.files}


@pytest.fixture(scope="session")
def trained3():
    return np.load(GOLDEN / "weights_3block_trained.npy", allow_pickle=False)


@pytest.fixture(scope="session")
def lib():
    from onitama_az import _abi
    return _abi.load()


@pytest.fixture(scope="session")
def orc():
    import oracle_ffi
    oracle_ffi.load()
    return oracle_ffi


def kat_state(d, color):
    from onitama_az import _abi
    a = np.zeros(1, dtype=_abi.STATE_DTYPE)
    a["kings"][0], a["pawns"][0], a["cards"][0], a["to_move"][0] = d["kings"], d["pawns"], d["deck"], color
    return a


def random_positions(orc, n, seed, max_plies=40, deal_seed=None):
    """Seeded positions from random play with the oracle's rules (both colours, all phases)."""
    import random
    rng = random.Random(seed)
    out, game = [], 0
    while len(out) < n:
        s = orc.initial_state(orc.deal_deck(deal_seed if deal_seed is not None else seed, game))
        game += 1
        for _ in range(rng.randint(0, max_plies)):
            moves = orc.movegen(s)
            if len(moves) == 0:
                break
            m = moves[rng.randrange(len(moves))]
            r = orc.make_move(s, tuple(int(m[k]) for k in ("from_", "to", "piece", "slot")), int(s["to_move"][0]))
            s["to_move"][0] ^= 1
            if r in (1, 2):
                break
        out.append(s.copy())
    return np.concatenate(out)
