"""NN kernel driver for rocprofv3 passes: nn_forward at a given batch, a few launches.
Usage: python tools/nn_prof.py [B] [blocks] [fp32h3|fp32x6|bf16|fp32] [reps]  (OAZ_NN_X6_V selects a variant
in the A/B build, OAZ_LIB=.../libonitama_az_ab.so)."""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "onitama-alphazero_amd"))
from onitama_az import _abi  # noqa: E402
from onitama_az.engine import Engine  # noqa: E402
from onitama_az.weights import random_weights  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
blocks = int(sys.argv[2]) if len(sys.argv) > 2 else 3
prec = {"fp32h3": _abi.FP32_SPLIT16, "fp32x6": _abi.FP32_SPLIT, "bf16": _abi.BF16, "fp32": _abi.FP32}[
    sys.argv[3] if len(sys.argv) > 3 else "fp32h3"]
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 5
g = np.load(ROOT / "tests/golden/nn_golden.npz")
states = np.concatenate([g["states"]] * (B // len(g["states"]) + 1))[:B]
with Engine(games=B, sims=1, blocks=blocks, evaluator=_abi.EVAL_NN, precision=prec) as e:
    e.load_weights(random_weights(0, blocks))
    for _ in range(reps):
        e.nn_forward(states)
print("ok")
