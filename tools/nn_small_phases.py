"""Per-wave phase breakdown of k_nn_h3s (one position per workgroup) from its phase-stamp build (the
A/B library, `make AB=1`, OAZ_NN_X6_V=70): s_memtime sums per phase written over each position's
policy row, plus the clock (s_memtime cycles per wall second of a timed loop) to convert.
Usage: OAZ_LIB=.../libonitama_az_ab.so python tools/nn_small_phases.py [B] [blocks]"""
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "onitama-alphazero_amd"))
os.environ["OAZ_NN_X6_V"] = os.environ.get("OAZ_NN_X6_V", "70")
from onitama_az import _abi  # noqa: E402
from onitama_az.engine import Engine  # noqa: E402
from onitama_az.weights import random_weights  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1
blocks = int(sys.argv[2]) if len(sys.argv) > 2 else 3
g = np.load(ROOT / "tests/golden/nn_golden.npz")
states = np.ascontiguousarray(np.concatenate([g["states"]] * (B // 256 + 1))[:B])
with Engine(games=max(B, 1), sims=1, blocks=blocks, evaluator=_abi.EVAL_NN, precision=_abi.FP32_SPLIT16) as e:
    e.load_weights(random_weights(0, blocks))
    for _ in range(50):
        e.nn_forward(states)
    acc = []
    for _ in range(200):
        p, _ = e.nn_forward(states)
        acc.append(p.reshape(B, 50)[:, :48].reshape(B, 8, 6))
flat = np.concatenate(acc).astype(np.float64)
names = ["start", "first_layer", "conv_mfma", "conv_epilogue_barrier", "heads_conv", "heads_mlp"]
mean = flat.mean(axis=0)
out = {"per_wave_mean_cycles": {f"w{w}": dict(zip(names, mean[w].round(0).tolist())) for w in range(8)},
       "all_waves": dict(zip(names, mean.mean(0).round(0).tolist())),
       "total_cycles_wave0": float(mean[0].sum()),
       "per_conv_mfma_cycles": float(mean.mean(0)[2]) / (2 * blocks)}
print(json.dumps(out, indent=1))
