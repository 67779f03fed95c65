"""Per-wave phase breakdown of k_nn_h3 from its phase-stamp build (the A/B library, `make AB=1`,
OAZ_NN_X6_V=36): s_memtime sums per phase, written over each workgroup's first policy rows.
Output: mean cycles per wave per phase.
Usage: OAZ_LIB=.../libonitama_az_ab.so python tools/nn_phases.py [B] [blocks] h3"""
import json
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "onitama-alphazero_amd"))
os.environ["OAZ_NN_X6_V"] = os.environ.get("OAZ_NN_X6_V", "36")  # (A/B build: OAZ_LIB)
from onitama_az import _abi  # noqa: E402
from onitama_az.engine import Engine  # noqa: E402
from onitama_az.weights import random_weights  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
blocks = int(sys.argv[2]) if len(sys.argv) > 2 else 3
g = np.load(ROOT / "tests/golden/nn_golden.npz")
states = np.concatenate([g["states"]] * (B // len(g["states"]) + 1))[:B]
prec = _abi.FP32_SPLIT16 if (sys.argv[3] if len(sys.argv) > 3 else "x6") == "h3" else _abi.FP32_SPLIT
with Engine(games=B, sims=1, blocks=blocks, evaluator=_abi.EVAL_NN, precision=prec) as e:
    e.load_weights(random_weights(0, blocks))
    e.nn_forward(states)
    p, _ = e.nn_forward(states)
h3 = (sys.argv[3] if len(sys.argv) > 3 else "x6") == "h3"
nph = 8 if h3 else 6  # k_nn_h3 also stamps the kernel start and the first-layer MFMAs
flat = p.reshape(B // 16, 800)[:, :8 * nph].reshape(-1, 8, nph).astype(np.float64)
names = ["first_layer", "conv", "barrier1", "epilogue", "barrier2", "heads", "start", "first_layer_mfma"][:nph]
mean = flat.mean(axis=0)  # [wave][phase]
out = {"per_wave_mean_cycles": {f"w{w}": dict(zip(names, mean[w].round(0).tolist())) for w in range(8)},
       "all_waves": dict(zip(names, mean.mean(0).round(0).tolist())),
       "per_conv": {k: float(v) / (2 * blocks) for k, v in zip(names, mean.mean(0)) if k in ("conv", "barrier1", "epilogue", "barrier2")}}
print(json.dumps(out, indent=1))
