"""Workgroup timeline of k_nn_h3 (A/B build, OAZ_NN_X6_V=60: each workgroup writes its start / end on
the constant 100 MHz clock and its HW_ID / XCC_ID over its first policy row). Reports the launch span,
per-CU busy time, the gaps between consecutive workgroups on a CU, and the tail (last finish minus the
per-CU last finishes). Usage: OAZ_LIB=.../libonitama_az_ab.so python tools/nn_timeline.py [B] [blocks]"""
import json
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "onitama-alphazero_amd"))
os.environ["OAZ_NN_X6_V"] = os.environ.get("OAZ_NN_X6_V", "60")
from onitama_az import _abi  # noqa: E402
from onitama_az.engine import Engine  # noqa: E402
from onitama_az.weights import random_weights  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
blocks = int(sys.argv[2]) if len(sys.argv) > 2 else 3
g = np.load(ROOT / "tests/golden/nn_golden.npz")
states = np.concatenate([g["states"]] * (B // len(g["states"]) + 1))[:B]
runs = []
with Engine(games=B, sims=1, blocks=blocks, evaluator=_abi.EVAL_NN, precision=_abi.FP32_SPLIT16) as e:
    e.load_weights(random_weights(0, blocks))
    for r in range(4):
        p, _ = e.nn_forward(states)
        runs.append(p.reshape(B // 16, 800)[:, :6].copy().view(np.uint32))
out = {}
for r, w in enumerate(runs[1:]):
    t0 = w[:, 0].astype(np.uint64) | (w[:, 1].astype(np.uint64) << 32)
    t1 = w[:, 2].astype(np.uint64) | (w[:, 3].astype(np.uint64) << 32)
    hw, xcc = w[:, 4], w[:, 5]
    cu = (xcc & 0xF) * 4096 + ((hw >> 13) & 0x7) * 512 + ((hw >> 12) & 1) * 256 + ((hw >> 8) & 0xF)
    base = t0.min()
    s, f = (t0 - base).astype(np.float64) * 10.0, (t1 - base).astype(np.float64) * 10.0  # ns
    span = f.max()
    gaps, busy, last = [], [], []
    for c in np.unique(cu):
        i = np.where(cu == c)[0]
        o = i[np.argsort(s[i])]
        busy.append(float((f[o] - s[o]).sum()))
        gaps.extend((s[o[1:]] - f[o[:-1]]).tolist())
        last.append(float(f[o].max()))
    out[f"run{r + 1}"] = {
        "workgroups": int(len(s)), "cus": int(len(np.unique(cu))), "span_us": span / 1e3,
        "wg_us_mean": float((f - s).mean()) / 1e3, "wg_us_p5_p95": [float(np.percentile(f - s, q)) / 1e3 for q in (5, 95)],
        "wgs_per_cu": [int(x) for x in np.percentile(np.bincount(np.unique(cu, return_inverse=True)[1]), [0, 50, 100])],
        "first_start_spread_us": float(np.sort(s)[255]) / 1e3,
        "gap_us_mean": float(np.mean(gaps)) / 1e3, "gap_us_p50_p95": [float(np.percentile(gaps, q)) / 1e3 for q in (50, 95)],
        "cu_busy_frac_of_span": float(np.mean(busy)) / span,
        "tail_us (span - median CU last finish)": (span - float(np.median(last))) / 1e3,
    }
print(json.dumps(out, indent=1))
