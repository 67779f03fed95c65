"""NN kernel microbench: parity vs the torch goldens and per-launch time at a given batch, over
interleaved rounds of one or more engines (block counts). Usage: python tools/nn_ab.py [--batch 65536] [--blocks 3,6]"""
import argparse
import json
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "onitama-alphazero_amd"))
from onitama_az import _abi  # noqa: E402
from onitama_az.engine import Engine  # noqa: E402
from onitama_az.weights import random_weights  # noqa: E402

FLOP = {3: 11_681_928, 5: 19_054_728, 6: 22_741_128}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--blocks", default="3")
    ap.add_argument("--precision", default="fp32,fp32x6,bf16")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--x6-variants", default="0", help="OAZ_NN_X6_V values to compare for fp32x6 / fp32h3")
    a = ap.parse_args()
    g = np.load(ROOT / "tests/golden/nn_golden.npz")
    w3 = np.load(ROOT / "tests/golden/weights_3block_trained.npy")
    engines = {}
    for v in [int(x) for x in a.blocks.split(",")]:
        for prec, var in [(p, x) for p in a.precision.split(",")
                          for x in (a.x6_variants.split(",") if p in ("fp32x6", "fp32h3") else ["0"])]:
            os.environ["OAZ_NN_X6_V"] = var
            e = Engine(games=a.batch, sims=1, blocks=v, evaluator=_abi.EVAL_NN,
                       precision={"bf16": _abi.BF16, "fp32x6": _abi.FP32_SPLIT,
                                  "fp32h3": _abi.FP32_SPLIT16}.get(prec, _abi.FP32))
            err = {}
            for name, blob, nb in (("trained3", w3, 3), ("random3", random_weights(0, 3), 3),
                                   ("random6", random_weights(1, 6), 6)):
                if nb != v:
                    continue
                e.load_weights(blob)
                p, val = e.nn_forward(g["states"])
                err[name] = {"policy": float(np.abs(p - g[f"policy_{name}"]).max()),
                             "value": float(np.abs(val - g[f"value_{name}"]).max())}
            e.load_weights(random_weights(0, v))
            engines[f"{v}-{prec}" + (f"-v{var}" if prec in ("fp32x6", "fp32h3") else "")] = (e, err, v, var)
    states = np.concatenate([g["states"]] * (a.batch // len(g["states"]) + 1))[: a.batch]
    res = {v: [] for v in engines}
    for _ in range(a.rounds):
        for v, (e, _, _, var) in engines.items():
            os.environ["OAZ_NN_X6_V"] = var
            e.nn_forward(states[:1024])
            e.kernel_times_reset()
            e.set_timing(True)
            for _ in range(a.reps):
                e.nn_forward(states)
            e.set_timing(False)
            t = e.kernel_times()
            res[v].append(t.nn_ms / t.nn_n)
    out = {}
    for v, ts in res.items():
        ms = float(np.median(ts))
        nb = engines[v][2]
        out[v] = {"median_ms": ms, "min_ms": float(min(ts)), "tflops": FLOP[nb] * a.batch / ms / 1e9,
                  "sims_per_s": a.batch / ms * 1e3, "max_err_vs_torch": engines[v][1]}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
