"""NN kernel driver for rocprofv3 PMC passes: `launches` forwards of one precision at one batch.
Usage: rocprofv3 --pmc ... -- python tools/nn_prof.py [--precision fp32x6] [--batch 65536] [--blocks 3]"""
import argparse
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "onitama-alphazero_amd"))
from onitama_az import _abi  # noqa: E402
from onitama_az.engine import Engine  # noqa: E402
from onitama_az.weights import random_weights  # noqa: E402

PREC = {"fp32": _abi.FP32, "bf16": _abi.BF16, "fp32x6": _abi.FP32_SPLIT, "fp32h3": _abi.FP32_SPLIT16}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--precision", default="fp32h3", choices=sorted(PREC))
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--blocks", type=int, default=3)
    ap.add_argument("--launches", type=int, default=3)
    a = ap.parse_args()
    g = np.load(ROOT / "tests/golden/nn_golden.npz")
    states = np.concatenate([g["states"]] * (a.batch // len(g["states"]) + 1))[: a.batch]
    with Engine(games=a.batch, sims=1, blocks=a.blocks, evaluator=_abi.EVAL_NN, precision=PREC[a.precision]) as e:
        e.load_weights(random_weights(0, a.blocks))
        for _ in range(a.launches):
            e.nn_forward(states)


if __name__ == "__main__":
    main()
