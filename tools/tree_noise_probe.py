"""Single-stream (oaz_config.parts = 1) C3 probe of the fused tree kernel with and without root
noise: per-simulation-step time of k_backup_select_seg, of k_root_noise and of the whole step.
Compares library builds (OAZ_LIB) that differ only in the noise chunk (OAZ_NOISE_CHUNK): with the
whole ply's noise drawn before the first select, no noise launch shares the CUs with the tree
kernel, which separates the fold's own cost from that contention. Experiment tool, not a test.

usage: OAZ_LIB=... [OAZ_PROBE_NOISE=1,0] python tools/tree_noise_probe.py [games] [sims]
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "onitama-alphazero_amd"))
import torch  # noqa: E402

from onitama_az import _abi  # noqa: E402
from onitama_az.engine import Engine  # noqa: E402
from onitama_az.weights import random_weights  # noqa: E402


def probe(games, sims, noise):
    with Engine(device=0, games=games, sims=sims, blocks=3, c_puct=5.0, train_noise=noise, max_plies=150,
                evaluator=_abi.EVAL_NN, precision=_abi.FP32_SPLIT16, fixed_deck=1, deck=[0, 1, 2, 3, 4],
                seed=20260101, sample_capacity=games * 8, parts=1, compact=0) as e:
        e.load_weights(random_weights(0, 3))
        e.selfplay_reset()
        e.selfplay_step(2)
        e.sync()
        e.kernel_times_reset()
        e.set_timing(8)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e.selfplay_step(2)
        e.sync()
        dt = time.perf_counter() - t0
        e.set_timing(False)
        kt = e.kernel_times()
    return {"noise": noise, "ms_per_ply": 1e3 * dt / 2,
            "backup_select_us": 1e3 * kt.backup_select_ms / max(1, kt.backup_select_n),
            "nn_us": 1e3 * kt.nn_ms / max(1, kt.nn_n),
            "noise_ms_per_ply": kt.noise_ms / 2}


if __name__ == "__main__":
    G = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    S = int(sys.argv[2]) if len(sys.argv) > 2 else 400
    lib = os.path.basename(os.environ.get("OAZ_LIB", "libonitama_az.so"))
    # OAZ_PROBE_NOISE: "1,0" (default), or one of them (a build that is only valid without root noise)
    for nz in [int(x) for x in os.environ.get("OAZ_PROBE_NOISE", "1,0").split(",")]:
        print(json.dumps({"lib": lib, **probe(G, S, nz)}), flush=True)
