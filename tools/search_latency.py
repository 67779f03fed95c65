"""Agent-API latency: one oaz_search (one move for each of G positions) at `sims` playouts, 3-block
fp16x3 network, train=false, for small G (the GUI / tournament / arena-tail case). Experiment tool.
OAZ_LAT_BUDGETS: comma-separated search_time budgets in ms (0 = none; default "0,400": the reference
Agent's config passes one, alphazero_mcts/mod.rs:34-43, and the engine checks it on the device).
usage: python tools/search_latency.py [sims] [reps]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "onitama-alphazero_amd"))
import numpy as np  # noqa: E402

from onitama_az import _abi  # noqa: E402
from onitama_az.engine import Engine  # noqa: E402
from onitama_az.game import initial_state_np  # noqa: E402
from onitama_az.weights import random_weights  # noqa: E402

sims = int(sys.argv[1]) if len(sys.argv) > 1 else 400
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
out = {}
Gs = [int(x) for x in os.environ.get("OAZ_LAT_G", "1,16,64,256,1024,2048").split(",")]
budgets = [float(x) for x in os.environ.get("OAZ_LAT_BUDGETS", "0,400").split(",")]
for G in Gs:
    roots = np.concatenate([initial_state_np([0, 1, 2, 3, 4]) for _ in range(G)])
    ev = _abi.EVAL_HASH if os.environ.get("OAZ_LAT_EVAL") == "hash" else _abi.EVAL_NN
    with Engine(games=G, sims=sims, blocks=3, c_puct=5.0, train_noise=0, evaluator=ev,
                precision=_abi.FP32_SPLIT16, step_kernels=int(os.environ.get("OAZ_LAT_STEP", "0"))) as e:
        e.load_weights(random_weights(0, 3))
        e.search(roots)
        for b in budgets:
            e.set_search_time(b * 1e-3)
            e.set_timing(0)
            ts, runs = [], []
            for _ in range(reps):
                t0 = time.perf_counter()
                e.search(roots)
                ts.append(time.perf_counter() - t0)
                runs.append(int(e.search_playouts(G).min()))
            e.set_timing(1)  # a separate timed search: per-launch kernel times (events add a little)
            e.kernel_times_reset()
            e.search(roots)
            kt = e.kernel_times()
            out[f"G{G}" + (f"_budget{b:g}ms" if b > 0 else "")] = {
                "ms_median": 1e3 * float(np.median(ts)), "ms_min": 1e3 * min(ts),
                "playouts_min": min(runs), "us_per_sim_step": 1e6 * float(np.median(ts)) / sims,
                "launches": int(kt.backup_select_n),
                "nn_us_per_launch": 1e3 * kt.nn_ms / max(kt.nn_n, 1),
                "backup_select_us_per_launch": 1e3 * kt.backup_select_ms / max(kt.backup_select_n, 1)}
print(json.dumps(out, indent=1))
