"""Where the one-launch search's time goes (k_search_lat's phase-stamp build, the A/B library `make AB=1`
with OAZ_LAT_DBG=1): the walker's s_memtime cycles per simulation in the expand / back up, the select, and
the wait for the evaluation (barriers + network or HASH), from the game's statistics slots; converted to us
with the loop's cycles over the launch's HIP-event time. Experiment tool, not a test.
usage: OAZ_LIB=.../libonitama_az_ab.so OAZ_LAT_DBG=1 python tools/lat_phases.py [sims] [G] [hash|nn]"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "onitama-alphazero_amd"))
import numpy as np  # noqa: E402

from onitama_az import _abi  # noqa: E402
from onitama_az.engine import Engine  # noqa: E402
from onitama_az.game import initial_state_np  # noqa: E402
from onitama_az.weights import random_weights  # noqa: E402

sims = int(sys.argv[1]) if len(sys.argv) > 1 else 400
G = int(sys.argv[2]) if len(sys.argv) > 2 else 1
ev = _abi.EVAL_HASH if (sys.argv[3] if len(sys.argv) > 3 else "nn") == "hash" else _abi.EVAL_NN
roots = np.concatenate([initial_state_np([0, 1, 2, 3, 4]) for _ in range(G)])
res = []
with Engine(games=G, sims=sims, blocks=3, c_puct=5.0, train_noise=0, evaluator=ev, precision=_abi.FP32_SPLIT16,
            step_kernels=0) as e:
    e.load_weights(random_weights(0, 3))
    e.search(roots)
    e.set_timing(1)
    for _ in range(5):
        e.kernel_times_reset()
        r = e.search(roots)
        kt = e.kernel_times()
        st = e.selfplay_stats()
        walk = {"mean_depth": r.stats.depth_sum / max(1, r.stats.sims), "nodes": int(r.stats.max_nodes),
                "expansions_per_sim": r.stats.expansions / max(1, r.stats.sims)}
        loop = st.passes / G
        us = 1e3 * kt.backup_select_ms / max(kt.backup_select_n, 1)
        res.append({"launch_us": us, "cycles_per_us": loop / us, "walk": walk,
                    "per_sim_cycles": {"backup": st.games_cut / G / sims, "select": st.red_wins / G / sims,
                                       "evaluation": st.blue_wins / G / sims, "loop": loop / sims,
                                       "probe_call": st.samples_dropped / G / sims,
                                       "walk_prologue": st.moves / G / sims,
                                       "walk_loads_keys": st.games_finished / G / sims}})
r = res[len(res) // 2]
r["per_sim_us"] = {k: v / r["cycles_per_us"] for k, v in r["per_sim_cycles"].items()}
print(json.dumps({"sims": sims, "G": G, "evaluator": "hash" if ev == _abi.EVAL_HASH else "nn", **r}, indent=1))
