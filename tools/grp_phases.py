"""Where k_search_grp's time goes (BASELINE C2's kernel; the phase-stamp build, the A/B library `make AB=1`
with OAZ_GRP_DBG=1): per simulation, thread 0's s_memtime cycles in the backups of wave 0's four games, their
selects, the barrier after the walks (the slowest walker wave), and the evaluation with its barriers, from the
statistics slots of each workgroup's first game, averaged over the workgroups; converted to us with the loop's
cycles over the launches' HIP-event time. Experiment tool, not a test.
usage: OAZ_LIB=.../libonitama_az_ab.so OAZ_GRP_DBG=1 python tools/grp_phases.py [games] [sims] [noise 0|1]"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "onitama-alphazero_amd"))
import numpy as np  # noqa: E402

from onitama_az import _abi  # noqa: E402
from onitama_az.engine import Engine  # noqa: E402
from onitama_az.game import initial_state_np  # noqa: E402
from onitama_az.weights import random_weights  # noqa: E402

G = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
sims = int(sys.argv[2]) if len(sys.argv) > 2 else 100
noise = int(sys.argv[3]) if len(sys.argv) > 3 else 1
roots = np.concatenate([initial_state_np([0, 1, 2, 3, 4]) for _ in range(G)])
res = []
with Engine(games=G, sims=sims, blocks=3, c_puct=5.0, train_noise=noise, evaluator=_abi.EVAL_NN,
            precision=_abi.FP32_SPLIT16, step_kernels=0) as e:
    e.load_weights(random_weights(0, 3))
    e.search(roots)
    e.set_timing(1)
    nwg = (G + 15) // 16
    for _ in range(5):
        e.kernel_times_reset()
        r = e.search(roots)
        kt = e.kernel_times()
        st = e.selfplay_stats()
        loop = st.passes / nwg
        us = 1e3 * kt.backup_select_ms  # every k_search_grp launch of the search
        per = {"backup": st.games_cut, "select": st.red_wins, "walk_barrier": st.moves, "evaluation": st.blue_wins}
        res.append({"search_us": us, "cycles_per_us": loop / us,
                    "mean_depth": r.stats.depth_sum / max(1, r.stats.sims),
                    "per_sim_cycles": {k: v / nwg / sims for k, v in per.items()} | {"loop": loop / sims}})
r = res[len(res) // 2]
r["per_sim_us"] = {k: v / r["cycles_per_us"] for k, v in r["per_sim_cycles"].items()}
print(json.dumps({"games": G, "sims": sims, "noise": noise, **r}, indent=1))
