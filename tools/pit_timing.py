"""Evaluator.pit wall time: the three fights (vs best, vs Random, vs pure MCTS; evaluator.rs:169-193)
one after the other and on threads of their own, same results asserted. new = the reference's
trained 3-block network, best = a random-init 3-block network. Experiment tool.
usage: python tools/pit_timing.py [game_amnt] [sims] [max_plies]"""
import json
import os
import sys
import time

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "onitama-alphazero_amd"))
import numpy as np  # noqa: E402

from onitama_az.evaluator import Evaluator, EvaluatorConfig  # noqa: E402
from onitama_az.mcts import ConvResNet, ConvResNetConfig  # noqa: E402

games = int(sys.argv[1]) if len(sys.argv) > 1 else 20
sims = int(sys.argv[2]) if len(sys.argv) > 2 else 400
max_plies = int(sys.argv[3]) if len(sys.argv) > 3 else 150
trained = np.load(os.path.join(ROOT, "tests", "golden", "weights_3block_trained.npy"))
new = ConvResNet(ConvResNetConfig(resnet_block_amnt=3), weights=trained)
best = ConvResNet(ConvResNetConfig(resnet_block_amnt=3), seed=7)
ev = Evaluator(EvaluatorConfig(game_amnt=games, max_plies=max_plies, seed=3), best, new)
ev.pit(sims=8, concurrent=True)  # warm-up: engines, kernels, thread pool
out = {"game_amnt": games, "sims": sims, "max_plies": max_plies}
res = {}
for conc in (False, True, False, True):
    t0 = time.perf_counter()
    pit, promote = ev.pit(sims=sims, concurrent=conc)
    dt = time.perf_counter() - t0
    key = "concurrent" if conc else "sequential"
    out.setdefault(key + "_s", []).append(round(dt, 3))
    res.setdefault(key, (pit, promote))
    print(key, round(dt, 3), flush=True)
a, b = res["sequential"][0], res["concurrent"][0]
for x, y in ((a.self_fight, b.self_fight), (a.random_fight, b.random_fight), (a.mcts_fight, b.mcts_fight)):
    assert x.results == y.results and x.plies == y.plies and x.rating_a == y.rating_a
out["plies_max"] = {k: max(getattr(a, k).plies) for k in ("self_fight", "random_fight", "mcts_fight")}
out["winrate_new"] = {k: getattr(a, k).winrate for k in ("self_fight", "random_fight", "mcts_fight")}
out["speedup"] = round(min(out["sequential_s"]) / min(out["concurrent_s"]), 3)
print(json.dumps(out))
