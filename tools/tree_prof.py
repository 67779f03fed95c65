"""Driver for rocprofv3 passes over the fused tree kernel: single-stream (parts = 1) C3 self-play,
2 unprofiled warm-up plies then 1 ply (select with --kernel-iteration-range in the profiler).
Experiment tool, not a test. usage: python tools/tree_prof.py [games] [sims] [plies]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "onitama-alphazero_amd"))
from onitama_az import _abi  # noqa: E402
from onitama_az.engine import Engine  # noqa: E402
from onitama_az.weights import random_weights  # noqa: E402

games = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
sims = int(sys.argv[2]) if len(sys.argv) > 2 else 400
plies = int(sys.argv[3]) if len(sys.argv) > 3 else 3
with Engine(device=0, games=games, sims=sims, blocks=3, c_puct=5.0, train_noise=1, max_plies=150,
            evaluator=_abi.EVAL_NN, precision=_abi.FP32_SPLIT16, fixed_deck=1, deck=[0, 1, 2, 3, 4],
            seed=20260101, sample_capacity=games * (plies + 2), parts=1, compact=0) as e:
    e.load_weights(random_weights(0, 3))
    e.selfplay_reset()
    for _ in range(plies):
        e.selfplay_step(1)
    e.sync()
print("ok")
