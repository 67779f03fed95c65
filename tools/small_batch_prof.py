"""Small-batch kernels under a profiler: one 400-playout oaz_search for G positions (the Agent API's
generate_move for G = 1; an arena's tail) and 200 batch-G oaz_nn_forward calls, 3-block fp16x3
network. Run it under `rocprofv3 --kernel-trace --stats` to read k_nn_h3s / k_backup_select_seg
durations without event overhead. Experiment tool.
usage: python tools/small_batch_prof.py [G] [sims]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "onitama-alphazero_amd"))
import numpy as np  # noqa: E402

from onitama_az import _abi  # noqa: E402
from onitama_az.engine import Engine  # noqa: E402
from onitama_az.game import initial_state_np  # noqa: E402
from onitama_az.weights import random_weights  # noqa: E402

G = int(sys.argv[1]) if len(sys.argv) > 1 else 1
sims = int(sys.argv[2]) if len(sys.argv) > 2 else 400
roots = np.concatenate([initial_state_np([0, 1, 2, 3, 4]) for _ in range(G)])
with Engine(games=G, sims=sims, blocks=3, c_puct=5.0, train_noise=0, evaluator=_abi.EVAL_NN,
            precision=_abi.FP32_SPLIT16) as e:
    e.load_weights(random_weights(0, 3))
    for _ in range(3):
        e.search(roots)
    for _ in range(200):
        e.nn_forward(roots)
print("done", G, sims)
