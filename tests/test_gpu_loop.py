"""GPU: the AlphaZero loop (alphazero-training/src/train.rs:158-412) over several ranks. Two ranks
share GPU 0 with gloo collectives (a one-GPU rehearsal of the torchrun layout; RCCL needs one GPU
per rank): sharded self-play, the sample all-gather, data-parallel epochs (gradient all-reduce, BN
statistics averaged), rank 0's pit broadcast. Every rank must end every iteration with identical
weights and take identical promotion decisions."""
import hashlib
import os
import socket

import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, folder, q):
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parents[1]
    sys.path.insert(0, str(root / "onitama-alphazero_amd"))
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from onitama_az.evaluator import EvaluatorConfig
    from onitama_az.mcts import AlphaZeroMctsConfig, ConvResNetConfig
    from onitama_az.train_loop import LoopConfig, train
    cfg = LoopConfig(iterations=2, training_epochs=2, train_batch_size=32, self_play_game_amnt=12,
                     evaluation_checkpoint=2, save_checkpoint=2,
                     model_config=ConvResNetConfig(resnet_block_amnt=2),
                     mcts_config=AlphaZeroMctsConfig(exploration_c=5.0, max_playouts=16, train=True),
                     evaluator_config=EvaluatorConfig(game_amnt=4), learning_rate=1e-2)
    seen = []

    def on_it(it, new, best):
        seen.append((it, hashlib.sha256(new.tobytes()).hexdigest(), hashlib.sha256(best.tobytes()).hexdigest()))

    stats = train(cfg, folder=folder, eval_sims=16, rank=rank, world=world, on_iteration=on_it)
    q.put((rank, seen, stats.was_best_change, [round(x, 6) for x in stats.loss],
           [g["positions_retrieved"] for g in stats.games_played]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_loop_two_ranks_identical_weights_and_decisions(tmp_path):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, 2, port, str(tmp_path), q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((r[0], r[1:]) for r in (q.get(timeout=280) for _ in range(2)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0] == res[1]  # weights hashes per iteration, promotions, losses, buffer sizes
    seen, promos, losses, buffers = res[0]
    assert [s[0] for s in seen] == [1, 2] and len(promos) == 1 and all(b > 0 for b in buffers)
    assert seen[0][1] != seen[1][1]  # training moved the weights
    assert (tmp_path / "stats.json").exists()
