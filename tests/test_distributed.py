"""CPU, world_size 2 over gloo: the multi-GPU path's exchange (padded all-gather of replay
samples) and the game-id sharding contract."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from onitama_az import dist as odist


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n = 3 + 5 * rank  # ragged counts: 3 and 8 samples
    rng = np.random.default_rng(rank)
    local = torch.from_numpy(rng.integers(0, 255, n * odist.SAMPLE_BYTES, dtype=np.uint8))
    out = odist.allgather_sample_bytes(local, world)
    q.put((rank, out.numpy().tobytes(), local.numpy().tobytes()))
    # empty contribution from one rank
    empty = torch.zeros(0, dtype=torch.uint8) if rank == 0 else local
    out2 = odist.allgather_sample_bytes(empty, world)
    q.put((rank + 10, out2.numpy().tobytes(), b""))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_allgather_samples_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(4):
        k, out, loc = q.get(timeout=100)
        res[k] = (out, loc)
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    expect = res[0][1] + res[1][1]
    assert res[0][0] == expect and res[1][0] == expect
    assert len(expect) == (3 + 8) * odist.SAMPLE_BYTES
    assert res[10][0] == res[1][1] and res[11][0] == res[1][1]


def test_global_game_ids_are_a_partition():
    games, world = 16, 4
    seen = set()
    for seq in range(3):
        for rank in range(world):
            ids = set(int(i) for i in odist.global_game_ids(rank, world, games, seq))
            assert not (ids & seen)
            seen |= ids
    assert seen == set(range(3 * world * games))


def test_c4_shard_game_ids_partition_each_sequence():
    """C4 (65,536 games per GPU x 8 ranks): the product rule (oaz_slot_game_ids, the function the
    self-play kernel's start_game calls) gives the 8 ranks disjoint id sets whose union is exactly
    [seq * 8G, (seq + 1) * 8G) for every game sequence, and rank 5's ids are (seq * 8 + 5) * G + slot
    (the reference's workers, train.rs:218-238, play disjoint games)."""
    G, W = 65536, 8
    for seq in (0, 1, 7):
        ids = np.concatenate([odist.global_game_ids(r, W, G, seq) for r in range(W)])
        assert ids.dtype == np.uint64 and len(ids) == W * G
        assert np.array_equal(np.sort(ids), np.arange(seq * W * G, (seq + 1) * W * G, dtype=np.uint64))
        r5 = odist.global_game_ids(5, W, G, seq)
        assert np.array_equal(r5, (seq * W + 5) * G + np.arange(G, dtype=np.uint64))
    with pytest.raises(Exception):
        odist.global_game_ids(8, W, G, 0)  # rank outside the world
