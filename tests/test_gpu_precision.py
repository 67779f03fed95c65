"""GPU: the fp32 NN arithmetic of the benchmarked kernels on real positions and real networks, the
search-level effect of the reduced-precision modes, and the multi-rank plumbing on one GPU.

  - split16 self-play with the reference's trained 3- and 5-block networks: the fp16 range holds
    (no fallback tile) and positions drawn from those games match a torch fp32 forward to 1e-5;
  - end-to-end statistics ("end-to-end parity is statistical"): searches with the
    fp16x3 split and bf16 kernels against the oracle's own fp32 network (net.rs:215-232);
  - the C-ABI sample all-gather (RCCL communicator) at world 1, byte-equal to samples_fetch;
  - oaz_selfplay_run with a rank/world configuration ends and plays exactly its share.
"""
import sys
from pathlib import Path

import numpy as np
import pytest
import torch

from onitama_az import _abi
from onitama_az.engine import Engine
from onitama_az.weights import named_from_blob, random_weights

pytestmark = pytest.mark.gpu

ROOT = Path(__file__).resolve().parents[1]
GOLDEN = ROOT / "tests" / "golden"
SEED = 20260101


def torch_fp32_forward(blob, blocks, states):
    """net.rs forward(train=false) in fp32 torch on the CPU (oracle/train_ref.py op graph)."""
    sys.path.insert(0, str(ROOT / "oracle"))
    from train_ref import forward
    from onitama_az.game import encode_batch
    named = {k: torch.from_numpy(np.ascontiguousarray(v, dtype=np.float32)) for k, v in
             named_from_blob(blob, blocks).items()}
    with torch.no_grad():
        p, v = forward(named, torch.from_numpy(encode_batch(states)), blocks, train=False)
    return p.numpy().reshape(-1, 2, 25), v.numpy().reshape(-1)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("blocks,fixture", [(3, "weights_3block_trained.npy"), (5, "weights_5block_trained.npy")])
def test_split16_selfplay_trained_weights_range_and_goldens(blocks, fixture):
    """128 self-play slots x 32 sims x 30 plies (3,840 plies, 122,880 NN evaluations) with the
    reference's trained network (models/model_5e-3_3_resnet.ot, model_5e-3.ot) on the fp16x3 split
    kernel: no activation leaves the fp16 range (no fallback tile), and on positions drawn from
    those games the kernel's outputs are within 1e-5 of a torch fp32 forward."""
    w = np.load(GOLDEN / fixture, allow_pickle=False)
    with Engine(games=128, sims=32, blocks=blocks, c_puct=5.0, train_noise=1, max_plies=150, evaluator=_abi.EVAL_NN,
                precision=_abi.FP32_SPLIT16, fixed_deck=0, seed=SEED, sample_capacity=128 * 64) as e:
        e.load_weights(w)
        e.selfplay_reset()
        e.selfplay_step(30)
        st = e.selfplay_stats()
        smp = e.samples_fetch(int(st.samples_ready))
        assert e.nn_fallbacks() == 0
    assert st.moves >= 300 and len(smp) > 0
    states = np.ascontiguousarray(smp["state"][:512])
    with Engine(games=len(states), sims=1, blocks=blocks, evaluator=_abi.EVAL_NN, precision=_abi.FP32_SPLIT16) as e:
        e.load_weights(w)
        p, v = e.nn_forward(states)
        assert e.nn_fallbacks() == 0
    tp, tv = torch_fp32_forward(w, blocks, states)
    assert np.abs(p - tp).max() < 1e-5 and np.abs(v - tv).max() < 1e-5


@pytest.mark.timeout(300)
@pytest.mark.parametrize("precision,move_agree,pi_l1", [(_abi.FP32_SPLIT16, 0.97, 0.02), (_abi.FP32, 0.97, 0.02),
                                                        (_abi.BF16, 0.75, 0.25)])
def test_search_statistics_vs_oracle_fp32_network(orc, precision, move_agree, pi_l1):
    """128 roots x 200 sims, trained 3-block network, no noise: the GPU search on each NN kernel
    against the oracle's search on its own fp32 C network. Evaluations differ only at the kernel's
    rounding level, so trees coincide until a near-tie flips; the moves must agree on >= move_agree
    of the roots and the mean L1 distance of pi stay <= pi_l1 (fp32-level kernels: 0.97 / 0.02; the
    bf16 throughput mode: 0.75 / 0.25)."""
    from conftest import random_positions
    w = np.load(GOLDEN / "weights_3block_trained.npy", allow_pickle=False)
    roots = random_positions(orc, 128, seed=9090)
    sims = 200
    with Engine(games=128, sims=sims, blocks=3, c_puct=5.0, train_noise=0, evaluator=_abi.EVAL_NN,
                precision=precision) as e:
        e.load_weights(w)
        r = e.search(roots)
    cfg = orc.search_cfg(sims=sims, c_puct=5.0, evaluator=orc.EVAL_NN, weights=w, blocks=3)
    mv, pi, _ = orc.search_batch(cfg, roots)
    agree = float(np.mean([r.moves[i].tobytes() == mv[i].tobytes() for i in range(len(roots))]))
    l1 = float(np.abs(r.pi.reshape(-1, 50) - pi.reshape(-1, 50)).sum(1).mean())
    print(f"precision {precision}: move agreement {agree:.3f}, mean pi L1 {l1:.4f}")
    assert agree >= move_agree and l1 <= pi_l1, (agree, l1)


@pytest.mark.timeout(300)
def test_default_precision_search_equals_exact_fp32_on_clear_moves(orc):
    """The default config's network arithmetic is the fp16x3 split (oaz_config_default, Options), not the
    exact-fp32 MFMA kernel a caller gets with OAZ_FP32 (the ABI-4 behaviour change). Pinned:
    256 roots x 200 simulations with the reference's trained 3-block network, no noise, one search with the
    default config and one with OAZ_FP32: wherever the exact-fp32 search's most visited child leads the
    runner-up by more than 2 % of the simulations, the default's move is the same; over all roots the
    moves agree on >= 97 % and pi differs by <= 0.02 in mean L1 (near-ties may flip: both are fp32-level)."""
    from conftest import random_positions
    w = np.load(GOLDEN / "weights_3block_trained.npy", allow_pickle=False)
    roots = random_positions(orc, 256, seed=4711)
    sims = 200
    cfg = _abi.default_config()
    assert cfg.precision == _abi.FP32_SPLIT16
    out = {}
    for name, prec in (("default", None), ("fp32", _abi.FP32)):
        kw = dict(games=256, sims=sims, blocks=3, c_puct=5.0, train_noise=0, evaluator=_abi.EVAL_NN)
        if prec is not None:
            kw["precision"] = prec
        with Engine(**kw) as e:
            e.load_weights(w)
            out[name] = e.search(roots)
    d, f = out["default"], out["fp32"]
    pf = f.pi.reshape(-1, 50)
    top2 = np.sort(pf, axis=1)[:, -2:]
    clear = (top2[:, 1] - top2[:, 0]) > 0.02
    same = np.array([d.moves[i].tobytes() == f.moves[i].tobytes() for i in range(len(roots))])
    assert clear.sum() >= 128 and same[clear].all(), (int(clear.sum()), int((~same[clear]).sum()))
    assert same.mean() >= 0.97 and np.abs(d.pi.reshape(-1, 50) - pf).sum(1).mean() <= 0.02


@pytest.mark.timeout(120)
def test_allgather_samples_c_abi_world1_equals_fetch():
    """oaz_allgather_samples at world 1 (RCCL communicator over one GPU): the gathered records are
    byte-equal to what samples_fetch returns from a twin engine (as sets: games finishing in the same
    ply append their samples in atomic order), and the engine's buffer is drained."""
    from onitama_az.dist import Comm, as_samples
    kw = dict(games=64, sims=16, c_puct=5.0, train_noise=1, evaluator=_abi.EVAL_HASH, blocks=0, max_plies=150,
              seed=77, fixed_deck=0)
    with Engine(**kw) as a, Engine(**kw) as b:
        for e in (a, b):
            e.selfplay_reset()
            e.selfplay_step(40)
        n = int(a.selfplay_stats().samples_ready)
        assert n > 0
        comm = Comm(0, 1, 0)
        out = torch.empty(n * 228, dtype=torch.uint8, device="cuda")
        total, counts = comm.allgather_samples(a, out)
        comm.close()
        assert total == n and counts == [n]
        ref = b.samples_fetch(n)
        key = lambda a: np.sort(np.frombuffer(a.tobytes(), dtype=np.dtype((np.void, 228))))
        assert np.array_equal(key(as_samples(out)), key(ref))
        assert a.selfplay_stats().samples_ready == 0


@pytest.mark.timeout(120)
def test_selfplay_run_rank_share_terminates(orc):
    """oaz_selfplay_run(n_games) with world 2 on one GPU (two engines, rank 0 and 1): each rank plays
    the global game ids below n_games that it owns ((k * world + rank) * games + slot) and returns;
    together they play every id once, and each game's samples equal the oracle's game."""
    G, n_games, sims = 4, 10, 8
    got = {}
    for rank in (0, 1):
        with Engine(games=G, sims=sims, c_puct=5.0, train_noise=0, evaluator=_abi.EVAL_HASH, blocks=0, max_plies=150,
                    seed=4242, fixed_deck=0, rank=rank, world=2) as e:
            smp, st = e.selfplay_run(n_games, cap=n_games * 152)
            got[rank] = (smp, st)
    assert got[0][1].games_finished == 6 and got[1][1].games_finished == 4  # ids 0-3, 8, 9 | 4-7
    ref = []
    for gid in range(n_games):
        cfg = orc.search_cfg(sims=sims, c_puct=5.0, evaluator=orc.EVAL_HASH, seed=4242)
        s, _, _, _ = orc.selfplay_game(cfg, gid, max_plies=150, deck=None)
        ref.append(s)
    ref = np.concatenate(ref)
    both = np.concatenate([got[0][0], got[1][0]])
    key = lambda a: np.sort(np.frombuffer(a.tobytes(), dtype=np.dtype((np.void, 228))))
    assert len(both) == len(ref) and np.array_equal(key(both), key(ref))
