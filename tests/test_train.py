"""Training step: oaz_trainer_* against oracle/train_ref.py, a float64
torch-CPU restatement of net.rs forward(train=true) + alphaloss + tch SGD (train.rs:264-313).

Tolerances (fp32 GPU vs fp64 CPU): gradients within 2e-4 x the tensor's max |g| (+1e-7), losses
within 1e-5 relative, parameters / running stats within 1e-6 + 1e-5 relative after the step.
"""
import sys
from pathlib import Path

import numpy as np
import pytest

from conftest import random_positions
from onitama_az import _abi
from onitama_az.weights import canonical_layout, named_from_blob, random_weights

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "oracle"))


def _batch(orc, n, seed):
    rng = np.random.default_rng(seed)
    states = random_positions(orc, n, seed=seed)
    samples = np.zeros(n, dtype=_abi.SAMPLE_DTYPE)
    samples["state"] = states
    pi = rng.random((n, 50)) * (rng.random((n, 50)) < 0.3)
    pi[:, 0] += 1e-3  # never an all-zero row
    samples["pi"] = (pi / pi.sum(1, keepdims=True)).astype(np.float32)
    samples["z"] = rng.integers(-1, 2, n).astype(np.float32)
    planes = np.stack([orc.encode(states[i]) for i in range(n)])
    return samples, planes


def _weights(seed, blocks):
    """Random init with non-trivial BN affine/running statistics."""
    rng = np.random.default_rng(seed)
    w = random_weights(seed, blocks).copy()
    off = 0
    for name, shape in canonical_layout(blocks):
        n = int(np.prod(shape))
        if name.endswith("running_var"):
            w[off:off + n] = rng.uniform(0.5, 2.0, n)
        elif name.endswith("running_mean") or (("bn" in name) and name.endswith("bias")):
            w[off:off + n] = rng.normal(0, 0.1, n)
        elif ("bn" in name) and name.endswith("weight"):
            w[off:off + n] = rng.uniform(0.7, 1.3, n)
        off += n
    return w.astype(np.float32)


def _close_grads(got, ref):
    errs = {}
    for k, g in ref.items():
        scale = float(np.abs(g).max())
        errs[k] = (float(np.abs(got[k].reshape(g.shape) - g).max()), scale)
    worst = sorted(errs.items(), key=lambda kv: -kv[1][0] / (2e-4 * kv[1][1] + 1e-7))[:4]  # closest to the bar
    print("gradient errors closest to the bar (err, max|g|):", [(k, f"{e:.2e}", f"{sc:.2e}") for k, (e, sc) in worst])
    for k, (err, scale) in errs.items():
        assert err <= 2e-4 * scale + 1e-7, (k, err, scale)


def _close_params(got, ref):
    for k, p in ref.items():
        np.testing.assert_allclose(got[k].reshape(p.shape), p, rtol=1e-5, atol=1e-6, err_msg=k)


# ---- CPU: the restatement itself ------------------------------------------------------------------
def test_reference_loss_quirks():
    import torch
    from train_ref import alphaloss
    v = torch.tensor([[0.5], [-0.25], [0.0]], dtype=torch.float64)
    z = torch.tensor([1.0, -1.0, 0.0], dtype=torch.float64)
    lv, _ = alphaloss(v, torch.full((3, 2, 25), 0.02, dtype=torch.float64), torch.zeros(3, 2, 25, dtype=torch.float64),
                      z, broadcast=True)
    ref = np.mean([(zj - vi) ** 2 for vi in (0.5, -0.25, 0.0) for zj in (1.0, -1.0, 0.0)])  # [B,B] broadcast
    assert abs(float(lv) - ref) < 1e-12
    lv2, _ = alphaloss(v, torch.full((3, 2, 25), 0.02, dtype=torch.float64), torch.zeros(3, 2, 25, dtype=torch.float64),
                       z, broadcast=False)
    assert abs(float(lv2) - np.mean([(1 - 0.5) ** 2, (-1 + 0.25) ** 2, 0.0])) < 1e-12
    p = torch.full((2, 2, 25), 1 / 50, dtype=torch.float64)
    pi = torch.zeros(2, 2, 25, dtype=torch.float64)
    pi[:, 0, 0] = 1.0
    _, lp = alphaloss(torch.zeros(2, 1, dtype=torch.float64), p, pi, torch.zeros(2, dtype=torch.float64))
    assert abs(float(lp) - np.log(50) / 25) < 1e-12  # sum over dim 1, mean over B*25


def test_choose_batches_without_replacement():
    from onitama_az.trainer import choose_batches
    idx = choose_batches(np.random.default_rng(0), 1000, 512, 3)
    assert idx.shape == (3, 512) and idx.dtype == np.int32
    for row in idx:
        assert len(set(row.tolist())) == 512 and row.min() >= 0 and row.max() < 1000


def test_trainer_without_device_is_a_loud_error(lib):
    if _abi.device_count() > 0:
        pytest.skip("a GPU is visible")
    from onitama_az.trainer import Trainer
    with pytest.raises(_abi.OazError, match="device"):
        Trainer(blocks=3)


# ---- GPU parity ---------------------------------------------------------------------------------
def _run_steps(orc, blocks, B, steps, broadcast=True, seed=1):
    from onitama_az.trainer import Trainer
    from train_ref import train_step
    samples, planes = _batch(orc, B * steps, seed)
    w = _weights(seed, blocks)
    named = named_from_blob(w, blocks)
    with Trainer(blocks=blocks, max_batch=B, value_loss_broadcast=broadcast) as tr:
        tr.set_weights(w)
        tr.load_samples(samples)
        idx = np.arange(B * steps, dtype=np.int32).reshape(steps, B)[:, ::-1].copy()  # non-trivial gather
        tr.set_batches(idx)
        bufs = None
        for s in range(steps):
            rows = idx[s]
            named, grads, lv, lp, bufs = train_step(named, planes[rows], samples["pi"][rows], samples["z"][rows],
                                                    blocks, bufs=bufs, broadcast=broadcast)
            tr.backward(s)
            g = named_from_blob(tr.grads(), blocks)
            _close_grads(g, grads)
            tr.apply(1.0)
            v, p, k = tr.losses()
            assert k == 1
            assert abs(v - lv) <= 1e-5 * abs(lv) + 1e-7 and abs(p - lp) <= 1e-5 * abs(lp) + 1e-7, (v, lv, p, lp)
            _close_params(named_from_blob(tr.get_weights(), blocks), named)


@pytest.mark.gpu
def test_train_step_matches_reference_restatement(orc):
    _run_steps(orc, blocks=3, B=64, steps=1)


@pytest.mark.gpu
def test_train_two_steps_momentum(orc):
    _run_steps(orc, blocks=2, B=32, steps=2, seed=5)


@pytest.mark.gpu
def test_train_step_elementwise_value_loss(orc):
    _run_steps(orc, blocks=1, B=16, steps=1, broadcast=False, seed=7)


@pytest.mark.gpu
def test_train_step_reference_batch_512(orc):
    _run_steps(orc, blocks=3, B=512, steps=1, seed=9)


@pytest.mark.gpu
def test_train_epochs_reduce_loss(orc):
    from onitama_az.trainer import Trainer, train_epochs
    samples, _ = _batch(orc, 1024, 11)
    with Trainer(blocks=2, max_batch=128, learning_rate=2e-2) as tr:
        tr.set_weights(_weights(11, 2))
        hist = train_epochs(tr, samples, epochs=6, batch=128, seed=0)
    assert len(hist) == 6 and all(h.steps == 8 for h in hist)
    assert hist[-1].loss < hist[0].loss, [h.loss for h in hist]


@pytest.mark.gpu
def test_alphazero_loop_end_to_end(tmp_path):
    """train.rs:158-412 in miniature: self-play -> SGD epochs -> pit -> checkpoints."""
    import json
    import os
    from onitama_az.evaluator import EvaluatorConfig
    from onitama_az.mcts import AlphaZeroMctsConfig, ConvResNetConfig
    from onitama_az.train_loop import LoopConfig, train
    from onitama_az.weights import blob_from_named, read_ot
    cfg = LoopConfig(model_config=ConvResNetConfig(resnet_block_amnt=1),
                     mcts_config=AlphaZeroMctsConfig(exploration_c=5.0, max_playouts=8, train=True),
                     iterations=2, training_epochs=2, train_batch_size=32, self_play_game_amnt=16,
                     save_checkpoint=2, evaluation_checkpoint=1, max_plies=40,
                     evaluator_config=EvaluatorConfig(game_amnt=2, max_plies=20, seed=3))
    st = train(cfg, folder=str(tmp_path), eval_sims=8)
    assert st.iteration == [1, 2] and len(st.fight_statistics) == 2
    assert all(g["positions_retrieved"] > 32 for g in st.games_played)
    assert all(np.isfinite(st.loss))
    files = os.listdir(tmp_path)
    ckpt = [f for f in files if f.startswith("model_2_") and f.endswith(".ot")]
    assert ckpt and "stats.json" in files
    w = blob_from_named(read_ot(str(tmp_path / ckpt[0])), 1)
    assert w.size == 240006 - 2 * 2 * (64 * 64 * 9 + 64 * 5)
    json.load(open(tmp_path / "stats.json"))
