"""CPU checks of bench.py's contract and accounting (no GPU): the metric and workloads are
BASELINE.json's, the FLOP counts behind `roofline.achieved` follow from the net.rs architecture
(SURVEY.md 8a-A7 / 8d), and the defaults give the driver's N=1 short run."""
import importlib.util
import json
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


@pytest.fixture(scope="module")
def bench():
    spec = importlib.util.spec_from_file_location("oaz_bench_contract", ROOT / "bench.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)  # main() is guarded: nothing runs at import
    return mod


@pytest.fixture(scope="module")
def baseline():
    return json.loads((ROOT / "BASELINE.json").read_text())


def test_metric_is_baselines(bench, baseline):
    assert bench.METRIC == baseline["metric"]


def test_configs_are_baselines(bench, baseline):
    cfgs = baseline["configs"]
    c2, c3, c5 = bench.CONFIGS["c2"], bench.CONFIGS["c3"], bench.CONFIGS["c5"]
    assert (c2["games"], c2["sims"], c2["blocks"], c2["precision"]) == (4096, 100, 3, "fp32")
    assert "4096" in cfgs[1] and "100 sims" in cfgs[1] and "3-block" in cfgs[1]
    assert (c3["games"], c3["sims"]) == (65536, 400) and "65536" in cfgs[2] and "400 sims" in cfgs[2]
    # C5: the full 16-card deck (random deals, not the fixed 5), 800 sims, 6 blocks, bf16
    assert (c5["sims"], c5["blocks"], c5["precision"], c5["fixed_deck"]) == (800, 6, "bf16", 0)
    assert "800 sims" in cfgs[4] and "6-block" in cfgs[4] and "bf16" in cfgs[4]


def _macs_per_position(blocks, onboard_taps):
    """net.rs:9-232: 3x3 conv 21->64 on 25 squares, `blocks` residual blocks of two 3x3 64->64
    convs, value head (1x1 conv 64->1, FC 25->64, FC 64->1), policy head (1x1 conv 64->2, FC
    50->50). `onboard_taps` = (square, tap) pairs counted for the 3x3 convs."""
    conv_in = onboard_taps * 21 * 64
    res = blocks * 2 * onboard_taps * 64 * 64
    value = 25 * 64 * 1 + 25 * 64 + 64 * 1
    policy = 25 * 64 * 2 + 50 * 50
    return conv_in + res + value + policy


def test_onboard_taps_of_a_5x5_board():
    n = sum(1 for r in range(5) for c in range(5) for dr in (-1, 0, 1) for dc in (-1, 0, 1)
            if 0 <= r + dr < 5 and 0 <= c + dc < 5)
    assert n == 169


@pytest.mark.parametrize("blocks", [3, 5, 6])
def test_flop_per_sim_from_architecture(bench, blocks):
    assert bench.FLOP_PER_SIM[blocks] == 2 * _macs_per_position(blocks, 25 * 9)
    assert bench.nonzero_flop_per_sim(blocks) == 2 * _macs_per_position(blocks, 169)


def test_peaks(bench):
    # split kernels: every fp32 MAC costs 6 bf16 (x6) or 3 fp16 (h3) MFMA products
    assert bench.PEAK_TFLOPS["fp32_split"] == pytest.approx(bench.PEAK_TFLOPS["bf16"] / 6)
    assert bench.PEAK_TFLOPS["fp32_split16"] == pytest.approx(bench.PEAK_TFLOPS["bf16"] / 3)
    assert set(bench.NN_KERNEL) >= {"fp32", "fp32_split", "fp32_split16", "bf16"}


def test_defaults_are_the_drivers_short_n1_run(bench, monkeypatch):
    monkeypatch.setattr(sys, "argv", ["bench.py"])
    a = bench.parse()
    assert (a.gpus, a.config, a.fp32_kernel, a.mode) == (1, "c3", "split16", "selfplay")
    assert a.steps >= 1 and a.warmup >= a.stagger  # staggered starts end inside the warm-up
    assert a.cpu_seconds <= 30  # the CPU baseline is a bounded sample


@pytest.mark.parametrize("games,parts,expect", [(65536, 0, 2), (4096, 0, 2), (2047, 0, 1), (65536, 1, 1),
                                                 (65536, 4, 4), (65536, 3, 2)])
def test_sim_parts_mirrors_engine(bench, games, parts, expect):
    # oaz_engine.cpp game_parts: auto = 2 from 2048 games; 1, 2 or 4 when set (the engine itself
    # rejects other values, test_host.py)
    assert bench.sim_parts(games, parts) == expect


def test_extra_modes_parse(bench, monkeypatch):
    # the SURVEY 8f rows with their own measurement: train (#2), pure_mcts (#4), arena (#1)
    for mode in ("train", "pure_mcts", "arena"):
        monkeypatch.setattr(sys, "argv", ["bench.py", "--mode", mode])
        assert bench.parse().mode == mode
    monkeypatch.setattr(sys, "argv", ["bench.py", "--mode", "arena", "--arena-games", "128"])
    assert bench.parse().arena_games == 128
    assert "games/sec" in bench.ARENA_METRIC


def test_train_byte_formula(bench):
    """train_algorithmic_bytes: per SGD step every activation-sized tensor the kernels read or write (S = 25 B
    rows x 64 fp32), the weight-gradient partials written and re-read per layer, and the SGD's five parameter
    passes; its write side alone (measured exactly by WRITE_SIZE on the GPU) is the
    intermediate tensors once each plus the partials."""
    blocks, B = 5, 512
    L, S = 1 + 2 * blocks, 25 * B * 64 * 4
    part = 9 * 25 * 2 * 64 * 64 * 4
    total = bench.train_algorithmic_bytes(blocks, B)
    assert 600e6 < total < 700e6, total
    # writes: Z and A per conv (forward), M of the last conv (heads), dZ per conv, M per input gradient,
    # the partials of L - 0.5 layers (layer 0 has 32 input channels), P and MOM (SGD)
    nparam = L * (64 * 64 * 9 + 5 * 64) - 64 * 43 * 9 + 64 + 5 + 64 * 25 + 64 + 64 + 1 + 128 + 10 + 2500 + 50
    writes = 2 * L * S + S + L * S + (L - 1) * S + (L - 0.5) * part + 2 * 4 * nparam
    assert abs(writes - 226e6) / 226e6 < 0.02, writes  # the GPU's WRITE_SIZE per step (profiles/r05b_train.json)


def test_pure_mcts_and_arena_defaults(bench, monkeypatch):
    monkeypatch.setattr(sys, "argv", ["bench.py", "--mode", "pure_mcts"])
    a = bench.parse()
    assert a.pm_games == 1 << 20 and a.pm_playouts == 400
    monkeypatch.setattr(sys, "argv", ["bench.py", "--mode", "arena"])
    assert bench.parse().arena_games == 131072


def test_grp_launches_per_ply(bench):
    """k_search_grp launches per ply follow the engine's root-noise chunk (max(16, min(512, sims))): a C2 ply
    (100 simulations) is one launch, the Agent default (5 000) ten."""
    assert [bench.grp_launches_per_ply(s) for s in (8, 16, 100, 512, 1000, 5000)] == [1, 1, 1, 1, 2, 10]
