"""CPU: pin the oracle to the reference's own known-answer tests and to torch goldens, and
cross-check its search against the independent pure-Python restatement (tests/pyref.py)."""
import numpy as np
import pytest

import pyref
from conftest import kat_state, random_positions

NAMES = ["Tiger", "Dragon", "Frog", "Rabbit", "Crab", "Elephant", "Goose", "Rooster", "Monkey",
         "Mantis", "Crane", "Horse", "Ox", "Boar", "Eel", "Cobra"]


def _mv_tuple(m):
    return (int(m["from_"]), int(m["to"]), int(m["piece"]))


def _notation(i):
    return "abcde"[i % 5] + str(5 - i // 5)


def test_bits_kat(kats):
    b = kats["bits"]
    v = b["get_bit"]["value"]
    assert [(v >> (31 - i)) & 1 for i in range(32)] == b["get_bit"]["expected"]  # common/mod.rs:82
    for (y, x), exp in b["from_2d_to_bitboard"]:
        assert 0x8000_0000 >> (y * 5 + x) == exp


def test_movegen_kats(orc, kats):  # state.rs:419-492, 818-889
    for case in kats["movegen"]:
        s = kat_state(case["state"], case["color"])
        got = sorted(_mv_tuple(m) for m in orc.movegen(s) if int(m["slot"]) == case["slot"])
        assert got == sorted(tuple(m) for m in case["moves"]), case["src"]


def test_make_move_kats(orc, kats):  # state.rs:494-816
    for case in kats["make_move"]:
        s = kat_state(case["state"], case["color"])
        res = orc.make_move(s, tuple(case["move"]), case["color"])
        assert res == case["result"], case["src"]
        for field, color, sq, val in case["bits"]:
            assert (int(s[field][0][color]) >> (31 - sq)) & 1 == val, case["src"]
        assert int(s["cards"][0][4]) == case["neutral"], case["src"]
        for field, color, val in case.get("equals", []):
            assert int(s[field][0][color]) == val, case["src"]
        for field, color in case.get("nonzero", []):
            assert int(s[field][0][color]) > 0, case["src"]


def test_expansion_order_kats(orc, kats):  # onitama-game/src/ai/mcts/mcts_arena.rs:403-457
    for case in kats["expansion"]:
        s = kat_state(case["state"], case["color"])
        got = [f"{NAMES[int(s['cards'][0][int(m['slot'])])]} {_notation(int(m['from_']))}-{_notation(int(m['to']))}"
               for m in orc.movegen(s)]
        assert got == case["children"], case["src"]


def test_pyref_rules_agree_with_oracle(orc):
    """Two independent restatements of the rules agree on 3000 random positions."""
    pos = random_positions(orc, 3000, seed=11)
    for s in pos:
        s = s.reshape(1)
        st = pyref.S(list(map(int, s["kings"][0])), list(map(int, s["pawns"][0])), list(map(int, s["cards"][0])),
                     int(s["to_move"][0]))
        ref = pyref.legal_moves(st, st.color)
        got = [(int(m["slot"]), int(m["from_"]), int(m["to"]), int(m["piece"])) for m in orc.movegen(s)]
        assert got == ref
        assert orc.current_state(s) == pyref.current_state(st)
        for mv in ref[:3]:
            a = s.copy()
            b = st.copy()
            r1 = orc.make_move(a, (mv[1], mv[2], mv[3], mv[0]), st.color)
            r2 = pyref.make_move(b, mv, st.color)
            assert r1 == r2
            assert list(map(int, a["kings"][0])) == b.kings and list(map(int, a["pawns"][0])) == b.pawns
            assert list(map(int, a["cards"][0])) == b.cards


def test_attack_maps_match_pyref(orc):
    assert np.array_equal(orc.attack_maps(), np.array(pyref.ATTACK, dtype=np.uint32))


def test_encoder_planes(orc):  # common.rs:26-80
    pos = random_positions(orc, 50, seed=3)
    for s in pos:
        s = s.reshape(1)
        p = orc.encode(s)
        color = int(s["to_move"][0])
        bits = [int(s["pawns"][0][0]), int(s["kings"][0][0]), int(s["pawns"][0][1]), int(s["kings"][0][1])]
        for c in range(4):
            assert [int(v) for v in p[c].reshape(-1)] == [(bits[c] >> (31 - i)) & 1 for i in range(25)]
        cards = set(int(s["cards"][0][i]) for i in ((0, 1) if color == 0 else (2, 3)))
        for k in range(16):
            assert np.all(p[4 + k] == (1.0 if k in cards else 0.0))
        assert np.all(p[20] == float(color))


@pytest.mark.parametrize("name,blocks", [("trained3", 3), ("random3", 3), ("random6", 6)])
def test_oracle_nn_matches_torch_goldens(orc, nn_golden, trained3, name, blocks):
    from onitama_az.weights import random_weights
    w = trained3 if name == "trained3" else random_weights(0 if name == "random3" else 1, blocks)
    p, v = orc.nn_forward(w, blocks, nn_golden["states"])
    np.testing.assert_allclose(p, nn_golden[f"policy_{name}"], atol=1e-5, rtol=0)
    np.testing.assert_allclose(v, nn_golden[f"value_{name}"], atol=1e-5, rtol=0)


def _pyref_state(s):
    s = s.reshape(1)
    return pyref.S(list(map(int, s["kings"][0])), list(map(int, s["pawns"][0])), list(map(int, s["cards"][0])),
                   int(s["to_move"][0]))


def test_oracle_search_matches_pyref(orc):
    """The C oracle's search equals the independent Python restatement node for node."""
    pos = random_positions(orc, 6, seed=5, max_plies=10)
    for s in pos:
        cfg = orc.search_cfg(sims=40, c_puct=5.0, evaluator=orc.EVAL_HASH)
        mv, pi, nodes, _ = orc.search(cfg, s)
        ref_mv, ref_pi, arena = pyref.search(_pyref_state(s), 40, 5.0)
        assert len(nodes) == len(arena)
        for nd, rn in zip(nodes, arena):
            assert int(nd["N"]) == rn.visits
            assert float(nd["W"]) == rn.reward  # bit-exact f64
            assert float(nd["P"]) == rn.prob
            assert bool(nd["flags"] & 1) == rn.expanded and bool(nd["flags"] & 2) == rn.terminal
            assert int(nd["nch"]) == len(rn.children)
        assert np.array_equal(pi.reshape(-1), np.array(ref_pi, dtype=np.float32))
        assert (int(mv["slot"]), int(mv["from_"]), int(mv["to"]), int(mv["piece"])) == ref_mv


def test_oracle_search_invariants(orc):
    pos = random_positions(orc, 8, seed=9)
    for s in pos:
        cfg = orc.search_cfg(sims=100, c_puct=5.0, evaluator=orc.EVAL_HASH)
        mv, pi, nodes, st = orc.search(cfg, s)
        assert st.sims == 100 and int(nodes[0]["N"]) == 100
        # a playout's evaluation is unused only when it ends on a won leaf (a won but unflagged leaf,
        # possible below a random root that is already won, is still expanded with its priors)
        assert st.sims - st.terminal_leaves <= st.nn_evals <= st.sims
        for i, nd in enumerate(nodes):  # visits of children = visits of parent minus its own eval
            if nd["flags"] & 1 and nd["nch"]:
                ch = nodes[int(nd["first"]): int(nd["first"]) + int(nd["nch"])]
                assert int(ch["N"].sum()) <= int(nd["N"]) - 1 or nd["flags"] & 2
        if nodes[0]["nch"]:
            assert abs(pi.sum() - 1.0) < 1e-6


def test_oracle_selfplay_game_semantics(orc):
    """train.rs:35-98: z = reward(final, colour); ply cap max_plies+2; colours alternate."""
    cfg = orc.search_cfg(sims=8, c_puct=5.0, evaluator=orc.EVAL_HASH)
    for gid in range(4):
        samples, res, plies, _ = orc.selfplay_game(cfg, gid, max_plies=150)
        assert len(samples) == plies <= 152
        cols = samples["state"]["to_move"]
        assert np.all(cols[1:] != cols[:-1])
        if res in (1, 2):
            win = 0 if res == 1 else 1
            assert np.all(samples["z"] == np.where(cols == win, 1.0, -1.0))
        else:
            assert plies == 152 and np.all(samples["z"] == 0)
    samples, res, plies, _ = orc.selfplay_game(cfg, 0, max_plies=2)  # cut after max_plies + 2 plies
    assert plies <= 4 and (res in (1, 2) or (plies == 4 and np.all(samples["z"] == 0)))


def test_cpu_baseline_libtorch_evaluator_matches_goldens(nn_golden, trained3, tmp_path):
    """bench.py's cpu_baseline program (oracle/cpu_baseline.cpp: batch-1 ATen CPU forwards, the
    reference's execution shape) evaluates the golden positions within 1e-5 of the torch goldens,
    so its sims/s are those of the same network."""
    import subprocess
    from pathlib import Path
    exe = Path(__file__).resolve().parents[1] / "oracle" / "build" / "oaz_cpu_baseline"
    if not exe.exists():
        pytest.skip("oaz_cpu_baseline not built (torch headers absent)")
    wf, sf, of = tmp_path / "w.f32", tmp_path / "s.bin", tmp_path / "o.f32"
    trained3.astype(np.float32).tofile(wf)
    nn_golden["states"].tofile(sf)
    subprocess.run([str(exe), "nn", str(wf), "3", str(sf), str(of)], check=True, timeout=120)
    out = np.fromfile(of, dtype=np.float32).reshape(-1, 51)
    assert len(out) == 256
    assert np.abs(out[:, :50] - nn_golden["policy_trained3"].reshape(256, 50)).max() < 1e-5
    assert np.abs(out[:, 50] - nn_golden["value_trained3"]).max() < 1e-5
