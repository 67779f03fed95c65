"""GPU parity tests: the HIP path (through the C ABI) against the oracle and the goldens.

Bars: rules/moves/masks/results bit-exact; NN within 1e-4 of torch-CPU goldens; MCTS trees
bit-exact (every node's N, W, P, move, children, flags) against the oracle whenever both run
the same evaluator outputs (HASH test evaluator, or the GPU network fed to the oracle).
"""
import ctypes as C
from pathlib import Path

import numpy as np
import pytest

from conftest import kat_state, random_positions
from onitama_az import _abi
from onitama_az.engine import Engine
from onitama_az.game import (Deck, DoneMove, GameState, Move, MoveResult, PieceKind, PlayerColor, State,
                             ORIGINAL_CARDS, CARD_NAMES, current_state_batch, encode_batch, movegen_batch,
                             movegen_masks_batch, step_batch)
from onitama_az.weights import random_weights

ROOT = Path(__file__).resolve().parents[1]

pytestmark = pytest.mark.gpu

NODE_FIELDS = ("W", "P", "N", "first", "mv", "nch", "flags")


def grp_launches(sims):
    """k_search_grp launches of an engine created with `sims` whose games fit one round of 16-game workgroups:
    one per root-noise chunk of max(16, min(512, sims)) simulations (oaz_engine.cpp, noise_chunk_for)."""
    c = max(16, min(512, sims))
    return (sims + c - 1) // c


def _mv(m):
    return tuple(int(m[k]) for k in ("from_", "to", "piece", "slot"))


# ---- rules -------------------------------------------------------------------------------
def test_rules_kats_through_mirror(kats):
    for case in kats["movegen"]:  # state.rs:419-492, 818-889
        d = case["state"]
        st = State(Deck([ORIGINAL_CARDS[i] for i in d["deck"]]), d["kings"], d["pawns"])
        card = st.deck.cards[case["slot"]]
        got = sorted(st.generate_legal_moves(PlayerColor(case["color"]), card))
        assert got == sorted(Move(a, b, PieceKind(c)) for a, b, c in case["moves"]), case["src"]
    for case in kats["make_move"]:  # state.rs:494-816
        d = case["state"]
        st = State(Deck([ORIGINAL_CARDS[i] for i in d["deck"]]), d["kings"], d["pawns"])
        f, t, p, slot = case["move"]
        res = st.make_move(Move(f, t, PieceKind(p)), PlayerColor(case["color"]), slot)
        assert res == MoveResult(case["result"]), case["src"]
        for field, color, sq, val in case["bits"]:
            assert (getattr(st, field)[color] >> (31 - sq)) & 1 == val
        assert st.deck.neutral_card().index == case["neutral"]
        for field, color, val in case.get("equals", []):
            assert getattr(st, field)[color] == val
    for case in kats["expansion"]:  # onitama-game/src/ai/mcts/mcts_arena.rs:403-457
        d = case["state"]
        st = State(Deck([ORIGINAL_CARDS[i] for i in d["deck"]]), d["kings"], d["pawns"])
        got = [f"{CARD_NAMES[st.deck.cards[s].index]} {Move.convert_idx_to_notation(m.from_)}-"
               f"{Move.convert_idx_to_notation(m.to)}" for s, m in st.generate_all_legal_moves(PlayerColor(case["color"]))]
        assert got == case["children"], case["src"]


def test_movegen_bitexact_vs_oracle(orc):
    pos = random_positions(orc, 20000, seed=101)
    masks = movegen_masks_batch(pos)
    moves, counts = movegen_batch(pos)
    for i in range(len(pos)):
        ref = orc.movegen(pos[i])
        assert counts[i] == len(ref)
        assert moves[i, : len(ref)].tobytes() == ref.tobytes()
        assert not moves[i, len(ref):].tobytes().strip(b"\0")  # the entries past the count are zero
        assert np.array_equal(masks[i], orc.movegen_masks(pos[i]))


def test_rules_entry_points_from_concurrent_threads(orc):
    """oaz_movegen / oaz_step / oaz_encode from 6 threads at once, every thread with its own batch size (the
    per-device rules context grows its scratch under its lock): each thread's results equal the serial ones."""
    import threading
    pos = random_positions(orc, 3000, seed=111)
    sizes = [3000, 17, 1000, 1, 2500, 640]
    ref = {}
    for n in set(sizes):
        sub = np.ascontiguousarray(pos[:n])
        mv, ct = movegen_batch(sub)
        ref[n] = (mv.copy(), ct.copy(), encode_batch(sub).copy())
    errs = []

    def run(n):
        try:
            sub = np.ascontiguousarray(pos[:n])
            for _ in range(5):
                mv, ct = movegen_batch(sub)
                pl = encode_batch(sub)
                assert np.array_equal(mv, ref[n][0]) and np.array_equal(ct, ref[n][1]), n
                assert np.array_equal(pl, ref[n][2]), n
                keep = ct > 0
                step_batch(np.ascontiguousarray(sub[keep]), np.ascontiguousarray(mv[keep, 0]))
        except Exception as ex:  # noqa: BLE001
            errs.append(ex)
    th = [threading.Thread(target=run, args=(n,)) for n in sizes]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs, errs


def test_step_and_terminal_bitexact_vs_oracle(orc):
    import random
    rng = random.Random(5)
    pos = random_positions(orc, 5000, seed=202)
    moves, counts = movegen_batch(pos)
    keep = counts > 0
    pos, moves, counts = pos[keep], moves[keep], counts[keep]
    pick = np.array([moves[i, rng.randrange(int(counts[i]))] for i in range(len(pos))], dtype=_abi.MOVE_DTYPE)
    gpu = pos.copy()
    res = step_batch(gpu, pick)
    for i in range(len(pos)):
        ref = pos[i: i + 1].copy()
        r = orc.make_move(ref, _mv(pick[i]), int(ref["to_move"][0]))
        ref["to_move"][0] ^= 1
        assert res[i] == r
        assert gpu[i: i + 1].tobytes() == ref.tobytes()
    cs = current_state_batch(gpu)
    assert [int(x) for x in cs] == [orc.current_state(gpu[i]) for i in range(len(gpu))]


def test_encode_vs_oracle(orc):
    pos = random_positions(orc, 500, seed=303)
    planes = encode_batch(pos)
    for i in range(len(pos)):
        assert np.array_equal(planes[i], orc.encode(pos[i]))


# ---- NN ----------------------------------------------------------------------------------
@pytest.mark.parametrize("precision", [_abi.FP32, _abi.FP32_SPLIT, _abi.FP32_SPLIT16])
@pytest.mark.parametrize("name,blocks", [("trained3", 3), ("random3", 3), ("random6", 6)])
def test_nn_matches_torch_goldens(nn_golden, trained3, name, blocks, precision):
    """The three fp32 kernels (exact fp32 MFMA, the bf16x6 split, the fp16x3 split) against the
    torch-CPU fp32 goldens of the net.rs op graph, within the north star's 1e-4."""
    w = trained3 if name == "trained3" else random_weights(0 if name == "random3" else 1, blocks)
    with Engine(games=256, sims=1, blocks=blocks, evaluator=_abi.EVAL_NN, precision=precision) as e:
        e.load_weights(w)
        p, v = e.nn_forward(nn_golden["states"])
    tol = 1e-4  # north_star: policy/value within 1e-4 fp32
    assert np.abs(p - nn_golden[f"policy_{name}"]).max() < tol
    assert np.abs(v - nn_golden[f"value_{name}"]).max() < tol
    assert np.allclose(p.reshape(-1, 50).sum(1), 1.0, atol=1e-5)


@pytest.mark.parametrize("name,blocks", [("trained3", 3), ("random3", 3), ("random6", 6)])
def test_nn_split16_error_at_fp32_level(nn_golden, trained3, name, blocks):
    """OAZ_FP32_SPLIT16 (hi/lo fp16 terms, three products) is an fp32 path, not a reduced-precision
    one: its distance to the torch fp32 goldens stays within 1e-5 (10x inside the north star's 1e-4;
    a single bf16 or fp16 product per MAC, or a two-term bf16 split, lands at 1e-4 - 1e-2) and within
    4x of the exact-fp32 MFMA kernel's own distance (+1e-6 for ties at the fp32 rounding level)."""
    w = trained3 if name == "trained3" else random_weights(0 if name == "random3" else 1, blocks)
    err = {}
    for prec in (_abi.FP32, _abi.FP32_SPLIT16):
        with Engine(games=256, sims=1, blocks=blocks, evaluator=_abi.EVAL_NN, precision=prec) as e:
            e.load_weights(w)
            p, v = e.nn_forward(nn_golden["states"])
        err[prec] = max(np.abs(p - nn_golden[f"policy_{name}"]).max(), np.abs(v - nn_golden[f"value_{name}"]).max())
    assert err[_abi.FP32_SPLIT16] < 1e-5, err
    assert err[_abi.FP32_SPLIT16] <= 4 * err[_abi.FP32] + 1e-6, err


# k_nn_h3s (one position per workgroup) runs launches of up to one round of workgroups (the CU count,
# 256 on MI355X; >= 64 on any device), k_nn_h3 (16-position tiles) larger ones: B = 64 and B = 1024 pick
# one each on every device.
SMALL_B, BIG_B = 64, 1024


@pytest.mark.parametrize("B,per_wg", [(SMALL_B, 1), (BIG_B, 16)])
def test_nn_split16_range_fallback_recomputes_all_tiles(nn_golden, trained3, B, per_wg):
    """Activations beyond the fp16 range (here every position's: BN-folded first-layer bias 1e5) make
    each workgroup recompute its positions (16, or 1 in k_nn_h3s) with the bf16x6 split inside the same
    launch: the results equal the OAZ_FP32_SPLIT engine's bit for bit, and the fallback counts every
    workgroup."""
    from onitama_az.weights import blob_from_named, named_from_blob
    named = {k: v.copy() for k, v in named_from_blob(trained3.copy(), 3).items()}
    named["bn1|bias"][:] = 1.0e5  # first-layer activations ~1e5 > 65504
    bad = blob_from_named(named, 3)
    states = np.ascontiguousarray(np.tile(nn_golden["states"], (B + 255) // 256)[:B])
    with Engine(games=B, sims=1, blocks=3, evaluator=_abi.EVAL_NN, precision=_abi.FP32_SPLIT16) as e:
        e.load_weights(bad)
        p16, v16 = e.nn_forward(states)
        assert e.nn_fallbacks() == B // per_wg
        e.load_weights(trained3)
        p, _ = e.nn_forward(states)
        assert e.nn_fallbacks() == B // per_wg  # sane weights: no further workgroup
    gold = np.tile(nn_golden["policy_trained3"], ((B + 255) // 256, 1, 1))[:B]
    assert np.abs(p - gold).max() < 1e-5
    with Engine(games=B, sims=1, blocks=3, evaluator=_abi.EVAL_NN, precision=_abi.FP32_SPLIT) as e:
        e.load_weights(bad)
        px, vx = e.nn_forward(states)
    assert np.isfinite(px).all() and np.isfinite(vx).all()
    assert np.array_equal(p16, px) and np.array_equal(v16, vx)


@pytest.mark.parametrize("reps,per_wg", [(1, 1), (4, 16)])
def test_nn_split16_range_fallback_only_overflowing_tiles(nn_golden, trained3, reps, per_wg):
    """Only positions whose mover holds card 7 (Rooster) overflow (its first-layer plane weights are
    scaled by 1e6): exactly the workgroups containing such a position are recomputed (bit-equal to the
    OAZ_FP32_SPLIT kernel) — single positions at 256 (k_nn_h3s), 16-position tiles at 1024 (k_nn_h3) —
    the others keep the fp16x3 result (bit-equal to a batch of those positions alone, and within 1e-5
    of exact fp32)."""
    from onitama_az.game import encode_batch
    from onitama_az.weights import blob_from_named, named_from_blob
    named = {k: v.copy() for k, v in named_from_blob(trained3.copy(), 3).items()}
    named["conv_init_1|weight"][:, 4 + 7] *= 1.0e6
    bad = blob_from_named(named, 3)
    states = np.ascontiguousarray(np.tile(nn_golden["states"], reps))
    n = len(states)
    planes = encode_batch(states)
    hot = planes[:, 4 + 7].reshape(n, -1).max(1) > 0  # the mover holds card 7
    wg_hot = hot.reshape(n // per_wg, per_wg).any(1)
    assert 0 < wg_hot.sum() < n // per_wg
    out = {}
    for prec in (_abi.FP32_SPLIT16, _abi.FP32_SPLIT, _abi.FP32):
        with Engine(games=n, sims=1, blocks=3, evaluator=_abi.EVAL_NN, precision=prec) as e:
            e.load_weights(bad)
            out[prec] = e.nn_forward(states)
            if prec == _abi.FP32_SPLIT16:
                assert e.nn_fallbacks() == int(wg_hot.sum())
    p16, px, pf = out[_abi.FP32_SPLIT16][0], out[_abi.FP32_SPLIT][0], out[_abi.FP32][0]
    rows = np.repeat(wg_hot, per_wg)
    assert np.array_equal(p16[rows], px[rows])
    assert np.abs(p16[~rows] - pf[~rows]).max() < 1e-5
    # the cold workgroups alone in a clean batch: the same fp16x3 bits
    cold = np.ascontiguousarray(states[~rows])
    with Engine(games=n, sims=1, blocks=3, evaluator=_abi.EVAL_NN, precision=_abi.FP32_SPLIT16) as e:
        e.load_weights(bad)
        pc, _ = e.nn_forward(cold)
        assert e.nn_fallbacks() == 0
    assert np.array_equal(pc, p16[~rows])


@pytest.mark.parametrize("name,blocks", [("trained3", 3), ("trained5", 5), ("random6", 6), ("random0", 0)])
def test_nn_small_batch_kernel_bitidentical_to_tiled(nn_golden, trained3, name, blocks):
    """k_nn_h3s (one position per workgroup: small batches, the Agent API) and k_nn_h3 (16-position
    tiles) compute the same fp16x3 arithmetic element for element, so a position's policy and value are
    bit-identical whichever kernel the batch size picks (B = 1, 64 / 1024) — the network stays
    batch-independent, which the real-network tree-parity tests rely on."""
    if name == "trained5":
        w = np.load(ROOT / "tests/golden/weights_5block_trained.npy")
    else:
        w = trained3 if name == "trained3" else random_weights(7, blocks)
    st = nn_golden["states"]
    with Engine(games=BIG_B, sims=1, blocks=blocks, evaluator=_abi.EVAL_NN, precision=_abi.FP32_SPLIT16) as e:
        e.load_weights(w)
        pb, vb = e.nn_forward(np.ascontiguousarray(np.tile(st, 4)))
        ps, vs = e.nn_forward(np.ascontiguousarray(st[:SMALL_B]))
        singles = [e.nn_forward(np.ascontiguousarray(st[k:k + 1])) for k in (0, 17, 200, 255)]
        assert e.nn_fallbacks() == 0
    assert np.array_equal(pb[256:512], pb[:256]) and np.array_equal(vb[768:], vb[:256])
    assert np.array_equal(ps.view(np.uint32), pb[:SMALL_B].view(np.uint32))
    assert np.array_equal(vs.view(np.uint32), vb[:SMALL_B].view(np.uint32))
    for k, (p1, v1) in zip((0, 17, 200, 255), singles):
        assert np.array_equal(p1[0].view(np.uint32), pb[k].view(np.uint32)) and v1[0] == vb[k], k
    if name == "trained3":
        assert np.abs(ps - nn_golden["policy_trained3"][:SMALL_B]).max() < 1e-5


@pytest.mark.parametrize("name,blocks", [("trained3", 3), ("random3", 3), ("random6", 6)])
def test_nn_bf16_mode_close_to_fp32_goldens(nn_golden, trained3, name, blocks):
    """OAZ_BF16 (BASELINE C5: bf16 MFMA inputs, fp32 accumulation) is a throughput mode, not the
    parity path: it must stay close to the fp32 torch goldens (tolerance 3e-2 absolute)."""
    w = trained3 if name == "trained3" else random_weights(0 if name == "random3" else 1, blocks)
    with Engine(games=256, sims=1, blocks=blocks, evaluator=_abi.EVAL_NN, precision=_abi.BF16) as e:
        e.load_weights(w)
        p, v = e.nn_forward(nn_golden["states"])
    assert np.abs(p - nn_golden[f"policy_{name}"]).max() < 3e-2
    assert np.abs(v - nn_golden[f"value_{name}"]).max() < 3e-2
    assert np.allclose(p.reshape(-1, 50).sum(1), 1.0, atol=1e-5)


@pytest.mark.parametrize("precision", [_abi.FP32, _abi.FP32_SPLIT16])
def test_nn_batch_position_invariance(orc, precision):
    pos = random_positions(orc, 64, seed=404)
    with Engine(games=1024, sims=1, blocks=3, precision=precision) as e:
        p1, v1 = e.nn_forward(pos)
        big = np.concatenate([pos[::-1], pos, pos[:7]])
        p2, v2 = e.nn_forward(big)
        huge = np.concatenate([pos[:5]] + [pos] * 14 + [pos[::-1]])  # > one round: the tiled kernel
        p3, v3 = e.nn_forward(huge)
    assert np.array_equal(p2[64:128], p1) and np.array_equal(v2[64:128], v1)
    assert np.array_equal(p2[:64][::-1], p1)
    assert np.array_equal(p3[5:69], p1) and np.array_equal(v3[-64:][::-1], v1)


# ---- search ------------------------------------------------------------------------------
def _compare_trees(e, g, nodes_ref):
    t = e.tree(g)
    assert len(t) == len(nodes_ref), (len(t), len(nodes_ref))
    for f in NODE_FIELDS:
        a, b = t[f], nodes_ref[f]
        if f == "first":  # defined only for expanded nodes
            a, b = np.where(t["flags"] & 1, a, 0), np.where(nodes_ref["flags"] & 1, b, 0)
        assert np.array_equal(a, b), f


# compact 0: every leaf evaluated in place (default), 1: leaf compaction; parts: the games on 1 or 2 streams
@pytest.mark.parametrize("compact,parts", [(0, 1), (1, 1), (0, 2), (1, 2)])
@pytest.mark.parametrize("sims,c_puct", [(64, 5.0), (200, 2.0)])
def test_search_hash_trees_bitexact(orc, sims, c_puct, compact, parts):
    roots = random_positions(orc, 12, seed=505 + sims)
    with Engine(games=len(roots), sims=sims, c_puct=c_puct, train_noise=0, evaluator=_abi.EVAL_HASH, blocks=0,
                compact=compact, parts=parts) as e:
        r = e.search(roots)
        evals = terminal = 0
        for g in range(len(roots)):
            cfg = orc.search_cfg(sims=sims, c_puct=c_puct, evaluator=orc.EVAL_HASH)
            mv, pi, nodes, st = orc.search(cfg, roots[g])
            _compare_trees(e, g, nodes)
            assert np.array_equal(r.pi[g].reshape(-1), pi.reshape(-1))
            assert _mv(r.moves[g]) == _mv(mv)
            evals += st.nn_evals
            terminal += st.terminal_leaves
    assert r.stats.sims == sims * len(roots)
    # leaf compaction: the network sees exactly the leaves whose evaluation the playout uses
    assert (r.stats.nn_evals, r.stats.terminal_leaves) == (evals, terminal)
    assert r.stats.sims - r.stats.terminal_leaves <= r.stats.nn_evals <= r.stats.sims


@pytest.mark.parametrize("games,parts", [(10, 4), (26, 2), (5, 4), (3, 4), (2, 4)])
def test_search_uneven_parts_compacted_trees_bitexact(orc, games, parts):
    """Games in uneven parts (10 in 4: 3 + 3 + 3 + 1; 26 in 2: the second part starts at game 13, an
    unaligned offset; 5 in 4 would leave the fourth part empty, so it runs as 3 + 2), each part on its
    own stream with its own compaction buckets and rows, leaf compaction forced: every tree equals the
    oracle's."""
    roots = random_positions(orc, games, seed=515)
    with Engine(games=len(roots), sims=96, c_puct=5.0, train_noise=0, evaluator=_abi.EVAL_HASH, blocks=0, compact=1,
                parts=parts) as e:
        r = e.search(roots)
        for g in range(len(roots)):
            mv, pi, nodes, st = orc.search(orc.search_cfg(sims=96, c_puct=5.0, evaluator=orc.EVAL_HASH), roots[g])
            _compare_trees(e, g, nodes)
            assert np.array_equal(r.pi[g].reshape(-1), pi.reshape(-1))
            assert _mv(r.moves[g]) == _mv(mv)


@pytest.mark.parametrize("compact,parts", [(0, 1), (1, 2)])
@pytest.mark.parametrize("precision", [_abi.FP32, _abi.FP32_SPLIT16])
def test_search_nn_trees_bitexact_with_gpu_evaluator(orc, precision, compact, parts):
    """Real network: the oracle's search is fed the GPU network's outputs (batch-1 calls of
    the same kernel), so both searches see identical evaluations and must agree exactly."""
    roots = random_positions(orc, 4, seed=606)
    w = random_weights(3, 3)
    sims = 48
    with Engine(games=len(roots), sims=sims, c_puct=5.0, train_noise=0, evaluator=_abi.EVAL_NN, blocks=3,
                precision=precision, compact=compact, parts=parts) as e, \
            Engine(games=4, sims=1, blocks=3, precision=precision) as ev:
        e.load_weights(w)
        ev.load_weights(w)
        r = e.search(roots)

        def cb(ctx, sp, pol, val):
            s = np.frombuffer(C.string_at(sp, 24), dtype=_abi.STATE_DTYPE).copy()
            p, v = ev.nn_forward(s)
            C.memmove(pol, p.ctypes.data, 200)
            val[0] = float(v[0])

        for g in range(len(roots)):
            cfg = orc.search_cfg(sims=sims, c_puct=5.0, evaluator=orc.EVAL_CALLBACK, fn=cb)
            mv, pi, nodes, _ = orc.search(cfg, roots[g])
            _compare_trees(e, g, nodes)
            assert _mv(r.moves[g]) == _mv(mv)


@pytest.mark.parametrize("evaluator", [_abi.EVAL_HASH, _abi.EVAL_NN, "nn_overflow"])
@pytest.mark.parametrize("games,sims,noise", [(1, 400, 0), (5, 60, 0), (256, 60, 0), (5, 60, 1), (300, 40, 0),
                                              (1000, 40, 1)])
def test_one_launch_search_equals_step_launches(orc, trained3, evaluator, games, sims, noise):
    """oaz_config.step_kernels 0 (auto) vs 1 (the per-simulation launches). Auto runs a search of <= CU-count
    games without root noise as ONE launch (k_search_lat: a workgroup per game runs all its simulations
    with the top of its tree in LDS), and otherwise up to 16 x CU-count games as one launch per noise
    chunk (k_search_grp: 16 games per workgroup). Every tree node, pi, move and search statistic is
    identical — also past the LDS-held nodes (400 simulations: ~5k nodes), with root noise, and when every
    evaluation leaves the fp16 range (nn_overflow: the in-kernel recompute, which moves k_search_lat's tree
    state out of LDS and back); with HASH both equal the oracle's trees (mcts_arena.rs:75-177)."""
    roots = random_positions(orc, games, seed=707 + games)
    w = random_weights(5, 3)
    if evaluator == "nn_overflow":
        from onitama_az.weights import blob_from_named, named_from_blob
        named = {k: v.copy() for k, v in named_from_blob(trained3.copy(), 3).items()}
        named["bn1|bias"][:] = 1.0e5
        w = blob_from_named(named, 3)
    ev = _abi.EVAL_HASH if evaluator == _abi.EVAL_HASH else _abi.EVAL_NN
    out = {}
    for sk in (0, 1):
        with Engine(games=games, sims=sims, c_puct=5.0, train_noise=noise, evaluator=ev, blocks=3,
                    precision=_abi.FP32_SPLIT16, step_kernels=sk, seed=99) as e:
            if ev == _abi.EVAL_NN:
                e.load_weights(w)
            e.set_timing(1)
            r = e.search(roots, root_value=True)
            kt = e.kernel_times()
            trees = [e.tree(g) for g in sorted({0, games // 2, games - 1})]
            out[sk] = (r, trees, kt)
            if evaluator == "nn_overflow":
                # every evaluation recomputed (the counter counts recomputed tiles: one position per workgroup in
                # k_nn_h3s / k_search_lat, up to 16 in k_search_grp and k_nn_h3)
                assert e.nn_fallbacks() >= (games + 15) // 16 * sims
    (r0, t0, k0), (r1, t1, k1) = out[0], out[1]
    if games <= 256 and not noise:  # k_search_lat: one launch (+ the root value's evaluation)
        assert (k0.backup_select_n, k0.nn_n, k0.select_n, k0.expand_n) == (1, 1, 0, 0)
    else:  # k_search_grp: one launch per noise chunk (up to 512 simulations), then the last expand / backup
        assert (k0.backup_select_n, k0.nn_n, k0.select_n, k0.expand_n) == (grp_launches(sims), 1, 0, 1)
    assert k1.select_n == k1.parts and k1.backup_select_n == (sims - 1) * k1.parts
    assert np.array_equal(r0.pi, r1.pi) and r0.moves.tobytes() == r1.moves.tobytes()
    assert np.array_equal(r0.root_value, r1.root_value)
    for f in ("sims", "expansions", "children", "terminal_leaves", "depth_sum", "stuck_leaves", "max_nodes", "nn_evals"):
        assert getattr(r0.stats, f) == getattr(r1.stats, f), f
    for a, b in zip(t0, t1):
        assert a.tobytes() == b.tobytes()
    if games == 1 and sims == 400:
        assert r0.stats.max_nodes > 3000  # past the LDS-held top of the tree
    if evaluator == _abi.EVAL_HASH and not noise:
        for g in sorted({0, games // 2, games - 1})[:2]:
            mv, pi, nodes, _ = orc.search(orc.search_cfg(sims=sims, c_puct=5.0, evaluator=orc.EVAL_HASH), roots[g])
            assert np.array_equal(r0.pi[g].reshape(-1), pi.reshape(-1)) and _mv(r0.moves[g]) == _mv(mv)


def test_search_with_root_noise_is_deterministic_and_consistent(orc):
    roots = random_positions(orc, 16, seed=707)
    kw = dict(games=16, sims=64, c_puct=5.0, train_noise=1, evaluator=_abi.EVAL_HASH, blocks=0, seed=99)
    with Engine(**kw) as e:
        r1 = e.search(roots)
        t1 = [e.tree(g) for g in range(16)]
    with Engine(**kw) as e:
        r2 = e.search(roots)
        t2 = [e.tree(g) for g in range(16)]
    assert np.array_equal(r1.pi, r2.pi) and r1.moves.tobytes() == r2.moves.tobytes()
    differs = 0
    for g in range(16):
        assert t1[g].tobytes() == t2[g].tobytes()
        root = t1[g][0]
        if root["nch"]:
            ch = t1[g][int(root["first"]): int(root["first"]) + int(root["nch"])]
            assert int(ch["N"].sum()) == 63  # first playout evaluates the root itself
        cfg = orc.search_cfg(sims=64, c_puct=5.0, evaluator=orc.EVAL_HASH)
        _, _, nodes, _ = orc.search(cfg, roots[g])
        differs += int(len(nodes) != len(t1[g]) or not np.array_equal(nodes["N"], t1[g]["N"]))
    assert differs > 0  # the noise changes the search


def test_search_no_legal_move_root_passes(orc, kats):
    """state.rs:852-889: Blue has no legal move. The reference's AZ search panics ("Must find the
    best child"); the engine returns a pass with the mover's first card and pi = 0 (Q6)."""
    case = [c for c in kats["movegen"] if "no_legal_moves_at_all" in c["src"]][0]
    root = kat_state(case["state"], 1)
    with Engine(games=1, sims=20, c_puct=5.0, train_noise=0, evaluator=_abi.EVAL_HASH, blocks=0) as e:
        r = e.search(root)
        t = e.tree(0)
    assert _mv(r.moves[0]) == (25, 25, 0, 2) and np.all(r.pi == 0)
    mv, pi, nodes, st = orc.search(orc.search_cfg(sims=20, c_puct=5.0, evaluator=orc.EVAL_HASH), root)
    assert _mv(mv) == (25, 25, 0, 2) and st.stuck_leaves == 19
    assert r.stats.stuck_leaves == 19 and t.tobytes() == nodes.tobytes()


def test_search_stuck_leaves_inside_tree_match_oracle(orc, kats):
    """Red to move in the no-move KAT position: Red moves that leave Blue without a move create
    expanded-but-childless nodes inside the tree (Q6); both searches must treat them alike."""
    case = [c for c in kats["movegen"] if "no_legal_moves_at_all" in c["src"]][0]
    root = kat_state(case["state"], 0)
    with Engine(games=1, sims=300, c_puct=5.0, train_noise=0, evaluator=_abi.EVAL_HASH, blocks=0) as e:
        r = e.search(root)
        mv, pi, nodes, st = orc.search(orc.search_cfg(sims=300, c_puct=5.0, evaluator=orc.EVAL_HASH), root)
        _compare_trees(e, 0, nodes)
    assert r.stats.stuck_leaves == st.stuck_leaves


@pytest.mark.parametrize("sims", [1, 2, 3])
def test_search_tiny_budgets(orc, sims):
    roots = random_positions(orc, 5, seed=808)
    with Engine(games=5, sims=sims, c_puct=5.0, train_noise=0, evaluator=_abi.EVAL_HASH, blocks=0) as e:
        r = e.search(roots)
        for g in range(5):
            mv, pi, nodes, _ = orc.search(orc.search_cfg(sims=sims, c_puct=5.0, evaluator=orc.EVAL_HASH), roots[g])
            _compare_trees(e, g, nodes)
            assert _mv(r.moves[g]) == _mv(mv) and np.array_equal(r.pi[g].reshape(-1), pi.reshape(-1))


def test_empty_and_single_inputs(orc):
    empty = np.zeros(0, dtype=_abi.STATE_DTYPE)
    moves, counts = movegen_batch(empty)
    assert moves.shape == (0, 40) and counts.shape == (0,)
    one = random_positions(orc, 1, seed=909)
    with Engine(games=4, sims=10, c_puct=5.0, train_noise=0, evaluator=_abi.EVAL_HASH, blocks=0) as e:
        assert len(e.search(empty).moves) == 0
        r = e.search(one)
        mv, _, _, _ = orc.search(orc.search_cfg(sims=10, c_puct=5.0, evaluator=orc.EVAL_HASH), one[0])
        assert _mv(r.moves[0]) == _mv(mv)
        with pytest.raises(_abi.OazError):
            e.search(np.concatenate([one] * 5))  # more roots than game slots


def test_search_root_noise_matches_oracle(orc):
    """Noise on: both sides draw the same Philox streams and run the same f64 log-domain
    Beta algorithm (Johnk) with polynomial log/exp by explicit fused multiply-adds (no libm), so the
    draws and the trees are bit-identical."""
    roots = random_positions(orc, 24, seed=1010)
    sims = 48
    with Engine(games=24, sims=sims, c_puct=5.0, train_noise=1, evaluator=_abi.EVAL_HASH, blocks=0, seed=77) as e:
        e.search(roots)
        same = 0
        for g in range(24):
            cfg = orc.search_cfg(sims=sims, c_puct=5.0, evaluator=orc.EVAL_HASH, train_noise=1, seed=77, game_id=g, ply=0)
            _, _, nodes, _ = orc.search(cfg, roots[g])
            t = e.tree(g)
            same += int(len(t) == len(nodes) and t.tobytes() == nodes.tobytes())
    assert same == 24, same


def _wide_roots(orc, n, seed):
    """Seeded positions whose mover has more than 32 legal moves (placed pieces, random cards): random play
    never reached one in 1 200 positions (max 26), so these are built to reach the workgroup fold's second
    pass (children 32 .. K - 1)."""
    import random
    rng = random.Random(seed)
    base = random_positions(orc, 1, seed=1)
    bit = lambda q: 1 << (31 - q)
    out = []
    while len(out) < n:
        color = rng.randint(0, 1)
        sq = rng.sample(range(25), 10)
        mine, opp = sq[:5], sq[5:5 + rng.randint(1, 5)]
        s = base.copy()
        k, p = [0, 0], [0, 0]
        k[color], p[color] = bit(mine[0]), sum(bit(q) for q in mine[1:])
        k[1 - color], p[1 - color] = bit(opp[0]), sum(bit(q) for q in opp[1:])
        s["kings"][0], s["pawns"][0] = k, p
        s["cards"][0] = rng.sample(range(16), 5)
        s["to_move"][0] = color
        if len(orc.movegen(s)) > 32:
            out.append(s)
    return np.concatenate(out)


@pytest.mark.parametrize("step_kernels", [0, 1])
def test_search_root_noise_wide_roots_match_oracle(orc, step_kernels):
    """Roots with 33-40 children and root noise: the per-step kernels' workgroup fold stages 32 children
    per pass, so a workgroup holding such a root folds its games in two passes (workgroup 0 mixes 3 wide
    roots with ordinary ones, workgroup 1 is all wide roots); step_kernels 0 is the one-launch search's
    per-segment fold over three chunks. Every tree equals the oracle's node for node."""
    roots = random_positions(orc, 64, seed=2024)
    wide = _wide_roots(orc, 35, seed=31)
    for slot, w in zip((3, 17, 30), wide[:3]):
        roots[slot] = w
    roots[32:] = wide[3:35]
    sims = 40
    with Engine(games=64, sims=sims, c_puct=5.0, train_noise=1, evaluator=_abi.EVAL_HASH, blocks=0, seed=91,
                step_kernels=step_kernels) as e:
        e.search(roots)
        bad = []
        for g in range(64):
            cfg = orc.search_cfg(sims=sims, c_puct=5.0, evaluator=orc.EVAL_HASH, train_noise=1, seed=91, game_id=g, ply=0)
            _, _, nodes, _ = orc.search(cfg, roots[g])
            t = e.tree(g)
            if not (len(t) == len(nodes) and t.tobytes() == nodes.tobytes()):
                bad.append(g)
    assert not bad, bad
    assert all(len(orc.movegen(roots[g:g + 1])) > 32 for g in (3, 17, 30, 32, 63))


def test_search_finds_win_in_one(kats):
    case = kats["tactics"][0]  # onitama-game/src/ai/mcts/mcts_arena.rs:459-483
    root = kat_state(case["state"], case["color"])
    for ev in (_abi.EVAL_HASH, _abi.EVAL_NN):
        with Engine(games=1, sims=400, c_puct=5.0, train_noise=0, evaluator=ev, blocks=3) as e:
            r = e.search(root)
        assert _mv(r.moves[0]) == tuple(case["expected"])


def test_search_large_batch_stats():
    from onitama_az.game import initial_state_np
    G = 4096
    roots = np.concatenate([initial_state_np([0, 1, 2, 3, 4])] * G)
    with Engine(games=G, sims=8, c_puct=5.0, train_noise=1, evaluator=_abi.EVAL_NN, blocks=3) as e:
        r = e.search(roots, root_value=True)
    assert r.stats.sims == 8 * G and r.stats.expansions >= G
    assert np.allclose(r.pi.reshape(G, -1).sum(1), 1.0, atol=1e-6)
    assert np.all(np.abs(r.root_value) <= 1.0)


# ---- self-play ---------------------------------------------------------------------------
def _sorted_rows(a):
    return np.sort(np.frombuffer(a.tobytes(), dtype=np.dtype((np.void, a.dtype.itemsize))))


@pytest.mark.parametrize("fixed,max_plies,compact,parts", [(True, 150, 0, 1), (False, 150, 0, 1), (False, 3, 0, 1),
                                                           (True, 150, 1, 2), (False, 150, 1, 4), (False, 3, 0, 2),
                                                           (False, 150, 1, 5)])
def test_selfplay_matches_oracle_games(orc, fixed, max_plies, compact, parts):
    n_games, slots, sims = 24, 8, 12
    if parts == 5:  # 5 slots in 4 parts (the fourth would be empty: runs as 3 + 2)
        slots, parts = 5, 4
    deck = [0, 1, 2, 3, 4]
    kw = dict(games=slots, sims=sims, c_puct=5.0, train_noise=0, evaluator=_abi.EVAL_HASH, blocks=0,
              max_plies=max_plies, seed=4242, fixed_deck=int(fixed), deck=deck, compact=compact, parts=parts)
    with Engine(**kw) as e:
        got, st = e.selfplay_run(n_games, cap=n_games * (max_plies + 2))
    assert st.games_finished == n_games
    ref = []
    for gid in range(n_games):
        cfg = orc.search_cfg(sims=sims, c_puct=5.0, evaluator=orc.EVAL_HASH, seed=4242)
        s, res, plies, _ = orc.selfplay_game(cfg, gid, max_plies=max_plies, deck=deck if fixed else None)
        assert plies <= max_plies + 2
        ref.append(s)
    ref = np.concatenate(ref)
    assert len(got) == len(ref)
    assert np.array_equal(_sorted_rows(got), _sorted_rows(ref))


@pytest.mark.parametrize("precision,blocks", [(_abi.FP32, 3), (_abi.FP32_SPLIT, 3), (_abi.FP32_SPLIT16, 3),
                                              (_abi.BF16, 6)])
def test_selfplay_nn_continuous_batching_runs(precision, blocks):
    # compaction forced: every NN kernel of the product build runs on bucket tile maps
    with Engine(games=256, sims=16, c_puct=5.0, train_noise=1, evaluator=_abi.EVAL_NN, blocks=blocks, max_plies=150,
                precision=precision, fixed_deck=0, compact=1) as e:
        e.selfplay_reset()
        e.selfplay_step(40)
        st = e.selfplay_stats()
        samples = e.samples_fetch(100000)
    assert st.moves == 40 * 256 - 0 or st.moves <= 40 * 256
    assert st.games_finished > 0 and len(samples) == st.samples_ready
    assert np.all(np.isin(samples["z"], [-1.0, 0.0, 1.0]))
    assert np.allclose(samples["pi"].sum(1), 1.0, atol=1e-6)


def test_selfplay_stagger_delays_slots():
    G, S = 64, 4
    with Engine(games=G, sims=4, c_puct=5.0, train_noise=0, evaluator=_abi.EVAL_HASH, blocks=0, stagger=S) as e:
        e.selfplay_reset()
        e.selfplay_step(6)
        st = e.selfplay_stats()
    # slot g plays 6 - (g % S) plies
    assert st.moves == sum(6 - (g % S) for g in range(G))


# ---- Agent / self-play API mirror ----------------------------------------------------------
def test_agent_api_mirror(orc):
    from onitama_az.mcts import AlphaZeroMcts, AlphaZeroMctsConfig, ConvResNet, ConvResNetConfig, TrainingAlphaZeroMcts
    from onitama_az.selfplay import TrainConfig, self_play
    from onitama_az.mcts import Options
    model = ConvResNet(ConvResNetConfig(resnet_block_amnt=3), seed=0)
    cfg = AlphaZeroMctsConfig(exploration_c=5.0, max_playouts=50, train=False)
    agent = AlphaZeroMcts(cfg, model)
    gs = GameState.with_deck(Deck([ORIGINAL_CARDS[i] for i in range(5)]))
    mv, value = agent.generate_move(gs)
    legal = gs.state.generate_all_legal_moves(gs.curr_player_color)
    assert (mv.used_card_idx, mv.mov) in legal and -1.0 <= value <= 1.0
    assert agent.name() == "AlphaZero MCTS AI"
    res = gs.progress(mv)
    assert res in (MoveResult.InProgress, MoveResult.Capture)
    tr = TrainingAlphaZeroMcts(cfg, model)
    mv2, pi = tr.generate_move_tensor(gs.state, gs.curr_player_color)
    assert pi.shape == (2, 25) and abs(pi.sum() - 1) < 1e-6
    data = self_play(tr, Options(), None, TrainConfig(mcts_config=cfg, self_play_game_amnt=3,
                                                       model_config=ConvResNetConfig(resnet_block_amnt=3)))
    assert len(data) > 0 and data[0].state.shape == (21, 5, 5)
    for d in data[:20]:
        assert d.z in (-1.0, 0.0, 1.0) and d.pi.shape == (2, 25)


def test_legacy_one_game_per_wave_tree_kernels_match_oracle(tmp_path):
    """OAZ_TREE_SEG=0 selects the one-game-per-wave k_select / k_expand_backup (the default runs four
    games per wave) in the A/B build (libonitama_az_ab.so, built by __graft_entry__.build(); the product
    library reads no environment switch). The switch is read once per process, so the check runs in a
    child process: noise-on searches whose trees must equal the oracle's node for node, as the default
    path's."""
    import subprocess
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parents[1]
    code = f"""
import sys
sys.path.insert(0, {str(root / 'onitama-alphazero_amd')!r}); sys.path.insert(0, {str(root / 'tests')!r})
import numpy as np
import oracle_ffi as orc
from conftest import random_positions
from onitama_az import _abi
from onitama_az.engine import Engine
orc.load()
roots = random_positions(orc, 10, seed=4242)
with Engine(games=10, sims=40, c_puct=5.0, train_noise=1, evaluator=_abi.EVAL_HASH, blocks=0, seed=31) as e:
    e.search(roots)
    for g in range(10):
        cfg = orc.search_cfg(sims=40, c_puct=5.0, evaluator=orc.EVAL_HASH, train_noise=1, seed=31, game_id=g, ply=0)
        _, _, nodes, _ = orc.search(cfg, roots[g])
        assert e.tree(g).tobytes() == nodes.tobytes(), g
print("legacy ok")
"""
    ab = root / "onitama-alphazero_amd" / "onitama_az" / "libonitama_az_ab.so"
    assert ab.exists(), "build() makes the A/B library"
    env = dict(__import__("os").environ, OAZ_TREE_SEG="0", OAZ_LIB=str(ab))
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and "legacy ok" in r.stdout, r.stdout + r.stderr


def test_set_search_params_per_agent_config(orc):
    """oaz_set_search_params: one engine (created for 64 sims, no noise) serves searches with other
    AlphaZeroMctsConfigs (32 sims, c = 2, noise on) exactly as an engine made for them would."""
    roots = random_positions(orc, 6, seed=1212)
    with Engine(games=6, sims=64, c_puct=5.0, train_noise=0, evaluator=_abi.EVAL_HASH, blocks=0, seed=5) as e:
        e.set_search_params(32, 2.0, True)
        r = e.search(roots)
        for g in range(6):
            cfg = orc.search_cfg(sims=32, c_puct=2.0, evaluator=orc.EVAL_HASH, train_noise=1, seed=5, game_id=g, ply=0)
            mv, pi, nodes, _ = orc.search(cfg, roots[g])
            _compare_trees(e, g, nodes)
            assert _mv(r.moves[g]) == _mv(mv)
        with pytest.raises(_abi.OazError):
            e.set_search_params(65, 2.0, False)  # beyond the creation budget


# ---- Q7: the wall-clock search budget (opt-in) -------------------------------------------------
@pytest.mark.parametrize("step_kernels", [0, 1])
def test_search_time_budget_stops_early_and_matches_oracle_at_that_budget(orc, step_kernels):
    """oaz_config.search_time_ns (mcts_arena.rs:78: `while playouts < max_playouts && elapsed <
    search_time`): a 25 ms budget on a 20 000-playout search stops early, and trees, pi and moves equal the
    oracle's search with the playouts each game ran. step_kernels 0: the one-launch search (k_search_lat)
    reads the device clock before every simulation, each game on its own, and stays ONE launch;
    1: the per-step loop stops every game after the same simulation step."""
    roots = random_positions(orc, 8, seed=1313)
    with Engine(games=8, sims=20000, c_puct=5.0, train_noise=0, evaluator=_abi.EVAL_HASH, blocks=0,
                parts=2, step_kernels=step_kernels) as e:
        e.set_timing(1)
        e.set_search_time(0.025)
        r = e.search(roots)
        k = e.kernel_times()
        n = e.search_playouts(8)
        assert np.all((n >= 1) & (n < 20000)), n
        assert e.last_sims() == int(n.max()) and r.stats.sims == int(n.sum())
        if step_kernels == 0:
            assert (k.backup_select_n, k.select_n, k.expand_n) == (1, 0, 0)  # one launch, no host round trip
        else:
            assert np.all(n == n[0])
        for g in range(8):
            mv, pi, nodes, _ = orc.search(orc.search_cfg(sims=int(n[g]), c_puct=5.0, evaluator=orc.EVAL_HASH), roots[g])
            _compare_trees(e, g, nodes)
            assert np.array_equal(r.pi[g].reshape(-1), pi.reshape(-1)) and _mv(r.moves[g]) == _mv(mv)
        e.set_search_time(0.0)  # off again: exactly `sims` playouts (the parity mode)
        e.set_search_params(64, 5.0, False)
        r = e.search(roots)
        assert e.last_sims() == 64 and r.stats.sims == 8 * 64
        assert np.array_equal(e.search_playouts(8), np.full(8, 64))


@pytest.mark.parametrize("step_kernels", [0, 1])
def test_search_time_budget_with_root_noise_then_full_search(orc, step_kernels):
    """Q7 with root noise: the budget stops the search wherever the clock says, usually inside a
    noise chunk whose successor's draws are already requested on the noise stream (step_kernels 0:
    k_search_grp checks the device clock before every simulation, its 16-game group stops together and
    the chunk launches after it exit at once; 1: the per-step loop). The trees equal the oracle's noisy
    search with the playouts that ran, and the engine's next search (ply 1, no budget, its noise ring
    restarted) equals the oracle's as well (mcts_arena.rs:75-81, 183-223)."""
    roots = random_positions(orc, 8, seed=1414)
    with Engine(games=8, sims=20000, c_puct=5.0, train_noise=1, evaluator=_abi.EVAL_HASH, blocks=0, seed=77,
                parts=2, step_kernels=step_kernels) as e:
        e.set_search_time(0.02)
        e.search(roots)
        n = e.search_playouts(8)
        assert np.all((n >= 1) & (n < 20000)) and np.all(n == n[0]), n  # one 16-game group / one step loop
        for g in range(8):
            cfg = orc.search_cfg(sims=int(n[g]), c_puct=5.0, evaluator=orc.EVAL_HASH, train_noise=1, seed=77,
                                 game_id=g, ply=0)
            _, _, nodes, _ = orc.search(cfg, roots[g])
            _compare_trees(e, g, nodes)
        e.set_search_time(0.0)
        e.set_search_params(48, 5.0, True)
        r = e.search(roots)
        assert e.last_sims() == 48 and r.stats.sims == 8 * 48
        for g in range(8):
            cfg = orc.search_cfg(sims=48, c_puct=5.0, evaluator=orc.EVAL_HASH, train_noise=1, seed=77, game_id=g, ply=1)
            mv, pi, nodes, _ = orc.search(cfg, roots[g])
            _compare_trees(e, g, nodes)
            assert np.array_equal(r.pi[g].reshape(-1), pi.reshape(-1)) and _mv(r.moves[g]) == _mv(mv)


def test_search_time_budget_groups_stop_independently(orc):
    """k_search_grp with a budget over several 16-game groups (40 games: three workgroups, the last one
    partial): each group stops on its own clock read, the games of one group share a count, and every tree
    equals the oracle's noisy search at its game's count."""
    roots = random_positions(orc, 40, seed=1616)
    with Engine(games=40, sims=20000, c_puct=5.0, train_noise=1, evaluator=_abi.EVAL_HASH, blocks=0, seed=78) as e:
        e.set_search_time(0.015)
        r = e.search(roots)
        n = e.search_playouts(40)
        assert np.all((n >= 1) & (n < 20000)), n
        for b in range(0, 40, 16):
            assert np.all(n[b: b + 16] == n[b]), n
        assert r.stats.sims == int(n.sum())
        for g in (0, 17, 39):
            cfg = orc.search_cfg(sims=int(n[g]), c_puct=5.0, evaluator=orc.EVAL_HASH, train_noise=1, seed=78,
                                 game_id=g, ply=0)
            mv, pi, nodes, _ = orc.search(cfg, roots[g])
            _compare_trees(e, g, nodes)
            assert np.array_equal(r.pi[g].reshape(-1), pi.reshape(-1)) and _mv(r.moves[g]) == _mv(mv)


def test_search_time_through_agent_config():
    """AlphaZeroMctsConfig applies search_time to the engine by default, as the reference always does
    (mcts_arena.rs:78); with enforce_search_time=False the search runs max_playouts exactly."""
    from onitama_az.mcts import AlphaZeroMcts, AlphaZeroMctsConfig, ConvResNet, ConvResNetConfig
    model = ConvResNet(ConvResNetConfig(resnet_block_amnt=3), seed=0)
    gs = GameState.with_deck(Deck([ORIGINAL_CARDS[i] for i in range(5)]))
    assert AlphaZeroMctsConfig().enforce_search_time  # the reference's semantics by default
    timed = AlphaZeroMcts(AlphaZeroMctsConfig(search_time=0.02, exploration_c=5.0, max_playouts=20000), model)
    mv, _ = timed.generate_move(gs)
    eng = model.__dict__["_search"]["engine"]
    assert 1 <= eng.last_sims() < 20000
    assert (mv.used_card_idx, mv.mov) in gs.state.generate_all_legal_moves(gs.curr_player_color)
    plain = AlphaZeroMcts(AlphaZeroMctsConfig(search_time=0.02, exploration_c=5.0, max_playouts=300,
                                              enforce_search_time=False), model)
    plain.generate_move(gs)
    assert eng.last_sims() == 300
