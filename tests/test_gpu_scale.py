"""GPU parity at the benchmarked sizes (BASELINE.json configs C2, C3, C5): the HIP path through
the C ABI at the launch shapes bench.py times, checked against the oracle (every game's pi and
move; full trees on a sample) and against the torch goldens.

  C3  65,536 games x 400 sims, fixed deck, root noise on      (HASH evaluator: bit-exact trees)
  C2  4,096 games x 100 sims, 3-block NN (fp16x3 split / fp32) (oracle fed the GPU network)
  C4  one rank's shard: rank 5 of 8, 65,536 self-play slots x 400 sims (HASH: trees + records)
  C5  65,536 games x 800 sims, 6-block bf16, 16-card deals     (properties + HASH trees)
  NN  B = 65,536 (4,096 workgroups) on the golden positions, every copy against the goldens

Reference semantics: mcts_arena.rs:75-177 (search, playout), train.rs:35-98 (self-play).
"""
import ctypes as C

import numpy as np
import pytest

from onitama_az import _abi
from onitama_az.engine import Engine
from onitama_az.game import initial_state_np, movegen_batch, step_batch
from onitama_az.weights import random_weights

pytestmark = pytest.mark.gpu

SEED = 20260101


def gpu_random_positions(n, seed, fixed_deck=True, max_plies=40):
    """n positions from seeded random play on the GPU rules (bit-exact with the oracle, test_gpu.py):
    game i is dealt (fixed deck or seeded 16-card deal) and plays a random number of plies in
    [0, max_plies], stopping at a win or a position without moves. The batched generator of the
    bench-size roots (the oracle's Python driver would take minutes at 65,536)."""
    rng = np.random.default_rng(seed)
    lib = _abi.load()
    if fixed_deck:
        s = np.concatenate([initial_state_np([0, 1, 2, 3, 4])] * n)
    else:
        decks = np.zeros((n, 5), dtype=np.uint8)
        d = (C.c_uint8 * 5)()
        for i in range(n):
            lib.oaz_deal_deck(C.c_uint64(seed), C.c_uint64(i), d)
            decks[i] = list(d)
        s = np.concatenate([initial_state_np(decks[i]) for i in range(n)])
    target = rng.integers(0, max_plies + 1, n)
    alive = np.ones(n, dtype=bool)
    for ply in range(max_plies):
        idx = np.nonzero(alive & (target > ply))[0]
        if len(idx) == 0:
            break
        sub = np.ascontiguousarray(s[idx])
        moves, counts = movegen_batch(sub)
        has = counts > 0
        alive[idx[~has]] = False
        idx, sub, moves, counts = idx[has], np.ascontiguousarray(sub[has]), moves[has], counts[has]
        pick = moves[np.arange(len(idx)), (rng.random(len(idx)) * counts).astype(np.int64)]
        res = step_batch(sub, pick)
        s[idx] = sub
        alive[idx[(res == _abi.RED_WIN) | (res == _abi.BLUE_WIN)]] = False
    return s


def _mv(m):
    return tuple(int(m[k]) for k in ("from_", "to", "piece", "slot"))


def _compare_trees(e, g, nodes_ref):
    t = e.tree(g)
    assert len(t) == len(nodes_ref), (g, len(t), len(nodes_ref))
    for f in ("W", "P", "N", "mv", "nch", "flags"):
        assert np.array_equal(t[f], nodes_ref[f]), (g, f)
    exp = (t["flags"] & 1) != 0
    assert np.array_equal(t["first"][exp], nodes_ref["first"][exp]), g


def _legal(roots, moves):
    """Every chosen move is one of the root's legal moves (or the pass when there is none)."""
    lm, counts = movegen_batch(roots)
    for i in range(len(roots)):
        k = int(counts[i])
        if k == 0:
            assert int(moves[i]["from_"]) == 25, i
        else:
            assert moves[i].tobytes() in {lm[i, j].tobytes() for j in range(k)}, i


# ---- NN at the C3 / C5 launch shape --------------------------------------------------------------
@pytest.mark.parametrize("precision,name,blocks,tol", [
    (_abi.FP32_SPLIT16, "trained3", 3, 1e-5), (_abi.FP32, "trained3", 3, 1e-4), (_abi.FP32_SPLIT, "trained3", 3, 1e-4),
    (_abi.BF16, "random6", 6, 3e-2)])
def test_nn_launch_shape_vs_goldens(nn_golden, trained3, precision, name, blocks, tol):
    """oaz_nn_forward at B = 65,536 (4,096 workgroups: the C3/C5 launch): the 256 golden positions
    tiled 256 times. Every copy within the tolerance of the torch goldens, and every copy of a
    position bit-identical to the others (results independent of the workgroup/XCD a tile lands on)."""
    w = trained3 if name == "trained3" else random_weights(1, 6)
    B = 65536
    states = np.tile(nn_golden["states"], B // 256)
    with Engine(games=B, sims=1, blocks=blocks, evaluator=_abi.EVAL_NN, precision=precision) as e:
        e.load_weights(w)
        p, v = e.nn_forward(states)
        assert e.nn_fallbacks() == 0
    p = p.reshape(B // 256, 256, 50)
    v = v.reshape(B // 256, 256)
    gp, gv = nn_golden[f"policy_{name}"].reshape(256, 50), nn_golden[f"value_{name}"]
    assert np.abs(p - gp[None]).max() < tol
    assert np.abs(v - gv[None]).max() < tol
    assert (p == p[:1]).all() and (v == v[:1]).all()


# ---- C3 ----------------------------------------------------------------------------------------
@pytest.mark.timeout(600)
def test_c3_search_every_game_vs_oracle(orc):
    """C3 shape: 65,536 roots (fixed deck [Tiger, Dragon, Frog, Rabbit, Crab], positions after 0-40
    random plies), 400 simulations, Dirichlet root noise on, the HASH evaluator (every value exact in
    fp32, so the trees are comparable bit for bit). Every game's pi and move equal the oracle's
    (root g keyed as game g, ply 0, as the engine's search mode does), 64 sampled trees equal node for
    node, and the run's statistics are consistent (sims, tree capacity)."""
    G, sims = 65536, 400
    roots = gpu_random_positions(G, seed=303)
    # leaf compaction on (compact=2: at 65 536 games it removes NN rounds), the C5 test runs it off
    with Engine(games=G, sims=sims, c_puct=5.0, train_noise=1, evaluator=_abi.EVAL_HASH, blocks=0, seed=SEED,
                compact=2) as e:
        r = e.search(roots)
        assert r.stats.sims == sims * G
        assert r.stats.max_nodes <= 1 + 40 * sims
        cfg = orc.search_cfg(sims=sims, c_puct=5.0, evaluator=orc.EVAL_HASH, train_noise=1, seed=SEED, game_id=0, ply=0)
        mv, pi, st = orc.search_batch(cfg, roots)
        assert np.array_equal(r.pi.reshape(G, 50), pi.reshape(G, 50))
        assert r.moves.tobytes() == mv.tobytes()
        assert (st.sims, st.expansions, st.children, st.depth_sum, st.max_nodes, st.nn_evals) == (
            r.stats.sims, r.stats.expansions, r.stats.children, r.stats.depth_sum, r.stats.max_nodes,
            r.stats.nn_evals)
        assert 0 < r.stats.nn_evals < r.stats.sims  # won leaves are left out of the NN batch
        sample = np.unique(np.concatenate([[0, G - 1], np.random.default_rng(3).integers(0, G, 62)]))
        for g in sample:
            c = orc.search_cfg(sims=sims, c_puct=5.0, evaluator=orc.EVAL_HASH, train_noise=1, seed=SEED,
                               game_id=int(g), ply=0)
            _, _, nodes, _ = orc.search(c, roots[g])
            _compare_trees(e, int(g), nodes)


@pytest.mark.timeout(300)
def test_c3_selfplay_full_shape_is_valid():
    """bench.py's C3 run (65,536 slots x 400 sims, 3-block fp16x3 split NN, noise on, staggered
    starts) for 14 plies: no sample dropped, trees within capacity, every finished game's samples
    well formed, no fp16-range fallback on random-init weights."""
    G, sims = 65536, 400
    with Engine(games=G, sims=sims, blocks=3, c_puct=5.0, train_noise=1, max_plies=150, evaluator=_abi.EVAL_NN,
                precision=_abi.FP32_SPLIT16, fixed_deck=1, deck=[0, 1, 2, 3, 4], seed=SEED, stagger=12,
                sample_capacity=G * 16) as e:
        e.load_weights(random_weights(0, 3))
        e.selfplay_reset()
        e.selfplay_step(14)
        st = e.selfplay_stats()
        smp = e.samples_fetch(int(st.samples_ready))
        fb = e.nn_fallbacks()
    assert st.samples_dropped == 0 and st.search.max_nodes <= 1 + 40 * sims
    assert st.moves == sum(14 - (g % 12) for g in range(G))  # stagger: slot g waits g % 12 plies
    assert st.search.sims == st.moves * sims
    assert fb == 0
    assert len(smp) == st.samples_ready
    assert np.all(np.isin(smp["z"], [-1.0, 0.0, 1.0]))
    s = smp["pi"].sum(1)
    assert np.all(np.isclose(s, 1.0, atol=1e-5) | (s == 0))  # 0: a pass position (no legal move)


# ---- C4 (one rank's shard) ----------------------------------------------------------------------
@pytest.mark.timeout(600)
def test_c4_rank5_of_8_shard_vs_oracle(orc):
    """C4's per-rank workload on one GPU: the self-play shard of rank 5 of 8 (65,536 slots, 400
    simulations, fixed deck, root noise on, HASH evaluator so trees compare bit for bit). Every slot
    plays global game id (seq * 8 + 5) * 65,536 + slot (oaz_slot_game_ids; the deal and the noise are
    keyed by it, train.rs:218-238 gives each worker its own games). max_plies = 0 cuts every game after
    two plies (train.rs:74-79), so after ply 1 every slot has emitted its two (s, pi, z) records.
    Checked against the oracle's games under the same global ids: 64 sampled slots' ply-0 and ply-1
    trees node for node (oaz_tree_dump after each ply) and pi, their records (state, pi, z = 0) byte-equal
    at the slot-order positions; the same slots' trees under rank 0's ids differ (another game's noise)."""
    from onitama_az.dist import global_game_ids
    G, sims, W, R = 65536, 400, 8, 5
    deck = [0, 1, 2, 3, 4]
    gids = global_game_ids(R, W, G, 0)
    assert int(gids[0]) == 5 * G
    sample = np.unique(np.concatenate([[0, G - 1], np.random.default_rng(45).integers(0, G, 62)]))
    cfg = lambda gid, ply=0: orc.search_cfg(sims=sims, c_puct=5.0, evaluator=orc.EVAL_HASH, train_noise=1,
                                            seed=SEED, game_id=int(gid), ply=ply)
    ref = {int(g): orc.selfplay_game(cfg(gids[g]), int(gids[g]), max_plies=0, deck=deck)[0] for g in sample}
    with Engine(games=G, sims=sims, c_puct=5.0, train_noise=1, evaluator=_abi.EVAL_HASH, blocks=0, seed=SEED,
                fixed_deck=1, deck=deck, rank=R, world=W, max_plies=0, sample_capacity=2 * G) as e:
        e.selfplay_reset()
        for ply in (0, 1):
            e.selfplay_step(1)
            for g in sample:
                root = np.ascontiguousarray(ref[int(g)][ply]["state"]).reshape(1)
                _, pi, nodes, _ = orc.search(cfg(gids[g], ply), root)
                _compare_trees(e, int(g), nodes)
                assert np.array_equal(pi.reshape(-1), ref[int(g)][ply]["pi"].reshape(-1))
        # the same slots under rank 0's ids are other games (other noise): their ply-1 trees differ
        differ = 0
        for g in sample[:8]:
            root = np.ascontiguousarray(ref[int(g)][1]["state"]).reshape(1)
            _, _, nodes, _ = orc.search(cfg(g, 1), root)
            t = e.tree(int(g))
            differ += int(len(t) != len(nodes) or not np.array_equal(t["N"], nodes["N"]))
        assert differ >= 6, differ
        st = e.selfplay_stats()
        assert (st.moves, st.games_finished, st.games_cut, st.samples_ready, st.samples_dropped) == (2 * G, G, G, 2 * G, 0)
        assert st.search.sims == 2 * G * sims
        smp = e.samples_fetch(2 * G)
    # every game ended in ply 1, and a ply's finished games append their records in slot order: slot g's two
    # records (state, pi, z = 0) are records 2g and 2g + 1, byte-equal to the oracle's game
    for g in sample:
        assert len(ref[int(g)]) == 2 and np.all(ref[int(g)]["z"] == 0.0)
        assert smp[2 * g: 2 * g + 2].tobytes() == ref[int(g)].tobytes(), g


# ---- C2 ----------------------------------------------------------------------------------------
@pytest.mark.timeout(600)
@pytest.mark.parametrize("precision", [_abi.FP32_SPLIT16, _abi.FP32])
def test_c2_search_nn_sampled_trees_vs_oracle(orc, precision):
    """C2 shape: 4,096 roots x 100 simulations, 3-block NN (random init, seed 0), noise on. 16
    sampled games are re-searched by the oracle fed the GPU network's outputs (batch-1 calls of the
    same batch-independent kernel) and must agree node for node; all 4,096 moves are legal and every
    pi is a distribution over the root's children."""
    G, sims = 4096, 100
    roots = gpu_random_positions(G, seed=202)
    w = random_weights(0, 3)
    with Engine(games=G, sims=sims, c_puct=5.0, train_noise=1, evaluator=_abi.EVAL_NN, blocks=3, precision=precision,
                seed=SEED) as e, Engine(games=4, sims=1, blocks=3, precision=precision) as ev:
        e.load_weights(w)
        ev.load_weights(w)
        r = e.search(roots, root_value=True)
        assert r.stats.sims == sims * G and r.stats.max_nodes <= 1 + 40 * sims
        _legal(roots, r.moves)
        s = r.pi.reshape(G, 50).sum(1)
        assert np.all(np.isclose(s, 1.0, atol=1e-5) | (s == 0))
        assert np.all(np.abs(r.root_value) <= 1.0)

        def cb(ctx, sp, pol, val):
            st = np.frombuffer(C.string_at(sp, 24), dtype=_abi.STATE_DTYPE).copy()
            p, v = ev.nn_forward(st)
            C.memmove(pol, p.ctypes.data, 200)
            val[0] = float(v[0])

        for g in np.random.default_rng(7).choice(G, 16, replace=False):
            c = orc.search_cfg(sims=sims, c_puct=5.0, evaluator=orc.EVAL_CALLBACK, fn=cb, train_noise=1, seed=SEED,
                               game_id=int(g), ply=0)
            mv, pi, nodes, _ = orc.search(c, roots[g])
            _compare_trees(e, int(g), nodes)
            assert _mv(r.moves[g]) == _mv(mv) and np.array_equal(r.pi[g].reshape(-1), pi.reshape(-1))
        assert e.nn_fallbacks() == 0


# ---- C5 ----------------------------------------------------------------------------------------
@pytest.mark.timeout(600)
def test_c5_bf16_search_full_shape_properties():
    """C5 shape on one GPU: 65,536 roots from random 16-card deals, 800 simulations, 6-block bf16
    network, noise on: exactly 800 NN evaluations per game, trees within capacity, legal moves,
    pi a distribution over the children, root values in [-1, 1]."""
    G, sims = 65536, 800
    roots = gpu_random_positions(G, seed=505, fixed_deck=False)
    with Engine(games=G, sims=sims, blocks=6, c_puct=5.0, train_noise=1, evaluator=_abi.EVAL_NN,
                precision=_abi.BF16, fixed_deck=0, seed=SEED) as e:
        e.load_weights(random_weights(0, 6))
        r = e.search(roots, root_value=True)
    assert r.stats.sims == sims * G and r.stats.max_nodes <= 1 + 40 * sims
    _legal(roots, r.moves)
    s = r.pi.reshape(G, 50).sum(1)
    assert np.all(np.isclose(s, 1.0, atol=1e-5) | (s == 0))
    assert np.all(np.abs(r.root_value) <= 1.0) and np.isfinite(r.root_value).all()


@pytest.mark.timeout(600)
def test_c5_search_hash_trees_vs_oracle(orc):
    """C5 tree shape (800 simulations, 16-card deals, noise on) with the HASH evaluator at the full
    65,536-game launch: 4,096 strided games' pi and moves equal the oracle's, 32 trees node for node."""
    G, sims = 65536, 800
    roots = gpu_random_positions(G, seed=606, fixed_deck=False)
    with Engine(games=G, sims=sims, c_puct=5.0, train_noise=1, evaluator=_abi.EVAL_HASH, blocks=0, seed=SEED,
                fixed_deck=0) as e:
        r = e.search(roots)
        assert r.stats.max_nodes <= 1 + 40 * sims
        sub = np.arange(0, G, 16)  # 4,096 strided games, each keyed by its own batch index
        c = orc.search_cfg(sims=sims, c_puct=5.0, evaluator=orc.EVAL_HASH, train_noise=1, seed=SEED, ply=0)
        mv, pi, _ = orc.search_batch(c, roots[sub], game_ids=sub)
        assert np.array_equal(r.pi[sub], pi) and r.moves[sub].tobytes() == mv.tobytes()
        for g in np.random.default_rng(11).choice(G, 32, replace=False):
            c = orc.search_cfg(sims=sims, c_puct=5.0, evaluator=orc.EVAL_HASH, train_noise=1, seed=SEED,
                               game_id=int(g), ply=0)
            _, _, nodes, _ = orc.search(c, roots[g])
            _compare_trees(e, int(g), nodes)
