"""The reference Agent's default configuration on the GPU (alphazero_mcts/mod.rs:34-43: search_time 400 ms,
max_playouts 5 000, c = sqrt(2)), through the one-launch searches the drop-in takes.

- 5 000 simulations run past k_search_lat's LDS-held path and sqrt(N) table (2 048 entries each,
  csrc/oaz_search_lat.hip), so its global-memory fallbacks execute on every simulation;
- with root noise the search is k_search_grp, 10 launches (512-simulation noise chunks);
- with a search_time budget the one-launch kernels read the device clock before every simulation
  (mcts_arena.rs:75-81) and the trees equal the oracle's search at the playouts each game ran.

Trees are compared node for node against the C oracle: with the HASH test evaluator, and with the real
network by feeding the oracle's search the GPU network's outputs (batch-1 calls of the same kernel).
"""
import ctypes as C
import math

import numpy as np
import pytest

from conftest import random_positions
from onitama_az import _abi
from onitama_az.engine import Engine
from onitama_az.weights import random_weights

pytestmark = pytest.mark.gpu

AGENT_PLAYOUTS = 5000        # AlphaZeroMctsConfig::default().max_playouts (mod.rs:34-43)
AGENT_TIME_S = 0.4           # AlphaZeroMctsConfig::default().search_time
AGENT_C = math.sqrt(2.0)     # AlphaZeroMctsConfig::default().exploration_c
NODE_FIELDS = ("W", "P", "N", "first", "mv", "nch", "flags")


def _mv(m):
    return tuple(int(m[k]) for k in ("from_", "to", "piece", "slot"))


def _compare_trees(e, g, nodes_ref):
    t = e.tree(g)
    assert len(t) == len(nodes_ref), (len(t), len(nodes_ref))
    for f in NODE_FIELDS:
        a, b = t[f], nodes_ref[f]
        if f == "first":  # defined only for expanded nodes
            a, b = np.where(t["flags"] & 1, a, 0), np.where(nodes_ref["flags"] & 1, b, 0)
        assert np.array_equal(a, b), f


def _gpu_callback(ev):
    """The oracle's NN callback: one batch-1 forward of the GPU network per leaf."""
    def cb(ctx, sp, pol, val):
        s = np.frombuffer(C.string_at(sp, 24), dtype=_abi.STATE_DTYPE).copy()
        p, v = ev.nn_forward(s)
        C.memmove(pol, p.ctypes.data, 200)
        val[0] = float(v[0])
    return cb


@pytest.mark.parametrize("games,noise", [(1, 0), (4, 0), (4, 1)])
def test_agent_default_playouts_hash_trees_match_oracle(orc, games, noise):
    """5 000 playouts per game with the HASH evaluator: k_search_lat (no noise: one launch, path and sqrt
    table past their LDS copies) or k_search_grp (noise: a launch per 512-simulation chunk); every node, pi
    and move equal the oracle's (mcts_arena.rs:75-323)."""
    roots = random_positions(orc, games, seed=1700 + games + noise)
    with Engine(games=games, sims=AGENT_PLAYOUTS, c_puct=AGENT_C, train_noise=noise, evaluator=_abi.EVAL_HASH,
                blocks=0, seed=91) as e:
        e.set_timing(1)
        r = e.search(roots)
        k = e.kernel_times()
        assert k.backup_select_n == (1 if not noise else (AGENT_PLAYOUTS + 511) // 512)  # noise chunks of 512
        assert k.select_n == 0
        assert r.stats.sims == AGENT_PLAYOUTS * games
        assert r.stats.max_nodes > 2 * 2048  # trees far past the LDS-held top
        for g in range(games):
            cfg = orc.search_cfg(sims=AGENT_PLAYOUTS, c_puct=AGENT_C, evaluator=orc.EVAL_HASH, train_noise=noise,
                                 seed=91, game_id=g, ply=0)
            mv, pi, nodes, st = orc.search(cfg, roots[g])
            _compare_trees(e, g, nodes)
            assert np.array_equal(r.pi[g].reshape(-1), pi.reshape(-1)) and _mv(r.moves[g]) == _mv(mv)


@pytest.mark.parametrize("games", [1, 4])
def test_agent_default_config_nn_trees_match_oracle(orc, trained3, games):
    """The drop-in Agent call as INTEGRATION.md writes it: the reference's default config (400 ms budget,
    5 000 playouts, c = sqrt 2), the trained 3-block network, the budget passed to the engine. The search is
    ONE launch (k_search_lat) whatever the budget; each game's tree equals the oracle's search, fed the GPU
    network's outputs, with the playouts that game ran (all 5 000 unless the 400 ms ran out first)."""
    roots = random_positions(orc, games, seed=1800 + games)
    with Engine(games=games, sims=AGENT_PLAYOUTS, c_puct=AGENT_C, train_noise=0, evaluator=_abi.EVAL_NN, blocks=3,
                precision=_abi.FP32_SPLIT16) as e, \
            Engine(games=4, sims=1, blocks=3, precision=_abi.FP32_SPLIT16) as ev:
        e.load_weights(trained3)
        ev.load_weights(trained3)
        e.set_search_time(AGENT_TIME_S)
        e.set_timing(1)
        r = e.search(roots, root_value=True)
        k = e.kernel_times()
        n = e.search_playouts(games)
        assert (k.backup_select_n, k.select_n, k.expand_n) == (1, 0, 0)
        assert np.all((n >= 1) & (n <= AGENT_PLAYOUTS)) and r.stats.sims == int(n.sum())
        assert e.nn_fallbacks() == 0
        cb = _gpu_callback(ev)
        for g in range(games):
            cfg = orc.search_cfg(sims=int(n[g]), c_puct=AGENT_C, evaluator=orc.EVAL_CALLBACK, fn=cb)
            mv, pi, nodes, _ = orc.search(cfg, roots[g])
            _compare_trees(e, g, nodes)
            assert np.array_equal(r.pi[g].reshape(-1), pi.reshape(-1)) and _mv(r.moves[g]) == _mv(mv)
        _, v = ev.nn_forward(roots)  # the returned value is the extra root evaluation (mod.rs:137-141)
        assert np.array_equal(r.root_value, v[:games])


def test_agent_short_budget_stops_inside_default_playouts(orc):
    """A budget that runs out before 5 000 playouts (15 ms at ~25 us per simulation): the one launch stops
    each game on its own device clock read (>= 1 playout), and the trees equal the oracle's at those
    counts; a second search on the same engine without a budget runs all 5 000 again."""
    roots = random_positions(orc, 2, seed=1900)
    w = random_weights(7, 3)
    with Engine(games=2, sims=AGENT_PLAYOUTS, c_puct=AGENT_C, train_noise=0, evaluator=_abi.EVAL_NN, blocks=3,
                precision=_abi.FP32_SPLIT16) as e, \
            Engine(games=2, sims=1, blocks=3, precision=_abi.FP32_SPLIT16) as ev:
        e.load_weights(w)
        ev.load_weights(w)
        e.set_search_time(0.015)
        r = e.search(roots)
        n = e.search_playouts(2)
        assert np.all((n >= 1) & (n < AGENT_PLAYOUTS)), n
        cb = _gpu_callback(ev)
        for g in range(2):
            mv, pi, nodes, _ = orc.search(orc.search_cfg(sims=int(n[g]), c_puct=AGENT_C, evaluator=orc.EVAL_CALLBACK,
                                                         fn=cb), roots[g])
            _compare_trees(e, g, nodes)
            assert np.array_equal(r.pi[g].reshape(-1), pi.reshape(-1)) and _mv(r.moves[g]) == _mv(mv)
        e.set_search_time(0.0)
        r = e.search(roots)
        assert r.stats.sims == 2 * AGENT_PLAYOUTS and e.last_sims() == AGENT_PLAYOUTS


def test_agent_mirror_default_config_one_launch(orc):
    """The Python Agent mirror with the reference's default AlphaZeroMctsConfig and its budget enforced: the
    search runs on the default fp16x3 network precision as one launch, and its move equals the oracle's
    search fed the same network at the playouts that ran."""
    from onitama_az.game import Deck, GameState, ORIGINAL_CARDS
    from onitama_az.mcts import AlphaZeroMcts, AlphaZeroMctsConfig, ConvResNet, ConvResNetConfig
    model = ConvResNet(ConvResNetConfig(resnet_block_amnt=3), seed=3)
    agent = AlphaZeroMcts(AlphaZeroMctsConfig(), model)  # the reference default: 400 ms, 5 000 playouts, c = sqrt(2)
    gs = GameState.with_deck(Deck([ORIGINAL_CARDS[i] for i in range(5)]))
    mv, value = agent.generate_move(gs)
    eng = model.__dict__["_search"]["engine"]
    assert eng.config.precision == _abi.FP32_SPLIT16
    n = int(eng.search_playouts(1)[0])
    assert 1 <= n <= AGENT_PLAYOUTS
    root = gs.state.to_np(gs.curr_player_color)
    with Engine(games=1, sims=1, blocks=3, precision=_abi.FP32_SPLIT16) as ev:
        ev.load_weights(model.weights)
        ref, _, _, _ = orc.search(orc.search_cfg(sims=n, c_puct=AGENT_C, evaluator=orc.EVAL_CALLBACK,
                                                 fn=_gpu_callback(ev)), root, tree=False)
        _, v = ev.nn_forward(root)
    assert (mv.used_card_idx, mv.mov.from_, mv.mov.to) == (int(ref["slot"]), int(ref["from_"]), int(ref["to"]))
    assert value == float(v[0])


def test_training_mirror_pi_matches_oracle(orc):
    """TrainingAlphaZeroMcts (the self-play agent, alphazero_mcts/mod.rs:163-214) without training noise:
    generate_move_tensor's move and pi (the visit distribution it returns for the replay buffer), and the
    batched generate_move_tensors over 4 roots, equal the oracle's search fed the same network (batch-1 calls
    of the mirror's precision) at max_playouts."""
    from onitama_az.game import Deck, GameState, ORIGINAL_CARDS
    from onitama_az.mcts import AlphaZeroMctsConfig, ConvResNet, ConvResNetConfig, TrainingAlphaZeroMcts
    model = ConvResNet(ConvResNetConfig(resnet_block_amnt=3), seed=5)
    cfg = AlphaZeroMctsConfig(exploration_c=5.0, max_playouts=60, train=False)
    tr = TrainingAlphaZeroMcts(cfg, model)
    gs = GameState.with_deck(Deck([ORIGINAL_CARDS[i] for i in range(5)]))
    mv, pi = tr.generate_move_tensor(gs.state, gs.curr_player_color)
    roots = random_positions(orc, 4, seed=2100)
    moves, pis = tr.generate_move_tensors(roots)
    with Engine(games=1, sims=1, blocks=3, precision=_abi.FP32_SPLIT16) as ev:
        ev.load_weights(model.weights)
        cb = _gpu_callback(ev)
        ref, ref_pi, _, _ = orc.search(orc.search_cfg(sims=60, c_puct=5.0, evaluator=orc.EVAL_CALLBACK, fn=cb),
                                       gs.state.to_np(gs.curr_player_color), tree=False)
        assert (mv.used_card_idx, mv.mov.from_, mv.mov.to) == (int(ref["slot"]), int(ref["from_"]), int(ref["to"]))
        assert np.array_equal(np.asarray(pi).reshape(-1), np.asarray(ref_pi).reshape(-1))
        for g in range(4):
            rmv, rpi, _, _ = orc.search(orc.search_cfg(sims=60, c_puct=5.0, evaluator=orc.EVAL_CALLBACK, fn=cb),
                                        roots[g], tree=False)
            assert _mv(moves[g]) == _mv(rmv)
            assert np.array_equal(np.asarray(pis[g]).reshape(-1), np.asarray(rpi).reshape(-1))
