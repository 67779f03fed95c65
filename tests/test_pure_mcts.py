"""Pure-MCTS agent (onitama-game/src/ai/mcts/mcts_arena.rs).

Pins: the reference's own tactical tests (mcts_arena.rs:459-553, moves in
tests/golden/reference_kats.json) on the oracle restatement and on the GPU; the GPU trees bit-exact
(every node's visits, reward, winrate, children, move, flags) against the oracle with the same
Philox rollout stream.
"""
import ctypes as C

import numpy as np
import pytest

from conftest import kat_state, random_positions
from onitama_az import _abi
from onitama_az.pure_mcts import default_config

# (min_node_visits, exploration_c, max_playouts) of each reference test
TACTIC_PARAMS = {"test_best_move_win": (5, 2.0 ** 0.5, 5000), "test_no_way_to_hide_for_blue": (5, 2.0, 5000),
                 "test_worst_case_capture_blue": (1, 1.0, 5000)}


def _cfg(playouts, min_visits=5, c=2.0 ** 0.5, seed=20260101):
    cfg = default_config()
    cfg.max_playouts, cfg.min_node_visits, cfg.exploration_c, cfg.seed = playouts, min_visits, c, seed
    return cfg


def _mv(m):
    return [int(m[k]) for k in ("from_", "to", "piece", "slot")]


def _tactics(kats):
    for case in kats["tactics"]:
        name = case["src"].split()[-1]
        yield case, TACTIC_PARAMS[name]


def test_config_defaults():  # ai/mcts/mod.rs:21-30
    cfg = default_config()
    assert (cfg.max_playouts, cfg.min_node_visits) == (5000, 5)
    assert cfg.exploration_c == np.float32(2.0 ** 0.5)


def test_oracle_reference_tactics(kats, orc):
    for case, (mv, c, po) in _tactics(kats):
        root = kat_state(case["state"], case["color"])
        for seed in (1, 2):
            m, _, _, _ = orc.pure_mcts(_cfg(po, mv, c, seed), 0, root[0])
            assert _mv(m) == case["expected"], (case["src"], seed)


def test_oracle_tree_invariants(orc):
    roots = random_positions(orc, 6, seed=31)
    for i in range(len(roots)):
        cfg = _cfg(300)
        m, v, nodes, st = orc.pure_mcts(cfg, i, roots[i])
        assert nodes[0]["visits"] == 300 and st.playouts == 300
        if nodes[0]["nch"]:
            ch = nodes[int(nodes[0]["first"]): int(nodes[0]["first"]) + int(nodes[0]["nch"])]
            # the first min_node_visits + 1 playouts ran before the root was expanded and the
            # expanding playout simulates from the root itself (mcts_arena.rs:118-130)
            assert int(ch["visits"].sum()) == 300 - 6 - 1
            assert np.all(ch["parent"] == 0)
        for n in nodes:  # winrate = reward / visits in f32 (MctsNode::update)
            if n["visits"]:
                assert n["winrate"] == np.float32(n["reward"]) / np.float32(n["visits"])


@pytest.mark.gpu
def test_gpu_trees_bitexact_vs_oracle(orc):
    from onitama_az.pure_mcts import pure_mcts_search
    roots = random_positions(orc, 24, seed=77)
    for min_visits, c, po in ((5, 2.0 ** 0.5, 300), (1, 1.0, 200), (0, 1.41, 64)):
        r = pure_mcts_search(roots, po, min_visits, c, seed=99, game_id0=1000, with_trees=True)
        for g in range(len(roots)):
            m, v, nodes, _ = orc.pure_mcts(_cfg(po, min_visits, c, 99), 1000 + g, roots[g])
            got = r.trees[g][: len(nodes)]
            assert got.tobytes() == nodes.tobytes(), (g, min_visits)
            assert _mv(r.moves[g]) == _mv(m) and r.values[g] == np.float32(v)


@pytest.mark.gpu
def test_gpu_workspace_kept_reused_concurrent_and_released(orc):
    """The device workspace kept between searches (oaz_pure_mcts_release_workspace): a smaller search after a
    larger one reuses it, threads searching at once on the same device (one of them on its own allocation)
    and a search after the release all give the oracle's trees."""
    import threading
    from onitama_az.pure_mcts import pure_mcts_search, release_workspace
    roots = random_positions(orc, 16, seed=78)
    ref = [orc.pure_mcts(_cfg(120, 5, 1.41, 7), 500 + g, roots[g])[2] for g in range(len(roots))]

    def check(r):
        for g in range(len(roots)):
            assert r.trees[g][: len(ref[g])].tobytes() == ref[g].tobytes(), g

    big = np.concatenate([roots] * 64)  # a larger search first: the kept buffer grows to it
    pure_mcts_search(big, 120, 5, 1.41, seed=7, game_id0=500)
    check(pure_mcts_search(roots, 120, 5, 1.41, seed=7, game_id0=500, with_trees=True))
    out, errs = [None] * 4, []

    def run(k):
        try:
            out[k] = pure_mcts_search(roots, 120, 5, 1.41, seed=7, game_id0=500, with_trees=True)
        except Exception as ex:  # noqa: BLE001
            errs.append(ex)
    th = [threading.Thread(target=run, args=(k,)) for k in range(4)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs, errs
    for r in out:
        check(r)
    release_workspace(0)
    release_workspace(0)  # nothing kept: fine
    check(pure_mcts_search(roots, 120, 5, 1.41, seed=7, game_id0=500, with_trees=True))


@pytest.mark.gpu
def test_gpu_reference_tactics(kats):
    from onitama_az.pure_mcts import pure_mcts_search
    for case, (mv, c, po) in _tactics(kats):
        root = kat_state(case["state"], case["color"])
        r = pure_mcts_search(np.concatenate([root] * 8), po, mv, c, seed=5)  # 8 independent streams
        for g in range(8):
            assert _mv(r.moves[g]) == case["expected"], (case["src"], g)


@pytest.mark.gpu
def test_gpu_no_legal_move_positions_match_oracle(orc, kats):
    """state.rs:852-889 KAT: Blue has no legal move. As the root it returns the pass move; with
    Red to move, rollouts run into Blue's forced passes (random own card, state.rs:139-142) and
    the trees must still match the oracle bit for bit."""
    from onitama_az.pure_mcts import pure_mcts_search
    case = [c for c in kats["movegen"] if "no_legal_moves_at_all" in c["src"]][0]
    blue, red = kat_state(case["state"], 1), kat_state(case["state"], 0)
    r = pure_mcts_search(blue, 50, 5, 1.41)
    assert _mv(r.moves[0]) == [25, 25, 0, 2]
    r = pure_mcts_search(np.concatenate([red, blue]), 400, 1, 1.41, seed=3, with_trees=True)
    assert r.stats.rollout_passes > 0
    for g, root in enumerate((red, blue)):
        m, v, nodes, _ = orc.pure_mcts(_cfg(400, 1, 1.41, 3), g, root[0])
        assert r.trees[g][: len(nodes)].tobytes() == nodes.tobytes()


@pytest.mark.gpu
def test_mcts_agent_api_and_arena():
    from onitama_az.evaluator import AlphaZeroAgent, EvaluatorConfig, RandomAgent, fight
    from onitama_az.game import Deck, GameState, MoveResult, ORIGINAL_CARDS
    from onitama_az.mcts import AlphaZeroMctsConfig, ConvResNet, ConvResNetConfig
    from onitama_az.pure_mcts import Mcts
    agent = Mcts(min_node_visits=5, exploration_c=1.41, max_playouts=400)  # evaluator.rs:340-345
    gs = GameState.with_deck(Deck([ORIGINAL_CARDS[i] for i in range(5)]))
    mv, value = agent.generate_move(gs)
    assert (mv.used_card_idx, mv.mov) in gs.state.generate_all_legal_moves(gs.curr_player_color)
    assert -1.0 <= value <= 1.0 and agent.name() == "MCTS AI"
    st = fight(EvaluatorConfig(game_amnt=8, seed=4), agent, RandomAgent(seed=3))
    assert st.general.wins >= 6, st.general  # random rollouts beat random play
    az = AlphaZeroAgent(AlphaZeroMctsConfig(max_playouts=16), ConvResNet(ConvResNetConfig(resnet_block_amnt=1), seed=1))
    st2 = fight(EvaluatorConfig(game_amnt=2, max_plies=20, seed=4), az, Mcts(max_playouts=64))
    assert len(st2.results) == 2
