"""The reference's pure-MCTS agent (onitama-game/src/ai/mcts/mod.rs:13-63) on the GPU.

`Mcts` mirrors the reference struct and Agent impl; every search runs in libonitama_az.so
(oaz_pure_mcts_search: one GPU thread per game, the whole random-rollout UCT search in one
launch). `generate_moves_np` answers a batch of positions at once (the arena's batched fights).
"""
from __future__ import annotations

import ctypes as C
import math
from dataclasses import dataclass
from typing import Optional, Tuple

import numpy as np

from . import _abi
from .game import DoneMove, GameState


def default_config() -> _abi.oaz_pure_mcts_config:
    cfg = _abi.oaz_pure_mcts_config()
    _abi.load().oaz_pure_mcts_config_default(C.byref(cfg))
    return cfg


@dataclass
class PureSearchResult:
    moves: np.ndarray                 # [G] MOVE_DTYPE (from == 25: pass)
    values: np.ndarray                # [G] float32 winrate of the chosen child
    stats: _abi.oaz_pure_mcts_stats
    trees: Optional[np.ndarray]       # [G, cap] PURE_NODE_DTYPE when requested


def pure_mcts_search(roots: np.ndarray, max_playouts: int = 5000, min_node_visits: int = 5,
                     exploration_c: float = math.sqrt(2.0), seed: int = 20260101, game_id0: int = 0,
                     rollout_cap: int = 1000, with_trees: bool = False, device: int = 0) -> PureSearchResult:
    roots = np.ascontiguousarray(roots, dtype=_abi.STATE_DTYPE).reshape(-1)
    cfg = default_config()
    cfg.max_playouts, cfg.min_node_visits = int(max_playouts), int(min_node_visits)
    cfg.exploration_c, cfg.seed, cfg.game_id0, cfg.rollout_cap = float(exploration_c), seed, game_id0, rollout_cap
    cfg.device = int(device)
    lib = _abi.load()
    G = len(roots)
    moves = np.zeros(G, dtype=_abi.MOVE_DTYPE)
    values = np.zeros(G, dtype=np.float32)
    st = _abi.oaz_pure_mcts_stats()
    cap = int(lib.oaz_pure_mcts_tree_capacity(C.byref(cfg))) if with_trees else 0
    trees = np.zeros((G, cap), dtype=_abi.PURE_NODE_DTYPE) if with_trees else None
    _abi.check(lib.oaz_pure_mcts_search(_abi.ptr(roots), G, C.byref(cfg), _abi.ptr(moves), _abi.ptr(values),
                                        C.byref(st), _abi.ptr(trees) if with_trees else None, cap))
    return PureSearchResult(moves, values, st, trees)


def release_workspace(device: int = 0) -> None:
    """Free the device buffer the searches on `device` keep between calls (oaz_pure_mcts_release_workspace)."""
    _abi.check(_abi.load().oaz_pure_mcts_release_workspace(int(device)))


@dataclass
class Mcts:  # ai/mcts/mod.rs:13-30 (search_time is not used: searches run exactly max_playouts)
    search_time: float = 1.0
    min_node_visits: int = 5
    exploration_c: float = math.sqrt(2.0)
    max_playouts: int = 5000
    seed: int = 20260101
    device: int = 0  # the GPU the searches run on (common.rs Options.device)

    def __post_init__(self):
        self._calls = 0

    def generate_move(self, game_state: GameState) -> Tuple[DoneMove, float]:  # mod.rs:37-52
        r = self._search(game_state.state.to_np(game_state.curr_player_color))
        return DoneMove.from_c(r.moves[0]), float(r.values[0])

    def generate_moves_np(self, roots: np.ndarray) -> np.ndarray:
        return self._search(roots).moves

    def _search(self, roots: np.ndarray) -> PureSearchResult:
        # a fresh rollout stream per call (the reference draws from thread_rng)
        g0 = self._calls << 20
        self._calls += 1
        return pure_mcts_search(roots, self.max_playouts, self.min_node_visits, self.exploration_c, self.seed, g0,
                                device=self.device)

    def reserve(self, n: int) -> None:
        pass

    def device_key(self):  # a stateless GPU search (its own buffers and stream per call): may run beside an engine's
        return ("pure_mcts", id(self))

    def name(self) -> str:
        return "MCTS AI"

    def id(self) -> int:  # mod.rs:57-62
        return (int(self.search_time * 1e9) + int(self.exploration_c) + self.max_playouts + self.min_node_visits)
