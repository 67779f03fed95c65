"""Arena / evaluator over the GPU engine — SURVEY.md 8f "next" #1.

Mirrors alphazero-training/src/evaluator.rs (FightStatistics, EvaluatorConfig, Evaluator::pit,
fight) and elo_rating.rs, but plays the `game_amnt` games of a fight in parallel: every ply,
the games whose mover belongs to one agent are searched in one batched `oaz_search` call and all
positions are stepped by the GPU step kernel. The per-game semantics (agent plays Red in even
games and Blue in odd ones, 152-ply cut, Elo updated game by game in game order) are the
reference's; only the order in which the games' moves are computed differs.
"""
from __future__ import annotations

from concurrent.futures import ThreadPoolExecutor
from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import _abi
from .game import Deck, MoveResult, PlayerColor, initial_state_np, movegen_batch, step_batch
from .mcts import AlphaZeroMcts, AlphaZeroMctsConfig, ConvResNet, _search_engine

K_ELO = 32.0    # elo_rating.rs:52
C_ELO = 2.5e-3  # elo_rating.rs:54 (1/400)


class EloRating:  # elo_rating.rs:56-71
    @staticmethod
    def elo_change(ra: float, rb: float, is_a_win: bool) -> Tuple[float, float]:
        ea = 1.0 / (1.0 + 10.0 ** (C_ELO * (rb - ra)))
        eb = 1.0 / (1.0 + 10.0 ** (C_ELO * (ra - rb)))
        sa = 1.0 if is_a_win else 0.0
        sb = 1.0 - sa
        return ra + K_ELO * (sa - ea), rb + K_ELO * (sb - eb)


@dataclass
class WinLoseDraws:  # evaluator.rs:22-27
    wins: int = 0
    loses: int = 0
    draws: int = 0


@dataclass
class RatingChange:  # evaluator.rs:29-35
    before_a: float
    after_a: float
    before_b: float
    after_b: float


@dataclass
class FightStatistics:  # evaluator.rs:37-110
    rating_a: float = 800.0
    rating_b: float = 800.0
    general: WinLoseDraws = field(default_factory=WinLoseDraws)
    winrate: float = 0.0
    color: List[WinLoseDraws] = field(default_factory=lambda: [WinLoseDraws(), WinLoseDraws()])
    color_winrate: List[float] = field(default_factory=lambda: [0.0, 0.0])
    rating_change_history: List[RatingChange] = field(default_factory=list)
    # not in the reference struct: per-game outcome and length, in game order (for parity tests)
    results: List[int] = field(default_factory=list)
    plies: List[int] = field(default_factory=list)

    def update(self, move_result: MoveResult, player_color: PlayerColor) -> None:
        lost = (move_result == MoveResult.BlueWin and player_color == PlayerColor.Red) or \
               (move_result == MoveResult.RedWin and player_color == PlayerColor.Blue)
        won = (move_result == MoveResult.BlueWin and player_color == PlayerColor.Blue) or \
              (move_result == MoveResult.RedWin and player_color == PlayerColor.Red)
        if lost or won:
            ra, rb = EloRating.elo_change(self.rating_a, self.rating_b, won)
            self.rating_change_history.append(RatingChange(self.rating_a, ra, self.rating_b, rb))
            self.rating_a, self.rating_b = ra, rb
            if won:
                self.general.wins += 1
                self.color[int(player_color)].wins += 1
            else:
                self.general.loses += 1
                self.color[int(player_color)].loses += 1
        else:
            self.rating_change_history.append(RatingChange(self.rating_a, self.rating_a, self.rating_b, self.rating_b))
            self.general.draws += 1
            self.color[int(player_color)].draws += 1
        self.update_winrate()

    def update_winrate(self) -> None:  # evaluator.rs:101-109 (NaN for a colour with no games, as in Rust)
        def rate(w: WinLoseDraws) -> float:
            n = w.wins + w.loses + w.draws
            return w.wins / n if n else float("nan")
        self.winrate = rate(self.general)
        self.color_winrate = [rate(self.color[0]), rate(self.color[1])]


@dataclass
class PitStatistics:  # evaluator.rs:112-118 (the alpha-beta opponent is out of scope)
    self_fight: FightStatistics
    random_fight: Optional[FightStatistics] = None
    mcts_fight: Optional[FightStatistics] = None


@dataclass
class EvaluatorConfig:  # evaluator.rs:120-137
    winrate_percent: float = 0.55
    game_amnt: int = 20
    deck: Optional[Deck] = None
    max_plies: int = 150
    seed: int = 20260101  # deals for deck=None (the reference uses thread_rng)


class BatchedAgent:
    """An Agent that can answer for many positions at once (STATE_DTYPE roots, colour =
    to_move). Returns MOVE_DTYPE moves."""

    def reserve(self, n: int) -> None:
        """Largest batch the coming fight will ask for (one engine is sized once for it)."""

    def generate_moves_np(self, roots: np.ndarray) -> np.ndarray:
        raise NotImplementedError

    def name(self) -> str:
        raise NotImplementedError

    def device_key(self):
        """What this agent's searches run on (None: the host). Two agents with different GPU keys can
        search their games of a ply at the same time (fight)."""
        return None


class AlphaZeroAgent(BatchedAgent):
    """AlphaZeroMcts (alphazero_mcts/mod.rs:122-161) answering a batch of positions with one
    GPU search per position, all advanced together."""

    def __init__(self, config: AlphaZeroMctsConfig, model: ConvResNet):
        self.mcts = AlphaZeroMcts(config, model)
        self.capacity = 1

    def reserve(self, n: int) -> None:
        self.capacity = max(self.capacity, n)

    def generate_moves_np(self, roots: np.ndarray) -> np.ndarray:
        self.reserve(len(roots))
        eng = _search_engine(self.mcts._cache, self.mcts.config, self.mcts.model, self.capacity)
        return eng.search(roots).moves

    def name(self) -> str:
        return self.mcts.name()

    def device_key(self):  # the model's shared search engine (one search at a time per engine)
        return ("engine", id(self.mcts.model))


class RandomAgent(BatchedAgent):
    """onitama-game/src/ai/random.rs:11-56, including its quirks (Q15): the card is drawn from
    the mover's two cards but `used_card_idx` is 0 or 1 even for Blue, and with no legal move
    for the drawn card it plays the imitation move a5->a4 with a pawn."""

    def __init__(self, seed: int = 0):
        self.rng = np.random.default_rng(seed)

    def generate_moves_np(self, roots: np.ndarray) -> np.ndarray:
        moves, counts = movegen_batch(roots)
        out = np.zeros(len(roots), dtype=_abi.MOVE_DTYPE)
        for i in range(len(roots)):
            card_idx = int(self.rng.integers(0, 2))
            base = 0 if int(roots[i]["to_move"]) == 0 else 2
            cand = [m for m in moves[i, : counts[i]] if int(m["slot"]) == base + card_idx]
            if cand:
                m = cand[int(self.rng.integers(0, len(cand)))]
                out[i] = (int(m["from_"]), int(m["to"]), int(m["piece"]), card_idx)
            else:
                out[i] = (0, 5, 0, card_idx)
        return out

    def name(self) -> str:
        return "Random AI"


def _apply(states: np.ndarray, idx: np.ndarray, moves: np.ndarray) -> np.ndarray:
    """Step states[idx] by moves (GPU step kernel); passes (from == 25) rotate the card on the
    host (state.rs:139-142). Returns MoveResult codes for idx."""
    res = np.full(len(idx), _abi.IN_PROGRESS, dtype=np.uint8)
    is_pass = moves["from_"] >= 25
    real = np.where(~is_pass)[0]
    if len(real):
        sub = np.ascontiguousarray(states[idx[real]])
        res[real] = step_batch(sub, moves[real])
        states[idx[real]] = sub
    for k in np.where(is_pass)[0]:
        s = states[idx[k]]
        slot = int(moves[k]["slot"])
        c = s["cards"].copy()
        c[slot], c[4] = c[4], c[slot]
        s["cards"] = c
        s["to_move"] ^= 1
        states[idx[k]] = s
    return res


def fight(config: EvaluatorConfig, agent: BatchedAgent, opponent: BatchedAgent, agent_rating: float = 800.0,
          opponent_rating: float = 800.0) -> FightStatistics:
    """evaluator.rs:355-399, with the game_amnt games played in parallel."""
    n = config.game_amnt
    decks = [config.deck.indices() if config.deck is not None else list(Deck.default(config.seed, k).indices())
             for k in range(n)]
    states = np.concatenate([initial_state_np(d) for d in decks]) if n else np.zeros(0, _abi.STATE_DTYPE)
    progress = np.full(n, _abi.IN_PROGRESS, dtype=np.uint8)
    active = np.ones(n, dtype=bool)
    budget = np.full(n, config.max_plies, dtype=np.int64)
    plies = np.zeros(n, dtype=np.int64)
    agent_red = np.arange(n) % 2 == 0  # agents = [agent, opponent], swapped after every game
    agent.reserve(n)
    opponent.reserve(n)
    ka, kb = (getattr(a, "device_key", lambda: None)() for a in (agent, opponent))  # (duck-typed agents)
    # two agents on different GPU engines search their games of a ply at the same time (the games
    # are disjoint, so the order of the two searches does not matter); the C ABI calls release the GIL
    concurrent = ka is not None and kb is not None and ka != kb
    with ThreadPoolExecutor(max_workers=2 if concurrent else 1) as pool:  # (joined on any exit)
        while active.any():
            red_to_move = states["to_move"] == 0
            agent_moves = active & (red_to_move == agent_red)
            turns = [(np.where(who)[0], ag) for who, ag in ((agent_moves, agent), (active & ~agent_moves, opponent))]
            turns = [(idx, ag) for idx, ag in turns if len(idx)]
            if concurrent and len(turns) == 2:
                futs = [pool.submit(ag.generate_moves_np, np.ascontiguousarray(states[idx])) for idx, ag in turns]
                moves = [f.result() for f in futs]
            else:
                moves = [ag.generate_moves_np(np.ascontiguousarray(states[idx])) for idx, ag in turns]
            for (idx, _), mv in zip(turns, moves):
                progress[idx] = _apply(states, idx, mv)
            plies[active] += 1
            won = (progress == _abi.RED_WIN) | (progress == _abi.BLUE_WIN)
            cut = active & ~won & (budget < 0)  # train/evaluator loop: `if max_plies < 0 { break }`
            budget[active] -= 1
            active &= ~won & ~cut
    stats = FightStatistics(agent_rating, opponent_rating)
    for k in range(n):  # Elo in game order, as the sequential reference loop
        stats.update(MoveResult(int(progress[k])), PlayerColor.Red if agent_red[k] else PlayerColor.Blue)
        stats.results.append(int(progress[k]))
        stats.plies.append(int(plies[k]))
    return stats


class Evaluator:  # evaluator.rs:139-193
    def __init__(self, config: EvaluatorConfig, best: ConvResNet, new: ConvResNet,
                 ratings: Sequence[Tuple[float, float]] = ((800.0, 800.0), (800.0, 800.0), (800.0, 800.0))):
        self.config, self.best, self.new, self.ratings = config, best, new, ratings

    def pit(self, sims: int = 400, concurrent: bool = True) -> Tuple[PitStatistics, bool]:
        """evaluator.rs:169-193. The reference starts the fights on threads of their own, each with
        its own copy of the networks (`VarStore::copy`, evaluator.rs:206-231); here each fight gets
        weight copies too, so every fight searches on engines of its own and the fights run at the
        same time (concurrent=True: a fight is tail-bound by its longest game's small late batches,
        so three tails overlap on one GPU). The fights share nothing, so their statistics equal the
        one-after-the-other run (concurrent=False). Device memory: four search engines of game_amnt
        trees each (1 + 40 sims nodes of 32 B per tree: 134 GB at 65 536 games x 400 sims), all
        released when pit returns."""
        cfg = AlphaZeroMctsConfig(search_time=0.4, max_playouts=sims, train=False)  # evaluator.rs:198-204
        from .pure_mcts import Mcts  # evaluator.rs:314-353: Mcts{400 ms, min visits 5, c 1.41, 400 playouts}

        def copy(m: ConvResNet) -> ConvResNet:  # train_vs.copy(self.new_nn_vs)
            return ConvResNet(m.config, m.options, weights=np.array(m.weights, copy=True))

        models = [copy(self.new), copy(self.best), copy(self.new), copy(self.new)]
        fights = [
            lambda: fight(self.config, AlphaZeroAgent(cfg, models[0]), AlphaZeroAgent(cfg, models[1]),
                          *self.ratings[0]),
            lambda: fight(self.config, AlphaZeroAgent(cfg, models[2]), RandomAgent(self.config.seed),
                          *self.ratings[1]),
            lambda: fight(self.config, AlphaZeroAgent(cfg, models[3]),
                          Mcts(search_time=0.4, min_node_visits=5, exploration_c=1.41, max_playouts=sims,
                               seed=self.config.seed, device=self.new.options.device), *self.ratings[2]),
        ]
        owned = [[models[0], models[1]], [models[2]], [models[3]]]  # each fight's network copies

        def release(ms):  # a fight's engines (the reference drops each fight's VarStores)
            for m in ms:
                eng = m.__dict__.get("_search", {}).get("engine")
                if eng is not None:
                    eng.close()

        try:
            if concurrent:
                with ThreadPoolExecutor(max_workers=len(fights)) as pool:  # handles joined in order
                    self_fight, random_fight, mcts_fight = [f.result() for f in [pool.submit(f) for f in fights]]
            else:  # one fight after the other, each fight's engines released when it ends
                out = []
                for f, ms in zip(fights, owned):
                    out.append(f())
                    release(ms)
                self_fight, random_fight, mcts_fight = out
        finally:
            for ms in owned:
                release(ms)
        return (PitStatistics(self_fight, random_fight, mcts_fight),
                self_fight.winrate > self.config.winrate_percent)
