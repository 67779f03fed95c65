"""Mirror of alphazero-training's search/agent API over the GPU engine.

Reference: alphazero-training/src/alphazero_mcts/mod.rs (AlphaZeroMctsConfig, reward,
TrainingAlphaZeroMcts::generate_move_tensor, AlphaZeroMcts as an Agent), net.rs
(ConvResNetConfig / ConvResNet::forward) and onitama-game/src/ai/agent.rs (trait Agent).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Optional, Tuple

import numpy as np

from . import _abi
from .engine import Engine
from .game import DoneMove, GameState, MoveResult, PlayerColor, State
from .weights import ot_blob, random_weights


@dataclass
class AlphaZeroMctsConfig:  # alphazero_mcts/mod.rs:26-43
    search_time: float = 0.4          # seconds (Q7)
    exploration_c: float = math.sqrt(2.0)
    max_playouts: int = 5000
    train: bool = False
    # Q7: True (default, the reference's semantics) stops each game's search at the first playout that ends
    # past search_time, as the reference's loop `while playouts < max_playouts && elapsed < search_time`
    # (mcts_arena.rs:78) does: on the device clock inside the one-launch searches (every game, or 16-game
    # group, on its own clock read); a batch of more than 16 x CU-count games stops together after the
    # simulation step that passes the budget. False runs exactly max_playouts playouts per search (the
    # parity and throughput mode: bench.py's arena line, the engine-level self-play)
    enforce_search_time: bool = True


def reward(move_result: MoveResult, reward_color: PlayerColor) -> float:  # mod.rs:45-53
    if move_result == MoveResult.RedWin:
        return 1.0 if reward_color == PlayerColor.Red else -1.0
    if move_result == MoveResult.BlueWin:
        return 1.0 if reward_color == PlayerColor.Blue else -1.0
    return 0.0


@dataclass
class ConvResNetConfig:  # net.rs:74-89
    hidden_channels: int = 64
    input_channels: int = 21
    resnet_block_amnt: int = 5


@dataclass
class Options:  # common.rs:8-23 (kind/device): precision and GPU ordinal
    # fp32 by the fp16x3 split (fp32-level error, the one-launch search's network); _abi.FP32 = exact fp32 MFMA
    precision: int = _abi.FP32_SPLIT16
    device: int = 0


class ConvResNet:
    """Weights holder; forward() runs the fused HIP kernel (net.rs:215-232)."""

    def __init__(self, net_config: ConvResNetConfig = None, options: Options = None,
                 weights: Optional[np.ndarray] = None, seed: int = 0):
        self.config = net_config or ConvResNetConfig()
        self.options = options or Options()
        if self.config.hidden_channels != 64 or self.config.input_channels != 21:
            raise ValueError("only hidden_channels=64, input_channels=21 are supported")
        b = self.config.resnet_block_amnt
        self.weights = weights if weights is not None else random_weights(seed, b)
        self.id = f"conv_input_{self.config.input_channels}_hidden_{self.config.hidden_channels}_resnet_{b}"
        self._engine: Optional[Engine] = None
        self._engine_batch = 0

    @staticmethod
    def from_model_file(path: str, options: Options = None) -> "ConvResNet":
        """alphazero_mcts/mod.rs:89-105, but a load error raises instead of keeping random
        weights (Q13)."""
        blob, b = ot_blob(path)  # the C ABI's reader (oaz_ot_read), as a Rust host would load it
        return ConvResNet(ConvResNetConfig(resnet_block_amnt=b), options, blob)

    def save(self, path: str) -> None:
        """VarStore::save of the model's variables (train.rs:414-430)."""
        from .weights import save_blob_ot
        save_blob_ot(path, self.weights, self.config.resnet_block_amnt)

    def _eval_engine(self, batch: int) -> Engine:
        if self._engine is None or self._engine_batch < batch:
            if self._engine is not None:
                self._engine.close()
            self._engine = Engine(device=self.options.device, games=max(batch, 64), sims=1,
                                  blocks=self.config.resnet_block_amnt, evaluator=_abi.EVAL_NN,
                                  precision=self.options.precision)
            self._engine.load_weights(self.weights)
            self._engine_batch = max(batch, 64)
        return self._engine

    def forward(self, states: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
        """policy [B,2,25] (softmax over all 50), value [B,1] for STATE_DTYPE positions
        (colour = state.to_move)."""
        pol, val = self._eval_engine(len(states)).nn_forward(states)
        return pol, val.reshape(-1, 1)


def _search_engine(cache: dict, config: AlphaZeroMctsConfig, model: ConvResNet, games: int) -> Engine:
    """The model's search engine, shared by every agent that uses the model (the reference shares
    one Arc<Mutex<ConvResNet>> between agent clones, mod.rs:84,124): it is rebuilt only when the
    batch or the simulation budget outgrows it; each agent's AlphaZeroMctsConfig is applied with
    oaz_set_search_params before its search."""
    shared = model.__dict__.setdefault("_search", {})
    key = (model.config.resnet_block_amnt, model.options.device, model.options.precision, id(model.weights))
    eng = shared.get("engine")
    if eng is None or shared.get("key") != key or shared["games"] < games or shared["sims"] < config.max_playouts:
        if eng is not None:
            eng.close()
        g, n = max(games, shared.get("games", 0)), max(config.max_playouts, shared.get("sims", 0))
        eng = Engine(device=model.options.device, games=g, sims=n, c_puct=config.exploration_c,
                     train_noise=int(config.train), blocks=model.config.resnet_block_amnt, evaluator=_abi.EVAL_NN,
                     precision=model.options.precision)
        eng.load_weights(model.weights)
        shared.update(engine=eng, key=key, games=g, sims=n)
    eng.set_search_params(config.max_playouts, config.exploration_c, config.train)
    eng.set_search_time(config.search_time if config.enforce_search_time else 0.0)
    return eng


class TrainingAlphaZeroMcts:  # alphazero_mcts/mod.rs:55-79
    def __init__(self, config: AlphaZeroMctsConfig, model: ConvResNet, options: Options = None):
        self.config, self.model, self.options = config, model, options or model.options
        self._cache: dict = {}

    def generate_move_tensor(self, state: State, curr_player_color: PlayerColor) -> Tuple[DoneMove, np.ndarray]:
        """(DoneMove, pi [2,25]) — one search of max_playouts simulations."""
        eng = _search_engine(self._cache, self.config, self.model, 1)
        r = eng.search(state.to_np(curr_player_color))
        return DoneMove.from_c(r.moves[0]), r.pi[0]

    def generate_move_tensors(self, roots: np.ndarray):
        """Batched form: one search per root, all advanced together on the GPU."""
        eng = _search_engine(self._cache, self.config, self.model, len(roots))
        r = eng.search(roots)
        return r.moves, r.pi


class Agent:  # onitama-game/src/ai/agent.rs:7-17
    def generate_move(self, game_state: GameState) -> Tuple[DoneMove, float]:
        raise NotImplementedError

    def name(self) -> str:
        raise NotImplementedError

    def clone_dyn(self) -> "Agent":
        raise NotImplementedError

    def id(self) -> int:
        raise NotImplementedError


class AlphaZeroMcts(Agent):  # alphazero_mcts/mod.rs:81-161
    def __init__(self, config: AlphaZeroMctsConfig, model: ConvResNet, options: Options = None):
        self.config, self.model, self.options = config, model, options or model.options
        self._cache: dict = {}

    @staticmethod
    def from_model_file(model_path: str, config: AlphaZeroMctsConfig, net_config: ConvResNetConfig = None,
                        options: Options = None) -> "AlphaZeroMcts":
        return AlphaZeroMcts(config, ConvResNet.from_model_file(model_path, options), options)

    def generate_move(self, game_state: GameState) -> Tuple[DoneMove, float]:
        """search + an extra root evaluation for the returned value (mod.rs:123-144)."""
        eng = _search_engine(self._cache, self.config, self.model, 1)
        r = eng.search(game_state.state.to_np(game_state.curr_player_color), root_value=True)
        return DoneMove.from_c(r.moves[0]), float(r.root_value[0])

    def generate_moves(self, game_states) -> Tuple[list, np.ndarray]:
        """Batched Agent call: one search per game state, advanced together (arena use)."""
        roots = np.concatenate([g.state.to_np(g.curr_player_color) for g in game_states])
        eng = _search_engine(self._cache, self.config, self.model, len(roots))
        r = eng.search(roots, root_value=True)
        return [DoneMove.from_c(m) for m in r.moves], r.root_value

    def name(self) -> str:
        return "AlphaZero MCTS AI"

    def clone_dyn(self) -> "AlphaZeroMcts":
        return AlphaZeroMcts(self.config, self.model, self.options)

    def id(self) -> int:  # mod.rs:154-160 (model id digits are not numeric here: hashed)
        return (int(self.config.search_time * 1e9) + int(self.config.exploration_c) + self.config.max_playouts
                + int(self.config.train) + (hash(self.model.id) & 0xFFFFFFFF))
