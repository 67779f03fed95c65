"""Mirror of the reference's self-play driver (alphazero-training/src/train.rs:27-154)."""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np

from . import _abi
from .engine import Engine
from .game import Deck, PlayerColor, encode_batch
from .mcts import AlphaZeroMctsConfig, ConvResNetConfig, Options, TrainingAlphaZeroMcts


@dataclass
class SelfPlayData:  # train.rs:27-33
    pi: np.ndarray          # [2,25] f32 visit distribution
    z: float                # reward(final result, player_color)
    state: np.ndarray       # [21,5,5] f32 planes (create_tensor_from_state)
    player_color: PlayerColor


@dataclass
class TrainConfig:  # train.rs:100-154 (self-play fields)
    model_config: ConvResNetConfig = field(default_factory=ConvResNetConfig)
    mcts_config: AlphaZeroMctsConfig = field(
        default_factory=lambda: AlphaZeroMctsConfig(search_time=0.2, exploration_c=2.0, max_playouts=400, train=True))
    self_play_game_amnt: int = 100
    max_plies: int = 150
    deck: Optional[Deck] = None
    thread_amnt: int = 1    # reference: worker threads; here: games advanced in parallel per worker
    seed: int = 20260101


def self_play(mcts: TrainingAlphaZeroMcts, options: Options, deck: Optional[Deck],
              config: TrainConfig) -> List[SelfPlayData]:
    """train.rs:35-98: play `self_play_game_amnt` games (all of them in parallel on the GPU) and
    return one SelfPlayData per ply."""
    n_games = config.self_play_game_amnt
    kw = dict(games=max(1, min(n_games, 65536)), sims=mcts.config.max_playouts,
              c_puct=mcts.config.exploration_c, train_noise=int(mcts.config.train),
              blocks=mcts.model.config.resnet_block_amnt, max_plies=config.max_plies,
              evaluator=_abi.EVAL_NN, precision=options.precision, seed=config.seed)
    if deck is not None:
        kw.update(fixed_deck=1, deck=deck.indices())
    with Engine(device=options.device, **kw) as eng:
        eng.load_weights(mcts.model.weights)
        samples, _st = eng.selfplay_run(n_games, cap=n_games * (config.max_plies + 2))
    planes = encode_batch(np.ascontiguousarray(samples["state"])) if len(samples) else np.zeros((0, 21, 5, 5), np.float32)
    return [SelfPlayData(s["pi"].reshape(2, 25).copy(), float(s["z"]), planes[i],
                         PlayerColor(int(s["state"]["to_move"]))) for i, s in enumerate(samples)]
