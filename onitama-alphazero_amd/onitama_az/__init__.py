"""onitama_az — MI355X-native Onitama AlphaZero self-play engine (host-side Python mirror).

The compute path is libonitama_az.so (HIP kernels for gfx950 behind the C ABI in
include/onitama_az.h). This package mirrors the reference's Python-visible names over that
ABI: game.* (onitama-game), mcts.* / selfplay.* (alphazero-training).
"""
from . import _abi
from ._abi import OazError, load
from .engine import Engine, SearchResult
from .game import (CARD_NAMES, ORIGINAL_CARDS, Card, Deck, DoneMove, GameState, Move, MoveResult,
                   PieceKind, PlayerColor, State)
from .mcts import (AlphaZeroMcts, AlphaZeroMctsConfig, ConvResNet, ConvResNetConfig, Options,
                   TrainingAlphaZeroMcts, reward)
from .selfplay import SelfPlayData, TrainConfig, self_play
from .evaluator import (AlphaZeroAgent, EloRating, Evaluator, EvaluatorConfig, FightStatistics, PitStatistics,
                        RandomAgent, fight)
from .pure_mcts import Mcts, pure_mcts_search
from .trainer import Trainer, train_epochs
from .train_loop import LoopConfig, Stats, train

__all__ = [
    "_abi", "OazError", "load", "Engine", "SearchResult", "CARD_NAMES", "ORIGINAL_CARDS", "Card", "Deck",
    "DoneMove", "GameState", "Move", "MoveResult", "PieceKind", "PlayerColor", "State", "AlphaZeroMcts",
    "AlphaZeroMctsConfig", "ConvResNet", "ConvResNetConfig", "Options", "TrainingAlphaZeroMcts", "reward",
    "SelfPlayData", "TrainConfig", "self_play", "AlphaZeroAgent", "EloRating", "Evaluator", "EvaluatorConfig",
    "FightStatistics", "PitStatistics", "RandomAgent", "fight", "Mcts", "pure_mcts_search", "Trainer", "train_epochs",
    "LoopConfig", "Stats", "train",
]
