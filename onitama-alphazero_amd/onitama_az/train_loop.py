"""The AlphaZero loop (alphazero-training/src/train.rs:158-412) over the GPU engine.

Per iteration: self-play with the best model (all games in parallel on the GPU, `oaz_selfplay_*`),
`training_epochs` epochs of SGD on the iteration's data buffer (`oaz_trainer_*`, one optimiser kept
across iterations as the reference keeps `opt`), every `evaluation_checkpoint` iterations a pit
against the best model, random and MCTS (promotion when the winrate beats `winrate_percent`), and
`.ot` checkpoints with `save_vs` names. Statistics mirror `stats.rs` (saved as JSON).

Multi-GPU (one process per GPU under torchrun, `rank`/`world`): every rank self-plays its share of
the iteration's games (global game ids, `oaz_selfplay_run`), the samples are all-gathered so every
rank holds the whole buffer in the same order (the join of train.rs:241-244), the epochs run data
parallel (`train_epochs_dp`: sharded batches, gradient all-reduce, BN statistics averaged), so every
rank ends the epochs with identical weights; rank 0 plays the pit and broadcasts the promotion
decision and ratings, and only rank 0 writes checkpoints and statistics.
"""
from __future__ import annotations

import dataclasses
import json
import os
import time
from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np

from . import _abi
from .engine import Engine
from .evaluator import EvaluatorConfig, Evaluator, PitStatistics
from .game import Deck
from .mcts import AlphaZeroMctsConfig, ConvResNet, ConvResNetConfig, Options
from .trainer import Trainer, train_epochs, train_epochs_dp
from .weights import checkpoint_path, random_weights, save_blob_ot


@dataclass
class LoopConfig:  # TrainConfig, train.rs:100-154 (defaults of Default::default)
    buffer_size: int = 180_000
    model_config: ConvResNetConfig = field(default_factory=lambda: ConvResNetConfig(resnet_block_amnt=5))
    mcts_config: AlphaZeroMctsConfig = field(
        default_factory=lambda: AlphaZeroMctsConfig(search_time=0.2, exploration_c=2.0, max_playouts=400, train=True))
    iterations: int = 10
    training_epochs: int = 10
    train_batch_size: int = 512
    self_play_game_amnt: int = 100
    l2_const: float = 1e-4
    learning_rate: float = 1e-2
    save_checkpoint: int = 5
    evaluation_checkpoint: int = 3
    thread_amnt: int = 1  # reference: worker threads x self_play_game_amnt games; here one GPU batch
    max_plies: int = 150
    deck: Optional[Deck] = None
    evaluator_config: EvaluatorConfig = field(default_factory=EvaluatorConfig)
    seed: int = 20260101


@dataclass
class Stats:  # stats.rs:7-24
    iteration: List[int] = field(default_factory=list)
    loss: List[float] = field(default_factory=list)
    policy_loss: List[float] = field(default_factory=list)
    value_loss: List[float] = field(default_factory=list)
    was_best_change: List[bool] = field(default_factory=list)
    fight_statistics: List[PitStatistics] = field(default_factory=list)
    games_played: List[dict] = field(default_factory=list)

    def save(self, path: str) -> None:
        with open(path, "w") as f:
            json.dump(dataclasses.asdict(self), f, default=float)


def _bcast(obj, world: int):
    """Rank 0's object on every rank (the pit result, the new best weights)."""
    if world == 1:
        return obj
    import torch.distributed as dist
    box = [obj]
    dist.broadcast_object_list(box, src=0)
    return box[0]


def train(config: LoopConfig, folder: Optional[str] = None, options: Options = None,
          initial_weights: Optional[np.ndarray] = None, eval_sims: int = 400, rank: int = 0, world: int = 1,
          comm=None, on_iteration=None) -> Stats:
    """train.rs:158-412. Returns the statistics (also written to <folder>/stats.json by rank 0).
    world > 1: an initialised torch.distributed group (rank, world); `comm` (onitama_az.dist.Comm,
    RCCL) carries the sample all-gather and the gradient all-reduce, without it they go over the
    default group through host copies (gloo tests / one-GPU rehearsals). on_iteration(it, new, best),
    if given, sees each iteration's trained and best weights (tests)."""
    from .dist import allgather_samples
    options = options or Options()
    blocks = config.model_config.resnet_block_amnt
    folder = _bcast(folder or os.path.join("models", time.strftime("%Y%m%d_%H%M%S")), world)
    if rank == 0:
        os.makedirs(folder, exist_ok=True)
    weights = np.asarray(initial_weights if initial_weights is not None else random_weights(config.seed, blocks),
                         dtype=np.float32)
    best = weights.copy()
    stats = Stats()
    ratings = [(800.0, 800.0), (800.0, 800.0), (800.0, 800.0)]  # vs best, random, mcts (train.rs:188-205)
    n_games = config.self_play_game_amnt * config.thread_amnt
    mc = config.mcts_config
    with Trainer(blocks=blocks, max_batch=config.train_batch_size, learning_rate=config.learning_rate,
                 weight_decay=config.l2_const, device=options.device) as tr:
        tr.set_weights(weights)
        for it in range(1, config.iterations + 1):
            # self-play with the best model (train.rs:210-250)
            per_rank = (n_games + world - 1) // world
            kw = dict(games=max(1, min(per_rank, 65536)), sims=mc.max_playouts, c_puct=mc.exploration_c,
                      train_noise=int(mc.train), blocks=blocks, max_plies=config.max_plies, evaluator=_abi.EVAL_NN,
                      precision=options.precision, seed=config.seed + it, rank=rank, world=world,
                      sample_capacity=max(1, per_rank) * (config.max_plies + 2))
            if config.deck is not None:
                kw.update(fixed_deck=1, deck=config.deck.indices())
            with Engine(device=options.device, **kw) as eng:
                eng.load_weights(best)
                if world == 1:
                    samples, _ = eng.selfplay_run(n_games, cap=n_games * (config.max_plies + 2))
                else:  # this rank's share, left on the device, then every rank's samples in rank order
                    import torch
                    eng.selfplay_run(n_games, cap=0)
                    samples = allgather_samples(eng, world, torch.device("cuda", options.device), comm=comm)
            stats.games_played.append({"games_amnt": n_games, "positions_retrieved": int(len(samples))})
            # training epochs (train.rs:257-325)
            if world == 1:
                hist = train_epochs(tr, samples, epochs=config.training_epochs, batch=config.train_batch_size,
                                    seed=config.seed + 1000 + it)
            else:
                hist = train_epochs_dp(tr, samples, epochs=config.training_epochs, batch=config.train_batch_size,
                                       seed=config.seed + 1000 + it, rank=rank, world=world, comm=comm)
            k = max(1, len(hist))
            stats.iteration.append(it)
            stats.loss.append(sum(h.loss for h in hist) / k)
            stats.value_loss.append(sum(h.value for h in hist) / k)
            stats.policy_loss.append(sum(h.policy for h in hist) / k)
            new = tr.get_weights()
            # evaluation (train.rs:340-377)
            if it % config.evaluation_checkpoint == 0:
                if rank == 0:
                    ev = Evaluator(config.evaluator_config, ConvResNet(config.model_config, options, best),
                                   ConvResNet(config.model_config, options, new), ratings)
                    pit, promote = ev.pit(sims=eval_sims)
                else:
                    pit, promote = None, None
                pit, promote = _bcast((pit, promote), world)  # one decision for every rank
                ratings = [(pit.self_fight.rating_a, pit.self_fight.rating_b),
                           (pit.random_fight.rating_a, pit.random_fight.rating_b),
                           (pit.mcts_fight.rating_a, pit.mcts_fight.rating_b)]
                stats.was_best_change.append(bool(promote))
                stats.fight_statistics.append(pit)
                if promote:
                    if rank == 0:
                        save_blob_ot(checkpoint_path(folder, it, True, time.strftime("%Y%m%d_%H%M%S")), new, blocks)
                    best = new.copy()
                    ratings[0] = (ratings[0][0], ratings[0][0])  # best inherits the new rating (train.rs:366-367)
            if it % config.save_checkpoint == 0 and rank == 0:
                save_blob_ot(checkpoint_path(folder, it, False, time.strftime("%Y%m%d_%H%M%S")), new, blocks)
            if rank == 0:
                stats.save(os.path.join(folder, "stats.json"))
            if on_iteration is not None:
                on_iteration(it, new, best)
    return stats
