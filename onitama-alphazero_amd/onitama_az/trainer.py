"""Trainer: the training half of the AlphaZero loop on the GPU.

Mirrors the body of `train()` (alphazero-training/src/train.rs:264-339): for each epoch,
`train_amnt = len(buffer) // batch` batches drawn with `choose_multiple` (a uniform draw without
replacement; seeded numpy here, the reference uses thread_rng), each one
`forward(train=true) -> alphaloss -> opt.backward_step` with nn::Sgd{momentum 0.9} and
weight decay l2_const (train.rs:181-186). Every step runs in libonitama_az.so
(oaz_trainer_*, csrc/oaz_train.hip); this module only draws indices and keeps statistics.

Data-parallel training (`world > 1`, train_epochs_dp): every rank runs backward on its own batch
shard, the flat gradient buffer is all-reduced (the C ABI's RCCL communicator, oaz_comm_*) on the
trainer's stream, then every rank applies the same SGD step (grad_scale = 1/world); BN running
statistics and losses are averaged over ranks after each epoch.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import List, Optional, Tuple

import numpy as np

from . import _abi


@dataclass
class EpochLoss:  # the per-epoch line of train.rs:316-324
    loss: float
    value: float
    policy: float
    steps: int


class Trainer:
    def __init__(self, blocks: int, max_batch: int = 512, learning_rate: float = 5e-3, momentum: float = 0.9,
                 weight_decay: float = 1e-4, value_loss_broadcast: bool = True, device: int = 0):
        lib = _abi.load()
        cfg = _abi.oaz_train_config()
        lib.oaz_train_config_default(C.byref(cfg))
        cfg.blocks, cfg.max_batch = int(blocks), int(max_batch)
        cfg.learning_rate, cfg.momentum, cfg.weight_decay = learning_rate, momentum, weight_decay
        cfg.value_loss_broadcast = int(bool(value_loss_broadcast))
        h = lib.oaz_trainer_create(C.byref(cfg), int(device))
        if not h:
            raise _abi.OazError(f"oaz_trainer_create failed: {lib.oaz_last_error().decode()}")
        self._h, self._lib, self.config, self.device = C.c_void_p(h), lib, cfg, device
        self.blocks = int(blocks)
        self.n_params = int(lib.oaz_weight_count(self.blocks, 64, 21))

    def close(self) -> None:
        if self._h:
            self._lib.oaz_trainer_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc: int) -> None:
        _abi.check(rc)

    # -- parameters ---------------------------------------------------------------------------
    def set_weights(self, blob: np.ndarray) -> None:
        blob = np.ascontiguousarray(blob, dtype=np.float32)
        self._check(self._lib.oaz_trainer_set_weights(self._h, _abi.ptr(blob), blob.size))

    def get_weights(self) -> np.ndarray:
        out = np.zeros(self.n_params, dtype=np.float32)
        self._check(self._lib.oaz_trainer_get_weights(self._h, _abi.ptr(out), out.size))
        return out

    def save_ot(self, path: str) -> None:
        """The training weights as a .ot checkpoint (oaz_trainer_save_ot; save_vs, train.rs:414-430)."""
        self._check(self._lib.oaz_trainer_save_ot(self._h, str(path).encode()))

    def grads(self) -> np.ndarray:
        out = np.zeros(self.n_params, dtype=np.float32)
        self._check(self._lib.oaz_trainer_get_grads(self._h, _abi.ptr(out), out.size))
        return out

    def grads_device(self) -> Tuple[int, int]:
        p, n = C.c_void_p(), C.c_size_t()
        self._check(self._lib.oaz_trainer_grads(self._h, C.byref(p), C.byref(n)))
        return int(p.value), int(n.value)

    def set_stream(self, stream_handle: Optional[int]) -> None:
        self._check(self._lib.oaz_trainer_set_stream(self._h, C.c_void_p(stream_handle or 0)))

    # -- data ------------------------------------------------------------------------------------
    def load_samples(self, samples: np.ndarray) -> None:
        samples = np.ascontiguousarray(samples, dtype=_abi.SAMPLE_DTYPE)
        self._check(self._lib.oaz_trainer_load_samples(self._h, _abi.ptr(samples), len(samples)))
        self.n_samples = len(samples)

    def bind_device_samples(self, dev_ptr: int, n: int) -> None:
        self._check(self._lib.oaz_trainer_bind_device_samples(self._h, C.c_void_p(dev_ptr), int(n)))
        self.n_samples = int(n)

    def set_batches(self, idx: np.ndarray) -> None:
        idx = np.ascontiguousarray(idx, dtype=np.int32)
        assert idx.ndim == 2
        self._check(self._lib.oaz_trainer_set_batches(self._h, _abi.ptr(idx), idx.shape[0], idx.shape[1]))

    # -- steps -------------------------------------------------------------------------------------
    def backward(self, b: int) -> None:
        self._check(self._lib.oaz_trainer_backward(self._h, int(b)))

    def apply(self, grad_scale: float = 1.0) -> None:
        self._check(self._lib.oaz_trainer_apply(self._h, C.c_float(grad_scale)))

    def train(self, first: int, count: int) -> None:
        self._check(self._lib.oaz_trainer_train(self._h, int(first), int(count)))

    def losses(self) -> Tuple[float, float, int]:
        """(sum of value losses, sum of policy losses, steps) since the previous call."""
        out = (C.c_double * 3)()
        self._check(self._lib.oaz_trainer_losses(self._h, C.byref(out)))
        return float(out[0]), float(out[1]), int(out[2])

    def sync(self) -> None:
        self._check(self._lib.oaz_trainer_sync(self._h))


def choose_batches(rng: np.random.Generator, n_samples: int, batch: int, n_batches: int) -> np.ndarray:
    """`data_buffer.iter().choose_multiple(&mut rng, batch)` per batch (train.rs:272-276): a uniform
    draw without replacement inside a batch, independent across batches."""
    return np.stack([rng.choice(n_samples, size=batch, replace=False) for _ in range(n_batches)]).astype(np.int32)


def train_epochs(trainer: Trainer, samples: np.ndarray, epochs: int = 10, batch: int = 512,
                 seed: int = 0) -> List[EpochLoss]:
    """The epoch loop of train.rs:264-325 on one GPU (stops early, as the reference, when the
    buffer holds fewer than `batch` samples)."""
    rng = np.random.default_rng(seed)
    trainer.load_samples(samples)
    out: List[EpochLoss] = []
    for _ in range(epochs):
        if len(samples) < batch:
            break
        n = len(samples) // batch
        trainer.set_batches(choose_batches(rng, len(samples), batch, n))
        trainer.train(0, n)
        v, p, k = trainer.losses()
        out.append(EpochLoss((v + p) / k, v / k, p / k, k))
    return out


class _DeviceArray:
    """Zero-copy view of a device buffer for torch.as_tensor (__cuda_array_interface__)."""

    def __init__(self, ptr: int, n: int):
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": "<f4", "data": (ptr, False), "version": 3,
                                         "strides": None}


def _allreduce_sum(t, comm, stream: int) -> None:
    """Sum over ranks in place: the C ABI's RCCL communicator on `stream`, or (no comm: gloo CPU
    tests / one-GPU rehearsals) torch.distributed through a host copy."""
    import torch
    import torch.distributed as dist
    if comm is not None:
        comm.allreduce_sum_(t, stream)
        return
    torch.cuda.current_stream().synchronize()
    h = t.cpu()
    dist.all_reduce(h)
    t.copy_(h.to(t.device))


def train_epochs_dp(trainer: Trainer, samples: np.ndarray, epochs: int, batch: int, seed: int, rank: int,
                    world: int, comm=None) -> List[EpochLoss]:
    """Data-parallel epochs (train.rs:264-325 over `world` GPUs): the global batch `batch` is split
    into `world` shards of batch/world samples; the gradient buffer is summed over ranks (RCCL via
    `comm`, an onitama_az.dist.Comm) and applied with grad_scale 1/world, so every rank takes the
    same SGD step. All ranks draw the same index stream (same seed, same gathered `samples`) and take
    their shard. BN batch statistics are per shard (DDP without SyncBatchNorm); the running
    statistics are averaged over ranks after each epoch, and the reported losses are the global
    ones, so every rank ends each epoch with identical weights and statistics."""
    import torch
    assert batch % world == 0 and (batch // world) % 16 == 0
    shard = batch // world
    # one explicit stream for the trainer's kernels, the collectives and the torch copies (the legacy
    # default stream, handle 0, would mean "the trainer's own stream" to oaz_trainer_set_stream and
    # leave the all-reduce unordered against backward / apply)
    ts = torch.cuda.Stream()
    with torch.cuda.stream(ts):
        out = _epochs_dp(trainer, samples, epochs, batch, seed, rank, world, comm, shard, ts.cuda_stream)
    trainer.sync()
    trainer.set_stream(None)
    return out


def _epochs_dp(trainer, samples, epochs, batch, seed, rank, world, comm, shard, stream) -> List[EpochLoss]:
    import torch
    trainer.set_stream(stream)
    dev = f"cuda:{torch.cuda.current_device()}"
    ptr, n = trainer.grads_device()
    grads = torch.as_tensor(_DeviceArray(ptr, n), device=dev)
    nbn = int(trainer._lib.oaz_trainer_bn_stats_count(trainer.blocks))
    bn = torch.empty(nbn, dtype=torch.float32, device=dev)
    rng = np.random.default_rng(seed)
    trainer.load_samples(samples)
    out: List[EpochLoss] = []
    for _ in range(epochs):
        if len(samples) < batch:
            break
        nb = len(samples) // batch
        idx = choose_batches(rng, len(samples), batch, nb)[:, rank * shard:(rank + 1) * shard]
        trainer.set_batches(idx)
        for b in range(nb):
            trainer.backward(b)
            if world > 1:
                _allreduce_sum(grads, comm, stream)
            trainer.apply(1.0 / world)
        v, p, k = trainer.losses()
        if world > 1:
            trainer._check(trainer._lib.oaz_trainer_bn_stats_pack(trainer._h, C.c_void_p(bn.data_ptr())))
            _allreduce_sum(bn, comm, stream)
            trainer._check(trainer._lib.oaz_trainer_bn_stats_unpack(trainer._h, C.c_void_p(bn.data_ptr()),
                                                                    C.c_float(1.0 / world)))
            tot = torch.tensor([v, p], dtype=torch.float32, device=dev)
            _allreduce_sum(tot, comm, stream)
            torch.cuda.current_stream().synchronize()
            v, p = (float(x) / world for x in tot.tolist())
        out.append(EpochLoss((v + p) / k, v / k, p / k, k))
    return out
