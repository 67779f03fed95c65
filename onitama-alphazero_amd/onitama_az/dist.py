"""Multi-GPU plumbing: one process per GPU, games sharded by global game id, and the one real
exchange of the path — the all-gather of (s, pi, z) replay samples, which
replaces the reference's join of its self-play workers' buffers (train.rs:241-244).

The product path is the C ABI's RCCL communicator (`oaz_comm_*`, `oaz_allgather_samples`:
counts all-gathered, then one grouped broadcast per rank into its offset — an all-gatherv with no
padding); this module is a thin caller that hands the communicator id from rank 0 to the others
over torch.distributed (any out-of-band channel works: a Rust host would use its own). The gloo
path (`allgather_sample_bytes`) is for CPU tests and one-GPU rehearsals, where RCCL cannot run
two ranks on one device."""
from __future__ import annotations

import ctypes as C
from typing import List, Optional, Tuple

import numpy as np
import torch
import torch.distributed as dist

from . import _abi

SAMPLE_BYTES = 228


def global_game_ids(rank: int, world: int, games: int, seq: int) -> np.ndarray:
    """Global ids of the seq-th game played in each slot of `rank`: oaz_slot_game_ids, the rule the
    self-play kernel keys deals and root noise with (id = (seq * world + rank) * games + slot)."""
    out = np.zeros(int(games), dtype=np.uint64)
    _abi.check(_abi.load().oaz_slot_game_ids(int(rank), int(world), int(games), int(seq), _abi.ptr(out)))
    return out


class Comm:
    """oaz_comm: an RCCL communicator of `world` ranks, one GPU each."""

    def __init__(self, rank: int, world: int, device: int, comm_id: Optional[bytes] = None):
        lib = _abi.load()
        cid = _abi.oaz_comm_id()
        if comm_id is None:
            if world != 1:
                raise ValueError("world > 1 needs the id made by rank 0 (Comm.unique_id / Comm.create)")
            _abi.check(lib.oaz_comm_unique_id(C.byref(cid)))
        else:
            C.memmove(C.addressof(cid), comm_id, 128)
        h = lib.oaz_comm_init(C.byref(cid), int(rank), int(world), int(device))
        if not h:
            raise _abi.OazError(f"oaz_comm_init failed: {lib.oaz_last_error().decode()}")
        self._h, self._lib = C.c_void_p(h), lib
        self.rank, self.world, self.device = rank, world, device

    @staticmethod
    def unique_id() -> bytes:
        cid = _abi.oaz_comm_id()
        _abi.check(_abi.load().oaz_comm_unique_id(C.byref(cid)))
        return C.string_at(C.addressof(cid), 128)

    @classmethod
    def create(cls, rank: int, world: int, device: int) -> "Comm":
        """Collective over an initialised torch.distributed group: rank 0 makes the id and
        broadcasts it (the out-of-band channel), every rank joins the RCCL communicator."""
        box: List[Optional[bytes]] = [cls.unique_id() if rank == 0 else None]
        if world > 1:
            dist.broadcast_object_list(box, src=0)
        return cls(rank, world, device, box[0])

    def close(self) -> None:
        if getattr(self, "_h", None):
            self._lib.oaz_comm_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self) -> C.c_void_p:
        return self._h

    def allgather_samples(self, eng, out: torch.Tensor) -> Tuple[int, List[int]]:
        """Every rank's buffered samples into `out` (uint8 CUDA tensor of k*228 bytes on this
        rank's GPU), rank order. Returns (total, per-rank counts)."""
        assert out.dtype == torch.uint8 and out.is_cuda and out.numel() % SAMPLE_BYTES == 0
        n = C.c_size_t(0)
        counts = np.zeros(self.world, dtype=np.uint64)
        _abi.check(self._lib.oaz_allgather_samples(eng.handle, self._h, C.c_void_p(out.data_ptr()),
                                                    out.numel() // SAMPLE_BYTES, C.byref(n), _abi.ptr(counts)))
        return int(n.value), [int(c) for c in counts]

    def stats(self) -> _abi.oaz_comm_stats:
        """ncclCommCount ranks and the HIP-event times of the last all-gather on the comm stream."""
        st = _abi.oaz_comm_stats()
        _abi.check(self._lib.oaz_comm_stats_get(self._h, C.byref(st)))
        return st

    def allreduce_sum_(self, t: torch.Tensor, stream: Optional[int] = None) -> None:
        assert t.dtype == torch.float32 and t.is_cuda and t.is_contiguous()
        _abi.check(self._lib.oaz_comm_allreduce_sum_f32(self._h, C.c_void_p(t.data_ptr()), t.numel(),
                                                        C.c_void_p(stream) if stream else None))

    def broadcast_(self, t: torch.Tensor, root: int = 0, stream: Optional[int] = None) -> None:
        assert t.is_cuda and t.is_contiguous()
        _abi.check(self._lib.oaz_comm_broadcast(self._h, C.c_void_p(t.data_ptr()), t.numel() * t.element_size(),
                                                int(root), C.c_void_p(stream) if stream else None))

    def sync(self) -> None:
        _abi.check(self._lib.oaz_comm_sync(self._h))


def allgather_sample_bytes(local: torch.Tensor, world: int) -> torch.Tensor:
    """gloo / CPU path (tests, one-GPU rehearsals). local: uint8 [n*228]. Returns uint8
    [total*228] with every rank's samples in rank order (counts all-gathered, padded to max)."""
    assert local.dtype == torch.uint8 and local.numel() % SAMPLE_BYTES == 0
    if world == 1:
        return local
    n = torch.tensor([local.numel() // SAMPLE_BYTES], dtype=torch.int64, device=local.device)
    counts = [torch.zeros(1, dtype=torch.int64, device=local.device) for _ in range(world)]
    dist.all_gather(counts, n)
    counts_l = [int(c.item()) for c in counts]
    mx = max(counts_l)
    padded = torch.zeros(mx * SAMPLE_BYTES, dtype=torch.uint8, device=local.device)
    padded[: local.numel()] = local
    parts = [torch.empty(mx * SAMPLE_BYTES, dtype=torch.uint8, device=local.device) for _ in range(world)]
    dist.all_gather(parts, padded)
    return torch.cat([parts[r][: counts_l[r] * SAMPLE_BYTES] for r in range(world)])


def as_samples(raw: torch.Tensor) -> np.ndarray:
    """uint8 [k*228] (any device) -> numpy oaz_sample records."""
    return np.frombuffer(raw.cpu().numpy().tobytes(), dtype=_abi.SAMPLE_DTYPE).copy()


def allgather_samples_device(eng, world: int, device: torch.device, comm: Comm) -> Tuple[torch.Tensor, int, List[int]]:
    """The RCCL exchange alone: every rank's buffered samples as raw 228-byte records in one uint8
    tensor on this rank's GPU (rank order), the total and the per-rank counts. No host copy."""
    st = eng.selfplay_stats()
    # capacity for the largest possible total: a counts pre-pass is inside the C call
    n_local = torch.tensor([int(st.samples_ready)], dtype=torch.int64, device=device)
    if world > 1:
        dist.all_reduce(n_local)
    out = torch.empty(max(1, int(n_local.item())) * SAMPLE_BYTES, dtype=torch.uint8, device=device)
    total, counts = comm.allgather_samples(eng, out)
    return out[: total * SAMPLE_BYTES], total, counts


def allgather_samples(eng, world: int, device: torch.device, comm: Optional[Comm] = None) -> np.ndarray:
    """Every rank's buffered samples (oaz_sample records, rank order) on every rank. With an RCCL
    `comm` the exchange is device to device through the C ABI; without one (gloo / CPU tests) the
    samples are fetched to the host and gathered over the default process group."""
    if comm is not None:
        raw, _, _ = allgather_samples_device(eng, world, device, comm)
        return as_samples(raw)
    local = eng.samples_fetch(int(eng.selfplay_stats().samples_ready))
    raw = torch.from_numpy(local.view(np.uint8).copy())
    return as_samples(allgather_sample_bytes(raw, world))
