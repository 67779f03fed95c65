"""Multi-GPU plumbing: one process per GPU, games sharded by global game id, and the one real
exchange of the path — the all-gather of (s, pi, z) replay samples. The
reference joins its self-play threads' buffers (train.rs:241-244); here every rank ends with
every rank's samples. RCCL has no all-gatherv: counts are all-gathered first and each rank's
payload is padded to the maximum (228 bytes per sample)."""
from __future__ import annotations

import torch
import torch.distributed as dist

SAMPLE_BYTES = 228


def global_game_ids(rank: int, world: int, games: int, seq: int) -> range:
    """Global ids of the seq-th game played in each slot of `rank` (matches the kernels:
    id = (seq * world + rank) * games + slot)."""
    base = (seq * world + rank) * games
    return range(base, base + games)


def allgather_sample_bytes(local: torch.Tensor, world: int) -> torch.Tensor:
    """local: uint8 [n*228] on this rank's device (cuda for RCCL, cpu for gloo).
    Returns uint8 [total*228] with every rank's samples in rank order."""
    assert local.dtype == torch.uint8 and local.numel() % SAMPLE_BYTES == 0
    if world == 1:
        return local
    n = torch.tensor([local.numel() // SAMPLE_BYTES], dtype=torch.int64, device=local.device)
    counts = torch.zeros(world, dtype=torch.int64, device=local.device)
    dist.all_gather_into_tensor(counts, n)
    counts_l = [int(c) for c in counts.tolist()]
    mx = max(counts_l)
    padded = torch.zeros(mx * SAMPLE_BYTES, dtype=torch.uint8, device=local.device)
    padded[: local.numel()] = local
    out = torch.empty(world * mx * SAMPLE_BYTES, dtype=torch.uint8, device=local.device)
    dist.all_gather_into_tensor(out, padded)
    parts = [out[r * mx * SAMPLE_BYTES: (r * mx + counts_l[r]) * SAMPLE_BYTES] for r in range(world)]
    return torch.cat(parts)


def allgather_samples(eng, world: int, device: torch.device, host: bool = False) -> int:
    """Move this rank's buffered samples device-to-device into a tensor and all-gather them over
    RCCL (xGMI on one node). Returns the number of samples every rank now holds. host=True
    gathers a host copy instead (gloo)."""
    st = eng.selfplay_stats()
    n = int(st.samples_ready)
    local = torch.empty(max(n, 0) * SAMPLE_BYTES, dtype=torch.uint8, device=device)
    if n:
        got = eng.samples_export_device(local.data_ptr(), local.numel())
        local = local[: got * SAMPLE_BYTES]
    if host:
        torch.cuda.synchronize()
        local = local.cpu()
    allg = allgather_sample_bytes(local, world)
    return allg.numel() // SAMPLE_BYTES
