"""Engine: owner of one oaz_engine (one GPU) — batched NN, search and self-play."""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import Optional, Tuple

import numpy as np

from . import _abi


@dataclass
class SearchResult:
    moves: np.ndarray        # [G] MOVE_DTYPE
    pi: np.ndarray           # [G, 2, 25] float32
    root_value: Optional[np.ndarray]  # [G] float32 (extra root evaluation)
    stats: _abi.oaz_search_stats


class Engine:
    """One engine on one GPU. Mirrors the state a reference worker thread owns (a model copy
    and its searches, train.rs:218-238) but for `games` games at once."""

    def __init__(self, config: Optional[_abi.oaz_config] = None, device: int = 0, **overrides):
        lib = _abi.load()
        cfg = config if config is not None else _abi.default_config()
        for k, v in overrides.items():
            if k == "deck":
                for i, c in enumerate(v):
                    cfg.deck[i] = int(c)
            else:
                setattr(cfg, k, v)
        self.config = cfg
        h = lib.oaz_create(C.byref(cfg), int(device))
        if not h:
            raise _abi.OazError(f"oaz_create failed: {lib.oaz_last_error().decode()}")
        self._h = C.c_void_p(h)
        self._lib = lib
        self.device = device

    # -- lifecycle --
    def close(self) -> None:
        if getattr(self, "_h", None):
            self._lib.oaz_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    @property
    def handle(self) -> C.c_void_p:
        return self._h

    def load_weights(self, blob: np.ndarray) -> None:
        blob = np.ascontiguousarray(blob, dtype=np.float32)
        _abi.check(self._lib.oaz_load_weights(self._h, _abi.ptr(blob), blob.size))

    def set_search_params(self, sims: int, c_puct: float, train_noise: bool) -> None:
        """Per-agent AlphaZeroMctsConfig for the next searches (sims <= the creation budget)."""
        _abi.check(self._lib.oaz_set_search_params(self._h, int(sims), float(c_puct), int(bool(train_noise))))

    def set_search_time(self, seconds: float) -> None:
        """Q7 wall-clock budget per search / ply (AlphaZeroMctsConfig.search_time); 0 = off (exactly
        `sims` playouts, the parity mode)."""
        _abi.check(self._lib.oaz_set_search_time(self._h, int(round(float(seconds) * 1e9))))

    def last_sims(self) -> int:
        """Simulations per game of the last search / ply (< sims when a search_time budget stopped it)."""
        n = C.c_int(0)
        _abi.check(self._lib.oaz_last_sims(self._h, C.byref(n)))
        return int(n.value)

    def search_playouts(self, games: int) -> np.ndarray:
        """Playouts each of the first `games` games of the last search ran (a device-side search_time
        budget stops every game, or 16-game group, on its own clock read)."""
        out = np.zeros(int(games), dtype=np.int32)
        _abi.check(self._lib.oaz_search_playouts(self._h, _abi.ptr(out), int(games)))
        return out

    def sync(self) -> None:
        _abi.check(self._lib.oaz_sync(self._h))

    # -- NN --
    def nn_forward(self, states: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
        """ConvResNet::forward(train=false) (net.rs:215-232): policy [B,2,25], value [B]."""
        states = np.ascontiguousarray(states, dtype=_abi.STATE_DTYPE)
        B = len(states)
        pol = np.zeros((B, 2, 25), dtype=np.float32)
        val = np.zeros(B, dtype=np.float32)
        _abi.check(self._lib.oaz_nn_forward(self._h, _abi.ptr(states), B, _abi.ptr(pol), _abi.ptr(val)))
        return pol, val

    def nn_fallbacks(self) -> int:
        """OAZ_FP32_SPLIT16: 16-position tiles recomputed with the bf16x6 split (fp16 range)."""
        n = C.c_uint64(0)
        _abi.check(self._lib.oaz_nn_fallbacks(self._h, C.byref(n)))
        return int(n.value)

    # -- search --
    def search(self, roots: np.ndarray, root_value: bool = False) -> SearchResult:
        roots = np.ascontiguousarray(roots, dtype=_abi.STATE_DTYPE)
        G = len(roots)
        moves = np.zeros(G, dtype=_abi.MOVE_DTYPE)
        pi = np.zeros((G, 2, 25), dtype=np.float32)
        rv = np.zeros(G, dtype=np.float32) if root_value else None
        st = _abi.oaz_search_stats()
        _abi.check(self._lib.oaz_search(self._h, _abi.ptr(roots), G, _abi.ptr(moves), _abi.ptr(pi),
                                        _abi.ptr(rv) if rv is not None else None, C.byref(st)))
        return SearchResult(moves, pi, rv, st)

    def tree(self, game: int) -> np.ndarray:
        n = C.c_int(0)
        _abi.check(self._lib.oaz_tree_dump(self._h, game, None, 0, C.byref(n)))
        out = np.zeros(n.value, dtype=_abi.NODE_DTYPE)
        _abi.check(self._lib.oaz_tree_dump(self._h, game, _abi.ptr(out), n.value, C.byref(n)))
        return out

    # -- self-play --
    def selfplay_reset(self) -> None:
        _abi.check(self._lib.oaz_selfplay_reset(self._h))

    def selfplay_step(self, moves: int = 1) -> None:
        _abi.check(self._lib.oaz_selfplay_step(self._h, int(moves)))

    def selfplay_stats(self) -> _abi.oaz_selfplay_stats:
        st = _abi.oaz_selfplay_stats()
        _abi.check(self._lib.oaz_selfplay_stats_get(self._h, C.byref(st)))
        return st

    def samples_fetch(self, cap: int) -> np.ndarray:
        out = np.zeros(cap, dtype=_abi.SAMPLE_DTYPE)
        n = C.c_size_t(0)
        _abi.check(self._lib.oaz_samples_fetch(self._h, _abi.ptr(out), cap, C.byref(n)))
        return out[: n.value]

    def samples_export_device(self, dev_ptr: int, cap_bytes: int) -> int:
        n = C.c_size_t(0)
        _abi.check(self._lib.oaz_samples_export_device(self._h, C.c_void_p(dev_ptr), cap_bytes, C.byref(n)))
        return n.value

    def selfplay_run(self, n_games: int, cap: int) -> Tuple[np.ndarray, _abi.oaz_selfplay_stats]:
        out = np.zeros(cap, dtype=_abi.SAMPLE_DTYPE)
        n = C.c_size_t(0)
        st = _abi.oaz_selfplay_stats()
        _abi.check(self._lib.oaz_selfplay_run(self._h, int(n_games), _abi.ptr(out), cap, C.byref(n), C.byref(st)))
        return out[: n.value], st

    # -- timing --
    def set_timing(self, on) -> None:
        """False/True: off / every launch; an int N > 1: the kernels of every N-th simulation step."""
        _abi.check(self._lib.oaz_set_timing(self._h, int(on) if not isinstance(on, bool) else (1 if on else 0)))

    def kernel_times(self) -> _abi.oaz_kernel_times:
        t = _abi.oaz_kernel_times()
        _abi.check(self._lib.oaz_kernel_times_get(self._h, C.byref(t)))
        return t

    def kernel_times_reset(self) -> None:
        _abi.check(self._lib.oaz_kernel_times_reset(self._h))
