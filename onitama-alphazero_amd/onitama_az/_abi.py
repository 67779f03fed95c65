"""ctypes binding of include/onitama_az.h (the C ABI of libonitama_az.so).

The product path is the HIP library; this module only marshals arguments. There is no CPU
fallback: if the library or a GPU is missing, calls raise OazError.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import numpy as np

LIB_NAME = "libonitama_az.so"
LIB_PATH = Path(__file__).resolve().parent / LIB_NAME

RED, BLUE = 0, 1
PAWN, KING = 0, 1
CAPTURE, RED_WIN, BLUE_WIN, IN_PROGRESS = 0, 1, 2, 3
EVAL_NN, EVAL_HASH = 0, 1
FP32, BF16, FP32_SPLIT, FP32_SPLIT16 = 0, 1, 2, 3  # OAZ_FP32 / OAZ_BF16 / OAZ_FP32_SPLIT / OAZ_FP32_SPLIT16
ERR_RANGE = -7  # OAZ_ERR_RANGE (ABI 1 only; ABI 2 recomputes fp16-range tiles, oaz_nn_fallbacks)
ERR_CAPACITY = -4
ERR_COMM = -8
ABI_VERSION = 5
MAX_MOVES = 40


class OazError(RuntimeError):
    """Error reported by the C ABI (status < 0) or a missing library/device."""


class oaz_state(C.Structure):
    _fields_ = [
        ("kings", C.c_uint32 * 2),
        ("pawns", C.c_uint32 * 2),
        ("cards", C.c_uint8 * 5),
        ("to_move", C.c_uint8),
        ("pad", C.c_uint8 * 2),
    ]


class oaz_move(C.Structure):
    _fields_ = [("from_", C.c_uint8), ("to", C.c_uint8), ("piece", C.c_uint8), ("slot", C.c_uint8)]


class oaz_node(C.Structure):
    _fields_ = [
        ("W", C.c_double),
        ("P", C.c_double),
        ("N", C.c_uint32),
        ("first", C.c_uint32),
        ("mv", C.c_uint16),
        ("nch", C.c_uint8),
        ("flags", C.c_uint8),
        ("pad", C.c_uint32),
    ]


class oaz_sample(C.Structure):
    _fields_ = [("state", oaz_state), ("pi", C.c_float * 50), ("z", C.c_float)]


class oaz_config(C.Structure):
    _fields_ = [
        ("blocks", C.c_int32),
        ("channels", C.c_int32),
        ("in_planes", C.c_int32),
        ("sims", C.c_int32),
        ("c_puct", C.c_double),
        ("train_noise", C.c_int32),
        ("max_plies", C.c_int32),
        ("dirichlet_alpha", C.c_double),
        ("dirichlet_eps", C.c_double),
        ("games", C.c_int32),
        ("evaluator", C.c_int32),
        ("precision", C.c_int32),
        ("fixed_deck", C.c_int32),
        ("deck", C.c_uint8 * 5),
        ("pad0", C.c_uint8 * 3),
        ("seed", C.c_uint64),
        ("rank", C.c_int32),
        ("world", C.c_int32),
        ("sample_capacity", C.c_int32),
        ("stagger", C.c_int32),
        ("compact", C.c_int32),
        ("parts", C.c_int32),
        ("search_time_ns", C.c_int64),
        ("step_kernels", C.c_int32),
        ("reserved", C.c_int32),
    ]


class oaz_search_stats(C.Structure):
    _fields_ = [
        ("sims", C.c_uint64),
        ("expansions", C.c_uint64),
        ("children", C.c_uint64),
        ("terminal_leaves", C.c_uint64),
        ("depth_sum", C.c_uint64),
        ("stuck_leaves", C.c_uint64),
        ("max_nodes", C.c_uint64),
        ("nn_evals", C.c_uint64),
    ]


class oaz_selfplay_stats(C.Structure):
    _fields_ = [
        ("moves", C.c_uint64),
        ("games_finished", C.c_uint64),
        ("games_cut", C.c_uint64),
        ("red_wins", C.c_uint64),
        ("blue_wins", C.c_uint64),
        ("samples_ready", C.c_uint64),
        ("samples_dropped", C.c_uint64),
        ("passes", C.c_uint64),
        ("search", oaz_search_stats),
    ]


class oaz_kernel_times(C.Structure):
    _fields_ = [
        ("select_ms", C.c_double),
        ("nn_ms", C.c_double),
        ("expand_ms", C.c_double),
        ("finalize_ms", C.c_double),
        ("select_n", C.c_uint64),
        ("nn_n", C.c_uint64),
        ("expand_n", C.c_uint64),
        ("finalize_n", C.c_uint64),
        ("nn_samples", C.c_uint64),
        ("noise_ms", C.c_double),
        ("noise_n", C.c_uint64),
        ("compact_ms", C.c_double),
        ("compact_n", C.c_uint64),
        ("backup_select_ms", C.c_double),
        ("backup_select_n", C.c_uint64),
        ("nn_busy_ms", C.c_double),
        ("nn_busy_n", C.c_uint64),
        ("parts", C.c_uint64),
    ]


class oaz_train_config(C.Structure):
    _fields_ = [
        ("blocks", C.c_int32),
        ("max_batch", C.c_int32),
        ("learning_rate", C.c_double),
        ("momentum", C.c_double),
        ("weight_decay", C.c_double),
        ("bn_momentum", C.c_double),
        ("bn_eps", C.c_double),
        ("value_loss_broadcast", C.c_int32),
        ("reserved", C.c_int32 * 7),
    ]


class oaz_pure_mcts_config(C.Structure):
    _fields_ = [
        ("max_playouts", C.c_int32),
        ("min_node_visits", C.c_int32),
        ("exploration_c", C.c_float),
        ("rollout_cap", C.c_int32),
        ("seed", C.c_uint64),
        ("game_id0", C.c_uint64),
        ("device", C.c_int32),
        ("reserved", C.c_int32 * 3),
    ]


class oaz_pure_mcts_stats(C.Structure):
    _fields_ = [(k, C.c_uint64) for k in ("playouts", "expansions", "rollout_plies", "rollout_passes",
                                          "rollouts_capped", "max_nodes", "tree_full")]


class oaz_comm_id(C.Structure):
    _fields_ = [("internal", C.c_char * 128)]


class oaz_comm_stats(C.Structure):
    _fields_ = [
        ("ranks", C.c_int32),
        ("rank", C.c_int32),
        ("allgather_calls", C.c_uint64),
        ("counts_ms", C.c_double),
        ("allgather_ms", C.c_double),
        ("allgather_records", C.c_uint64),
        ("allgather_bytes", C.c_uint64),
        ("own_records", C.c_uint64),
    ]


assert C.sizeof(oaz_state) == 24
assert C.sizeof(oaz_move) == 4
assert C.sizeof(oaz_node) == 32
assert C.sizeof(oaz_sample) == 228
assert C.sizeof(oaz_config) == 120 and oaz_config.search_time_ns.offset == 104

STATE_DTYPE = np.dtype(
    [("kings", "<u4", 2), ("pawns", "<u4", 2), ("cards", "u1", 5), ("to_move", "u1"), ("pad", "u1", 2)]
)
MOVE_DTYPE = np.dtype([("from_", "u1"), ("to", "u1"), ("piece", "u1"), ("slot", "u1")])
NODE_DTYPE = np.dtype(
    [("W", "<f8"), ("P", "<f8"), ("N", "<u4"), ("first", "<u4"), ("mv", "<u2"), ("nch", "u1"),
     ("flags", "u1"), ("pad", "<u4")]
)
SAMPLE_DTYPE = np.dtype([("state", STATE_DTYPE), ("pi", "<f4", 50), ("z", "<f4")])
PURE_NODE_DTYPE = np.dtype([("visits", "<u4"), ("reward", "<f4"), ("winrate", "<f4"), ("first", "<u4"),
                            ("parent", "<u4"), ("mv", "<u2"), ("nch", "u1"), ("flags", "u1")])
assert PURE_NODE_DTYPE.itemsize == 24
assert STATE_DTYPE.itemsize == 24 and NODE_DTYPE.itemsize == 32 and SAMPLE_DTYPE.itemsize == 228

# C prototypes: name -> (restype, argtypes)
_P = C.POINTER
_VOIDP = C.c_void_p
_PROTOS = {
    "oaz_abi_version": (C.c_int, []),
    "oaz_last_error": (C.c_char_p, []),
    "oaz_config_default": (None, [_P(oaz_config)]),
    "oaz_device_count": (C.c_int, [_P(C.c_int)]),
    "oaz_attack_maps": (None, [_VOIDP]),
    "oaz_weight_count": (C.c_size_t, [C.c_int, C.c_int, C.c_int]),
    "oaz_nn_device_bytes": (C.c_size_t, [C.c_int, C.c_int]),
    "oaz_random_weights": (C.c_int, [C.c_uint64, C.c_int, _VOIDP, C.c_size_t]),
    "oaz_deal_deck": (None, [C.c_uint64, C.c_uint64, _VOIDP]),
    "oaz_initial_state": (None, [_VOIDP, _VOIDP]),
    "oaz_slot_game_ids": (C.c_int, [C.c_int, C.c_int, C.c_int, C.c_uint64, _VOIDP]),
    "oaz_hash_eval": (None, [_VOIDP, _VOIDP, _VOIDP]),
    "oaz_root_noise": (C.c_double, [C.c_uint64, C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32, C.c_double, C.c_int]),
    "oaz_movegen": (C.c_int, [_VOIDP, C.c_int, _VOIDP, _VOIDP, _VOIDP]),
    "oaz_step": (C.c_int, [_VOIDP, _VOIDP, C.c_int, _VOIDP]),
    "oaz_current_state": (C.c_int, [_VOIDP, C.c_int, _VOIDP]),
    "oaz_encode": (C.c_int, [_VOIDP, C.c_int, _VOIDP]),
    "oaz_create": (_VOIDP, [_P(oaz_config), C.c_int]),
    "oaz_destroy": (None, [_VOIDP]),
    "oaz_get_config": (C.c_int, [_VOIDP, _P(oaz_config)]),
    "oaz_set_search_params": (C.c_int, [_VOIDP, C.c_int, C.c_double, C.c_int]),
    "oaz_set_search_time": (C.c_int, [_VOIDP, C.c_int64]),
    "oaz_last_sims": (C.c_int, [_VOIDP, _P(C.c_int)]),
    "oaz_search_playouts": (C.c_int, [_VOIDP, _VOIDP, C.c_int]),
    "oaz_load_weights": (C.c_int, [_VOIDP, _VOIDP, C.c_size_t]),
    "oaz_weight_tensor_count": (C.c_size_t, [C.c_int]),
    "oaz_weight_tensor_info": (C.c_int, [C.c_int, C.c_size_t, C.c_char_p, C.c_size_t, _P(C.c_size_t)]),
    "oaz_weights_from_named": (C.c_int, [C.c_int, _VOIDP, _VOIDP, _VOIDP, C.c_size_t, _VOIDP, C.c_size_t]),
    "oaz_load_weights_named": (C.c_int, [_VOIDP, _VOIDP, _VOIDP, _VOIDP, C.c_size_t]),
    "oaz_ot_read": (C.c_int, [C.c_char_p, _VOIDP, C.c_size_t, _P(C.c_size_t), _P(C.c_int)]),
    "oaz_load_ot": (C.c_int, [_VOIDP, C.c_char_p]),
    "oaz_ot_write": (C.c_int, [C.c_char_p, _VOIDP, C.c_size_t, C.c_int]),
    "oaz_checkpoint_path": (C.c_int, [C.c_char_p, C.c_int64, C.c_int, C.c_char_p, C.c_char_p, C.c_size_t]),
    "oaz_sync": (C.c_int, [_VOIDP]),
    "oaz_set_timing": (C.c_int, [_VOIDP, C.c_int]),
    "oaz_kernel_times_get": (C.c_int, [_VOIDP, _P(oaz_kernel_times)]),
    "oaz_kernel_times_reset": (C.c_int, [_VOIDP]),
    "oaz_nn_forward": (C.c_int, [_VOIDP, _VOIDP, C.c_int, _VOIDP, _VOIDP]),
    "oaz_nn_fallbacks": (C.c_int, [_VOIDP, _P(C.c_uint64)]),
    "oaz_search": (C.c_int, [_VOIDP, _VOIDP, C.c_int, _VOIDP, _VOIDP, _VOIDP, _P(oaz_search_stats)]),
    "oaz_tree_dump": (C.c_int, [_VOIDP, C.c_int, _VOIDP, C.c_int, _P(C.c_int)]),
    "oaz_selfplay_reset": (C.c_int, [_VOIDP]),
    "oaz_selfplay_step": (C.c_int, [_VOIDP, C.c_int]),
    "oaz_selfplay_stats_get": (C.c_int, [_VOIDP, _P(oaz_selfplay_stats)]),
    "oaz_samples_fetch": (C.c_int, [_VOIDP, _VOIDP, C.c_size_t, _P(C.c_size_t)]),
    "oaz_samples_export_device": (C.c_int, [_VOIDP, _VOIDP, C.c_size_t, _P(C.c_size_t)]),
    "oaz_selfplay_run": (C.c_int, [_VOIDP, C.c_int, _VOIDP, C.c_size_t, _P(C.c_size_t), _P(oaz_selfplay_stats)]),
    "oaz_comm_unique_id": (C.c_int, [_P(oaz_comm_id)]),
    "oaz_comm_init": (_VOIDP, [_P(oaz_comm_id), C.c_int, C.c_int, C.c_int]),
    "oaz_comm_destroy": (None, [_VOIDP]),
    "oaz_allgather_samples": (C.c_int, [_VOIDP, _VOIDP, _VOIDP, C.c_size_t, _P(C.c_size_t), _VOIDP]),
    "oaz_comm_allreduce_sum_f32": (C.c_int, [_VOIDP, _VOIDP, C.c_size_t, _VOIDP]),
    "oaz_comm_broadcast": (C.c_int, [_VOIDP, _VOIDP, C.c_size_t, C.c_int, _VOIDP]),
    "oaz_comm_sync": (C.c_int, [_VOIDP]),
    "oaz_comm_stats_get": (C.c_int, [_VOIDP, _P(oaz_comm_stats)]),
    "oaz_pure_mcts_config_default": (None, [_P(oaz_pure_mcts_config)]),
    "oaz_pure_mcts_tree_capacity": (C.c_size_t, [_P(oaz_pure_mcts_config)]),
    "oaz_pure_mcts_search": (C.c_int, [_VOIDP, C.c_int, _P(oaz_pure_mcts_config), _VOIDP, _VOIDP,
                                       _P(oaz_pure_mcts_stats), _VOIDP, C.c_size_t]),
    "oaz_pure_mcts_release_workspace": (C.c_int, [C.c_int]),
    "oaz_train_config_default": (None, [_P(oaz_train_config)]),
    "oaz_trainer_create": (_VOIDP, [_P(oaz_train_config), C.c_int]),
    "oaz_trainer_destroy": (None, [_VOIDP]),
    "oaz_trainer_set_stream": (C.c_int, [_VOIDP, _VOIDP]),
    "oaz_trainer_set_weights": (C.c_int, [_VOIDP, _VOIDP, C.c_size_t]),
    "oaz_trainer_get_weights": (C.c_int, [_VOIDP, _VOIDP, C.c_size_t]),
    "oaz_trainer_save_ot": (C.c_int, [_VOIDP, C.c_char_p]),
    "oaz_trainer_load_samples": (C.c_int, [_VOIDP, _VOIDP, C.c_size_t]),
    "oaz_trainer_bind_device_samples": (C.c_int, [_VOIDP, _VOIDP, C.c_size_t]),
    "oaz_trainer_set_batches": (C.c_int, [_VOIDP, _VOIDP, C.c_int, C.c_int]),
    "oaz_trainer_backward": (C.c_int, [_VOIDP, C.c_int]),
    "oaz_trainer_grads": (C.c_int, [_VOIDP, _P(C.c_void_p), _P(C.c_size_t)]),
    "oaz_trainer_get_grads": (C.c_int, [_VOIDP, _VOIDP, C.c_size_t]),
    "oaz_trainer_apply": (C.c_int, [_VOIDP, C.c_float]),
    "oaz_trainer_bn_stats_count": (C.c_size_t, [C.c_int]),
    "oaz_trainer_bn_stats_pack": (C.c_int, [_VOIDP, _VOIDP]),
    "oaz_trainer_bn_stats_unpack": (C.c_int, [_VOIDP, _VOIDP, C.c_float]),
    "oaz_trainer_train": (C.c_int, [_VOIDP, C.c_int, C.c_int]),
    "oaz_trainer_losses": (C.c_int, [_VOIDP, _P(C.c_double * 3)]),
    "oaz_trainer_sync": (C.c_int, [_VOIDP]),
}

EXPORTED_SYMBOLS = tuple(_PROTOS)

_lib = None


def load(path: str | os.PathLike | None = None) -> C.CDLL:
    """Load libonitama_az.so (built in-tree by __graft_entry__.build()). Raises OazError."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    # OAZ_LIB: another in-tree build of the same ABI (the A/B build, `make AB=1`, for tools/ only)
    p = Path(path) if path else Path(os.environ["OAZ_LIB"]) if os.environ.get("OAZ_LIB") else LIB_PATH
    if not p.exists():
        raise OazError(f"{p} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'`")
    lib = C.CDLL(str(p), mode=C.RTLD_GLOBAL)
    for name, (res, args) in _PROTOS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.oaz_abi_version() != ABI_VERSION:
        raise OazError("ABI version mismatch")
    if path is None:
        _lib = lib
    return lib


def check(rc: int) -> None:
    if rc < 0:
        msg = load().oaz_last_error()
        raise OazError(f"C ABI error {rc}: {msg.decode() if msg else ''}")


def ptr(a: np.ndarray) -> C.c_void_p:
    assert a.flags["C_CONTIGUOUS"]
    return C.c_void_p(a.ctypes.data)


def device_count() -> int:
    n = C.c_int(0)
    load().oaz_device_count(C.byref(n))
    return n.value


def default_config() -> oaz_config:
    c = oaz_config()
    load().oaz_config_default(C.byref(c))
    return c
