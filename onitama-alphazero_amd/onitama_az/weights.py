"""Weights: canonical blob order, random init, and a safe reader for the reference's .ot files.

Canonical order = the order in which the reference's tch VarStore creates the variables
(net.rs:101-213), with tch's '|'-joined names:
    conv_init_1|{weight,bias}, bn1|{weight,bias,running_mean,running_var},
    resnet_{i}|resnet_small_block{1,2}|small_block_conv|{weight,bias},
    resnet_{i}|resnet_small_block{1,2}|small_block_bn|{weight,bias,running_mean,running_var},
    vh_conv|..., vh_bn|..., vh_linear1|..., vh_linear2|...,
    policy_conv|..., policy_bn|..., ph_linear2|...

The .ot files (TorchScript zip archives written by VarStore::save) are read WITHOUT unpickling
or executing anything: data.pkl is walked opcode by opcode with pickletools.genops and only
the (name -> storage key, shape, stride, offset) records are interpreted; tensor bytes come
straight from the stored zip members (little-endian f32).
"""
from __future__ import annotations

import ctypes as C
import pickletools
import zipfile
from typing import Dict, List, Tuple

import numpy as np

from . import _abi

CH, INP = 64, 21
_BN = ("weight", "bias", "running_mean", "running_var")


def canonical_layout(blocks: int) -> List[Tuple[str, Tuple[int, ...]]]:
    out: List[Tuple[str, Tuple[int, ...]]] = []

    def conv(name, cout, cin, k):
        out.append((f"{name}|weight", (cout, cin, k, k)))
        out.append((f"{name}|bias", (cout,)))

    def bn(name, c):
        out.extend((f"{name}|{f}", (c,)) for f in _BN)

    conv("conv_init_1", CH, INP, 3)
    bn("bn1", CH)
    for i in range(blocks):
        for j in (1, 2):
            p = f"resnet_{i}|resnet_small_block{j}"
            conv(f"{p}|small_block_conv", CH, CH, 3)
            bn(f"{p}|small_block_bn", CH)
    conv("vh_conv", 1, CH, 1)
    bn("vh_bn", 1)
    out.append(("vh_linear1|weight", (CH, 25)))
    out.append(("vh_linear1|bias", (CH,)))
    out.append(("vh_linear2|weight", (1, CH)))
    out.append(("vh_linear2|bias", (1,)))
    conv("policy_conv", 2, CH, 1)
    bn("policy_bn", 2)
    out.append(("ph_linear2|weight", (50, 50)))
    out.append(("ph_linear2|bias", (50,)))
    return out


def weight_count(blocks: int) -> int:
    return int(sum(int(np.prod(s)) for _, s in canonical_layout(blocks)))


def blob_from_named(named: Dict[str, np.ndarray], blocks: int) -> np.ndarray:
    parts = []
    for name, shape in canonical_layout(blocks):
        if name not in named:
            raise KeyError(f"missing tensor {name}")
        a = np.asarray(named[name], dtype=np.float32)
        if tuple(a.shape) != shape:
            raise ValueError(f"{name}: shape {a.shape} != {shape}")
        parts.append(a.reshape(-1))
    return np.ascontiguousarray(np.concatenate(parts))


def named_from_blob(blob: np.ndarray, blocks: int) -> Dict[str, np.ndarray]:
    out, off = {}, 0
    for name, shape in canonical_layout(blocks):
        n = int(np.prod(shape))
        out[name] = blob[off: off + n].reshape(shape)
        off += n
    assert off == len(blob)
    return out


def random_weights(seed: int, blocks: int) -> np.ndarray:
    """The engine's random init (oaz_random_weights): U(+-1/sqrt(fan_in)), BN identity."""
    n = weight_count(blocks)
    w = np.zeros(n, dtype=np.float32)
    _abi.check(_abi.load().oaz_random_weights(C.c_uint64(seed), blocks, _abi.ptr(w), n))
    return w


def blocks_from_names(names) -> int:
    idx = {int(n.split("|")[0].split("_")[1]) for n in names if n.startswith("resnet_")}
    return (max(idx) + 1) if idx else 0


# ---- through the C ABI (the product path of model loading) ---------------------------------------
def ot_blob(path: str) -> Tuple[np.ndarray, int]:
    """(canonical blob, blocks) of a VarStore .ot archive, read by the library's C reader
    (oaz_ot_read: restricted pickle machine, nothing executed)."""
    lib = _abi.load()
    n, blocks = C.c_size_t(0), C.c_int(0)
    _abi.check(lib.oaz_ot_read(str(path).encode(), None, 0, C.byref(n), C.byref(blocks)))
    out = np.zeros(n.value, dtype=np.float32)
    _abi.check(lib.oaz_ot_read(str(path).encode(), _abi.ptr(out), out.size, C.byref(n), C.byref(blocks)))
    return out, int(blocks.value)


def tensor_table(blocks: int) -> List[Tuple[str, int]]:
    """The library's canonical (name, numel) table (oaz_weight_tensor_info)."""
    lib = _abi.load()
    out = []
    for i in range(lib.oaz_weight_tensor_count(blocks)):
        name, n = C.create_string_buffer(128), C.c_size_t(0)
        _abi.check(lib.oaz_weight_tensor_info(blocks, i, name, 128, C.byref(n)))
        out.append((name.value.decode(), int(n.value)))
    return out


def blob_from_named_c(named: Dict[str, np.ndarray], blocks: int) -> np.ndarray:
    """oaz_weights_from_named: tensors placed by name (either '|' or '.' separators)."""
    keep = [np.ascontiguousarray(v, dtype=np.float32).reshape(-1) for v in named.values()]
    names = (C.c_char_p * len(keep))(*[k.encode() for k in named])
    data = (C.c_void_p * len(keep))(*[a.ctypes.data for a in keep])
    sizes = (C.c_size_t * len(keep))(*[a.size for a in keep])
    out = np.zeros(weight_count(blocks), dtype=np.float32)
    _abi.check(_abi.load().oaz_weights_from_named(blocks, names, data, sizes, len(keep), _abi.ptr(out), out.size))
    return out


# ---- safe .ot reader (Python restatement, a cross-check of the C reader) -----------------------------
class _Sym:
    """Symbolic stand-in for a pickle GLOBAL/REDUCE result (never resolved or called)."""

    def __init__(self, name, args=None):
        self.name, self.args = name, args


def _walk_pickle(data: bytes):
    """Interpret a restricted opcode subset into plain Python values; nothing is imported."""
    stack, memo, marks = [], {}, []
    for op, arg, _pos in pickletools.genops(data):
        n = op.name
        if n in ("PROTO", "FRAME", "STOP"):
            continue
        if n in ("BINUNICODE", "SHORT_BINUNICODE", "BININT1", "BININT2", "BININT", "LONG1",
                 "BINFLOAT", "SHORT_BINSTRING", "BINSTRING", "UNICODE", "INT"):
            stack.append(arg)
        elif n == "NEWTRUE":
            stack.append(True)
        elif n == "NEWFALSE":
            stack.append(False)
        elif n == "NONE":
            stack.append(None)
        elif n == "GLOBAL":
            stack.append(_Sym(arg))
        elif n in ("BINPUT", "LONG_BINPUT"):
            memo[arg] = stack[-1]
        elif n == "MEMOIZE":
            memo[len(memo)] = stack[-1]
        elif n in ("BINGET", "LONG_BINGET"):
            stack.append(memo[arg])
        elif n == "MARK":
            marks.append(len(stack))
        elif n == "TUPLE":
            k = marks.pop()
            t = tuple(stack[k:])
            del stack[k:]
            stack.append(t)
        elif n == "EMPTY_TUPLE":
            stack.append(())
        elif n == "TUPLE1":
            stack[-1:] = [tuple(stack[-1:])]
        elif n == "TUPLE2":
            stack[-2:] = [tuple(stack[-2:])]
        elif n == "TUPLE3":
            stack[-3:] = [tuple(stack[-3:])]
        elif n == "EMPTY_DICT":
            stack.append({})
        elif n == "EMPTY_LIST":
            stack.append([])
        elif n == "SETITEMS":
            k = marks.pop()
            items = stack[k:]
            del stack[k:]
            d = stack[-1]
            if isinstance(d, dict):
                for i in range(0, len(items), 2):
                    d[items[i]] = items[i + 1]
        elif n == "SETITEM":
            v = stack.pop()
            key = stack.pop()
            if isinstance(stack[-1], dict):
                stack[-1][key] = v
        elif n == "APPENDS":
            k = marks.pop()
            items = stack[k:]
            del stack[k:]
            if isinstance(stack[-1], list):
                stack[-1].extend(items)
        elif n == "APPEND":
            v = stack.pop()
            if isinstance(stack[-1], list):
                stack[-1].append(v)
        elif n == "BINPERSID":
            stack.append(_Sym("persid", stack.pop()))
        elif n in ("REDUCE", "NEWOBJ"):
            args = stack.pop()
            f = stack.pop()
            stack.append(_Sym(getattr(f, "name", "?"), args))
        elif n == "BUILD":
            state = stack.pop()
            obj = stack[-1]
            if isinstance(obj, _Sym) and isinstance(state, dict):
                obj.args = (obj.args, state)
        else:
            raise ValueError(f"unsupported pickle opcode {n}")
    return stack[-1] if stack else None


def _find_tensors(obj, out):
    """name -> _rebuild_tensor_v2 args from every dict reachable from obj; iterative, and every
    container is expanded once (memo aliasing can make shared or cyclic containers)."""
    todo, seen = [obj], set()
    while todo:
        o = todo.pop()
        if not isinstance(o, (dict, list, tuple, _Sym)) or id(o) in seen:
            continue
        seen.add(id(o))
        if isinstance(o, dict):
            for k, v in o.items():
                if isinstance(v, _Sym) and v.name == "torch._utils _rebuild_tensor_v2":
                    out[k] = v.args
                else:
                    todo.append(v)
        elif isinstance(o, _Sym):
            todo.append(o.args)
        else:
            todo.extend(o)


def read_ot(path: str) -> Dict[str, np.ndarray]:
    """Named fp32 tensors of a tch VarStore .ot archive (VarStore::save, train.rs:414-430)."""
    z = zipfile.ZipFile(path)
    pkl = [n for n in z.namelist() if n.endswith("/data.pkl") or n == "data.pkl"]
    if not pkl:
        raise ValueError(f"{path}: no data.pkl")
    root = pkl[0][: -len("data.pkl")]
    obj = _walk_pickle(z.read(pkl[0]))
    recs: Dict[str, tuple] = {}
    _find_tensors(obj, recs)
    out = {}
    for name, args in recs.items():
        # args = (persistent_id, offset, shape, stride, requires_grad, hooks)
        # persistent_id.args = ('storage', <GLOBAL torch FloatStorage>, key, location, numel)
        pers, offset, shape, stride = args[0], args[1], tuple(args[2]), tuple(args[3])
        storage_type = pers.args[1].name if isinstance(pers.args[1], _Sym) else ""
        if storage_type != "torch FloatStorage":
            raise ValueError(f"{name}: unsupported storage {storage_type}")
        key = pers.args[2]
        raw = np.frombuffer(z.read(f"{root}data/{key}"), dtype="<f4")
        n = int(np.prod(shape)) if shape else 1
        a = np.lib.stride_tricks.as_strided(raw[offset:], shape=shape, strides=tuple(4 * s for s in stride)) \
            if shape else raw[offset: offset + 1].reshape(())
        out[name] = np.array(a, dtype=np.float32).reshape(shape)
        assert out[name].size == n
    return out


# ---- .ot writer (train.rs:414-430 save_vs) -------------------------------------------------------
# The product writer is the library's (oaz_ot_write, through save_blob_ot / Trainer.save_ot); the
# Python writer below is an independent restatement of the same archive (Python's zipfile, a
# different zip implementation), kept to write archives from arbitrary named tensors in tests and
# to cross-check the C writer byte for byte (tests/test_host.py).
def _pk_str(s: str) -> bytes:
    b = s.encode("utf-8")
    return b"X" + len(b).to_bytes(4, "little") + b


def _pk_int(v: int) -> bytes:
    if 0 <= v < 256:
        return b"K" + bytes([v])
    if 0 <= v < 65536:
        return b"M" + v.to_bytes(2, "little")
    return b"J" + int(v).to_bytes(4, "little", signed=True)


def _pk_tuple(items) -> bytes:
    return b"(" + b"".join(items) + b"t"


def _data_pkl(entries: List[Tuple[str, Tuple[int, ...]]]) -> bytes:
    """The TorchScript module pickle of a tch VarStore (protocol 2): a `__torch__ Module` whose
    state dict maps each '|' name to torch._utils._rebuild_tensor_v2(storage '<i>', 0, shape,
    contiguous stride, False, OrderedDict())."""
    out = [b"\x80\x02", b"c__torch__\nModule\n", b")\x81}("]
    for i, (name, shape) in enumerate(entries):
        numel = int(np.prod(shape)) if shape else 1
        stride, acc = [], 1
        for d in reversed(shape):
            stride.append(acc)
            acc *= d
        stride.reverse()
        pers = _pk_tuple([_pk_str("storage"), b"ctorch\nFloatStorage\n", _pk_str(str(i)), _pk_str("cpu"),
                          _pk_int(numel)]) + b"Q"
        args = _pk_tuple([pers, _pk_int(0), _pk_tuple([_pk_int(d) for d in shape]),
                          _pk_tuple([_pk_int(s) for s in stride]), b"\x89",
                          b"ccollections\nOrderedDict\n)R"])
        out.append(_pk_str(name) + b"ctorch._utils\n_rebuild_tensor_v2\n" + args + b"R")
    out.append(b"ub.")
    return b"".join(out)


def _torch_py(names: List[str]) -> bytes:
    lines = ["class Module(Module):",
             "  __parameters__ = [" + "".join(f'"{n}", ' for n in names) + "]",
             "  __buffers__ = []",
             "  __annotations__ = []"]
    lines += [f'  __annotations__["{n}"] = Tensor' for n in names]
    return ("\n".join(lines) + "\n").encode()


class _AlignedZip:
    """Stored zip members whose data start on 64-byte boundaries (the torch archive convention,
    padding carried in an 'FB' extra field), so readers may mmap the tensors."""

    def __init__(self, path: str):
        self.z = zipfile.ZipFile(path, "w", compression=zipfile.ZIP_STORED)

    def add(self, name: str, data: bytes):
        info = zipfile.ZipInfo(name, date_time=(1980, 1, 1, 0, 0, 0))
        info.compress_type = zipfile.ZIP_STORED
        start = self.z.fp.tell() + 30 + len(name.encode())
        pad = (-(start + 4)) % 64
        info.extra = b"FB" + pad.to_bytes(2, "little") + b"Z" * pad
        self.z.writestr(info, data)

    def close(self):
        self.z.close()


def write_ot(path: str, named: Dict[str, np.ndarray], archive: str = None) -> None:
    """Write named fp32 tensors as a tch VarStore .ot archive (TorchScript zip: data/<i>, data.pkl,
    code/__torch__.py, constants.pkl, version; every member stored), the format read_ot and the
    reference's VarStore::load read. Python restatement of oaz_ot_write (see above)."""
    import os
    archive = archive or os.path.splitext(os.path.basename(path))[0]
    names = list(named)
    entries = [(n, tuple(np.asarray(named[n]).shape)) for n in names]
    z = _AlignedZip(path)
    try:
        for i, n in enumerate(names):
            z.add(f"{archive}/data/{i}", np.ascontiguousarray(named[n], dtype="<f4").tobytes())
        z.add(f"{archive}/data.pkl", _data_pkl(entries))
        z.add(f"{archive}/code/__torch__.py", _torch_py(names))
        z.add(f"{archive}/constants.pkl", b"\x80\x02).")
        z.add(f"{archive}/version", b"3\n")
    finally:
        z.close()


def checkpoint_path(folder: str, iteration: int, is_best: bool, stamp: str = None) -> str:
    """save_vs naming (train.rs:414-422): <folder>/[best_]model_<iter>_<YYYYmmdd_HHMMSS>.ot, by the
    library (oaz_checkpoint_path); stamp None = the local time now."""
    buf = C.create_string_buffer(4096)
    _abi.check(_abi.load().oaz_checkpoint_path(str(folder).encode(), int(iteration), int(bool(is_best)),
                                               None if stamp is None else str(stamp).encode(), buf, len(buf)))
    return buf.value.decode()


def save_blob_ot(path: str, blob: np.ndarray, blocks: int) -> None:
    """A canonical blob as a .ot checkpoint, written by the library (oaz_ot_write)."""
    b = np.ascontiguousarray(blob, dtype=np.float32)
    _abi.check(_abi.load().oaz_ot_write(str(path).encode(), _abi.ptr(b), b.size, int(blocks)))
