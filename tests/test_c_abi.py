"""The C ABI from a plain C program (tests/c/abi_smoke.c), compiled with gcc against
include/onitama_az.h and linked to the in-tree libonitama_az.so — the way a non-Python host
(the reference's Rust through `extern "C"`) uses the engine."""
import os
import re
import shutil
import subprocess
from pathlib import Path

import numpy as np
import pytest

from onitama_az import _abi

ROOT = Path(__file__).resolve().parents[1]


def _build(tmp_path) -> Path:
    cc = shutil.which("gcc") or shutil.which("cc")
    if cc is None:
        pytest.skip("no C compiler")
    exe = tmp_path / "abi_smoke"
    lib_dir = _abi.LIB_PATH.parent
    rocm = Path(os.environ.get("ROCM_PATH", "/opt/rocm")) / "lib"
    subprocess.run([cc, "-O1", "-Wall", "-o", str(exe), str(ROOT / "tests/c/abi_smoke.c"), f"-I{ROOT / 'include'}",
                    f"-L{lib_dir}", "-lonitama_az", f"-Wl,-rpath,{lib_dir}", f"-L{rocm}", "-lamdhip64",
                    f"-Wl,-rpath,{rocm}", "-lm"], check=True)
    return exe


def _model_files(tmp_path):
    """The reference's trained 3-block network as a VarStore .ot archive (weights.write_ot, tensors
    in a non-canonical order) and the torch-CPU goldens of it (tests/golden/nn_golden.npz) as
    golden.bin: int32 n, n states, n x 50 policy, n values."""
    from onitama_az.weights import named_from_blob, write_ot
    blob = np.load(ROOT / "tests/golden/weights_3block_trained.npy")
    named = named_from_blob(blob, 3)
    order = sorted(named, key=lambda k: (len(k), k[::-1]))  # not the creation order
    ot = tmp_path / "model_3block.ot"
    write_ot(str(ot), {k: named[k] for k in order})
    g = np.load(ROOT / "tests/golden/nn_golden.npz")
    gold = tmp_path / "golden.bin"
    with open(gold, "wb") as f:
        f.write(np.int32(len(g["states"])).tobytes())
        f.write(np.ascontiguousarray(g["states"]).tobytes())
        f.write(np.ascontiguousarray(g["policy_trained3"], dtype="<f4").tobytes())
        f.write(np.ascontiguousarray(g["value_trained3"], dtype="<f4").tobytes())
    return ot, gold


def _run(exe, *args, env=None, timeout=300):
    return subprocess.run([str(exe), *map(str, args)], capture_output=True, text=True, timeout=timeout, env=env)


def _rccl_symbols():
    """The RCCL entry points the product resolves with dlsym (csrc/oaz_comm.cpp rccl_load)."""
    src = (ROOT / "onitama-alphazero_amd/csrc/oaz_comm.cpp").read_text()
    names = re.findall(r'sym\(h, "(\w+)"', src)
    assert len(names) == 10, names
    return names


def _build_multirank(tmp_path):
    """tests/c/rccl_stub.c as tmp/librccl.so.1 (soname librccl.so.1) and tests/c/comm_multirank.c
    linked to it and to libonitama_az.so. The stub is a NEEDED library of the program, so the
    engine's dlopen("librccl.so.1") returns the stub already mapped (same soname); the run also puts
    its directory first on LD_LIBRARY_PATH."""
    cc = shutil.which("gcc") or shutil.which("cc")
    if cc is None:
        pytest.skip("no C compiler")
    rocm = Path(os.environ.get("ROCM_PATH", "/opt/rocm")) / "lib"
    stub = tmp_path / "librccl.so.1"
    subprocess.run([cc, "-O1", "-Wall", "-shared", "-fPIC", "-o", str(stub), "-Wl,-soname,librccl.so.1",
                    str(ROOT / "tests/c/rccl_stub.c"), f"-L{rocm}", "-lamdhip64", f"-Wl,-rpath,{rocm}", "-lpthread"],
                   check=True)
    exe = tmp_path / "comm_multirank"
    lib_dir = _abi.LIB_PATH.parent
    subprocess.run([cc, "-O1", "-Wall", "-o", str(exe), str(ROOT / "tests/c/comm_multirank.c"), f"-I{ROOT / 'include'}",
                    f"-L{lib_dir}", "-lonitama_az", f"-Wl,-rpath,{lib_dir}", f"-L{tmp_path}", "-l:librccl.so.1",
                    f"-Wl,-rpath,{tmp_path}", f"-L{rocm}", "-lamdhip64", f"-Wl,-rpath,{rocm}", "-lpthread"],
                   check=True)
    env = dict(os.environ, LD_LIBRARY_PATH=f"{tmp_path}:" + os.environ.get("LD_LIBRARY_PATH", ""))
    return stub, exe, env


def _check_written_checkpoint(out_dir):
    """The checkpoint the C program wrote (oaz_ot_write, save_vs naming) is byte-equal to the Python
    restatement of the writer (weights.write_ot, Python's zipfile) for the same tensors, and reads back
    through the Python safe reader."""
    from onitama_az.weights import named_from_blob, read_ot, write_ot, blob_from_named
    blob = np.load(ROOT / "tests/golden/weights_3block_trained.npy")
    p = out_dir / "best_model_7_20260101_120000.ot"
    assert p.exists(), sorted(out_dir.iterdir())
    ref_dir = out_dir / "py"
    ref_dir.mkdir()
    write_ot(str(ref_dir / p.name), named_from_blob(blob, 3))
    assert p.read_bytes() == (ref_dir / p.name).read_bytes()
    assert np.array_equal(blob_from_named(read_ot(str(p)), 3), blob)


def test_c_host_without_device(tmp_path):
    if _abi.device_count() > 0:
        pytest.skip("a GPU is visible")
    out = tmp_path / "ckpt"
    out.mkdir()
    r = _run(_build(tmp_path), *_model_files(tmp_path), out)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "OK host" in r.stdout and "OK model-host" in r.stdout and "OK no-device" in r.stdout
    assert "OK ot-write" in r.stdout
    _check_written_checkpoint(out)


@pytest.mark.gpu
def test_c_host_on_gpu(tmp_path):
    out = tmp_path / "ckpt"
    out.mkdir()
    r = _run(_build(tmp_path), *_model_files(tmp_path), out)
    assert r.returncode == 0, r.stdout + r.stderr
    for tag in ("OK model-host", "OK ot-write", "OK model ", "OK search", "OK selfplay", "OK comm", "OK pure_mcts",
                "OK train", "OK trainer-save"):
        assert tag in r.stdout, r.stdout
    _check_written_checkpoint(out)


def test_rccl_stub_exports_what_the_product_resolves(tmp_path):
    """The multi-rank test double exports every RCCL symbol oaz_comm.cpp dlsym()s (CPU: build + nm)."""
    stub, exe, _ = _build_multirank(tmp_path)
    nm = subprocess.run(["nm", "-D", "--defined-only", str(stub)], capture_output=True, text=True, check=True).stdout
    exported = {ln.split()[-1] for ln in nm.splitlines() if ln.strip()}
    missing = [s for s in _rccl_symbols() if s not in exported]
    assert not missing, missing
    assert exe.exists()


@pytest.mark.gpu
@pytest.mark.parametrize("world,delay_us", [(2, 0), (3, 0), (4, 0), (8, 0), (3, 3000), (8, 1000)])
def test_c_allgather_samples_multirank(tmp_path, world, delay_us):
    """The product exchange (oaz_allgather_samples, oaz_comm_broadcast, oaz_comm_allreduce_sum_f32) at
    world 2, 3, 4 and 8 (the C4 node's rank count): ranks are threads of one plain C process on GPU 0 over the RCCL test double
    (tests/c/rccl_stub.c), which is asynchronous as RCCL is: each collective is enqueued on the caller's
    stream and runs later on a proxy thread, so the results also test the product's stream ordering.
    Ragged counts with a zero-count rank, the capacity error, a local failure on one rank seen by every
    rank (kLocalFailure), and every rank's output byte-equal to the rank-order concatenation
    (train.rs:241-244). With delay_us the stub sleeps that long on each stream before an operation's copies,
    so every call returns well before its data moves (all of them counted as pending). See
    tests/c/comm_multirank.c."""
    _, exe, env = _build_multirank(tmp_path)
    env["RCCL_STUB_DELAY_US"] = str(delay_us)
    r = _run(exe, world, env=env, timeout=100)  # (the stub's own rendezvous timeout is 60 s)
    assert r.returncode == 0, r.stdout + r.stderr
    for rank in range(world):
        assert f"OK rank {rank}:" in r.stdout, r.stdout
    m = re.search(rf"OK multirank {world} \((\d+) stub collectives, (\d+) calls returned before", r.stdout)
    assert m, r.stdout
    ops, pending = int(m.group(1)), int(m.group(2))
    # per rank: 4 counts all-gathers, W - 1 grouped broadcasts, W broadcasts, 2 all-reduces; most of them
    # (the ones that move bytes on the GPU) usually still pending when the call returned
    assert ops >= world * (5 + 2 * world) and pending > 0, r.stdout
    if delay_us:  # every operation that moves bytes on a rank: the counts all-gathers, the root's peers' copies
        assert pending >= world * 4, r.stdout
    print(r.stdout)


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_c_allgather_samples_c4_volume_world8(tmp_path):
    """The C4 exchange at its own volume on one GPU: 8 ranks (threads of one C process over the asynchronous
    RCCL test double), each with BASELINE C4's 65,536 self-play slots (HASH evaluator, 2 simulations, root noise
    on, games cut after 20 plies, 30 plies). Every rank receives more than 2^31 bytes of (s, pi, z) records
    (~9.8 M records), and its device output is byte-equal to the rank-order concatenation of the ranks' twin
    engines' oaz_samples_fetch (train.rs:241-244), so 64-bit offsets and counts hold past 2^31 bytes and
    2^31 / 228 records."""
    _, exe, env = _build_multirank(tmp_path)
    env["RCCL_STUB_DELAY_US"] = "0"
    r = _run(exe, 8, "c4", env=env, timeout=500)
    assert r.returncode == 0, r.stdout + r.stderr
    for rank in range(8):
        assert f"OK rank {rank}:" in r.stdout, r.stdout
    assert "OK multirank 8 c4" in r.stdout, r.stdout
    gb = [float(x) for x in re.findall(r"records \(([0-9.]+) GB\) gathered", r.stdout)]
    assert len(gb) == 8 and min(gb) > 2 ** 31 * 1e-9, r.stdout
    print(r.stdout)
