"""The C ABI from a plain C program (tests/c/abi_smoke.c), compiled with gcc against
include/onitama_az.h and linked to the in-tree libonitama_az.so — the way a non-Python host
(the reference's Rust through `extern "C"`) uses the engine."""
import os
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


def _run(exe, *args):
    return subprocess.run([str(exe), *map(str, args)], capture_output=True, text=True, timeout=300)


def test_c_host_without_device(tmp_path):
    if _abi.device_count() > 0:
        pytest.skip("a GPU is visible")
    r = _run(_build(tmp_path), *_model_files(tmp_path))
    assert r.returncode == 0, r.stdout + r.stderr
    assert "OK host" in r.stdout and "OK model-host" in r.stdout and "OK no-device" in r.stdout


@pytest.mark.gpu
def test_c_host_on_gpu(tmp_path):
    r = _run(_build(tmp_path), *_model_files(tmp_path))
    assert r.returncode == 0, r.stdout + r.stderr
    for tag in ("OK model-host", "OK model ", "OK search", "OK selfplay", "OK comm", "OK pure_mcts", "OK train"):
        assert tag in r.stdout, r.stdout
