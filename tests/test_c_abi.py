"""The C ABI from a plain C program (tests/c/abi_smoke.c), compiled with gcc against
include/onitama_az.h and linked to the in-tree libonitama_az.so — the way a non-Python host
(the reference's Rust through `extern "C"`) uses the engine."""
import os
import shutil
import subprocess
from pathlib import Path

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
                    f"-Wl,-rpath,{rocm}"], check=True)
    return exe


def _run(exe):
    return subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)


def test_c_host_without_device(tmp_path):
    if _abi.device_count() > 0:
        pytest.skip("a GPU is visible")
    r = _run(_build(tmp_path))
    assert r.returncode == 0, r.stderr
    assert "OK host" in r.stdout and "OK no-device" in r.stdout


@pytest.mark.gpu
def test_c_host_on_gpu(tmp_path):
    r = _run(_build(tmp_path))
    assert r.returncode == 0, r.stdout + r.stderr
    for tag in ("OK search", "OK selfplay", "OK comm", "OK pure_mcts", "OK train"):
        assert tag in r.stdout, r.stdout
