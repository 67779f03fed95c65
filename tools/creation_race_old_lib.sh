#!/bin/bash
# Reproduces profiles/r06a_creation_race_old_lib.log: builds the library of 08b85c8~1 (before engine creation
# zeroed its counters on the engine's own stream) with its own Python package into scratch_old/ (git-ignored),
# here on the CPU; then, on the GPU box, scratch_old/run_old.py runs tests/test_gpu_streams.py against it:
#   bash tools/creation_race_old_lib.sh && gpurun -- 'python -u scratch_old/run_old.py'
set -e
cd "$(dirname "$0")/.."
WT=$(mktemp -d /tmp/oaz_oldwt.XXXX)
git worktree add -f "$WT" 08b85c8~1 >/dev/null
make -C "$WT/onitama-alphazero_amd/csrc" -j8 >/dev/null
rm -rf scratch_old/onitama_az && mkdir -p scratch_old
cp -r "$WT/onitama-alphazero_amd/onitama_az" scratch_old/
rm -rf scratch_old/onitama_az/__pycache__ scratch_old/onitama_az/libonitama_az_ab.so
git worktree remove --force "$WT"
cat > scratch_old/run_old.py <<'PY'
# tests/test_gpu_streams.py against the library of 08b85c8~1 (expected to fail there)
import sys
sys.path.insert(0, "scratch_old")
sys.path.insert(0, "tests")
import onitama_az
print("package:", onitama_az.__file__, flush=True)
import test_gpu_streams as t
try:
    t.test_creation_behind_busy_null_stream_equals_quiet_run()
    print("OLD LIB: test PASSED", flush=True)
except AssertionError as ex:
    print("OLD LIB: test FAILED:", repr(ex)[:2000], flush=True)
PY
echo "scratch_old/ ready"
