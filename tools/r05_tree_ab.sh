#!/bin/bash
# Round-5 tree-kernel check: parity of the product build (tree, noise and self-play tests, smoke), then a
# same-box A/B of the fused tree kernel between the builds named in $NAMES (tools/tree_ab.sh, single-stream
# C3 with / without root noise) and per-build FETCH_SIZE / WRITE_SIZE passes over it (tools/tree_pmc.sh).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-tree}
L=$PWD/onitama-alphazero_amd/onitama_az
# TEST_LIB: run the parity tests and the smoke on libonitama_az_$TEST_LIB.so instead of the product build
[ -n "${TEST_LIB:-}" ] && export OAZ_LIB=$L/libonitama_az_$TEST_LIB.so
if [ -z "${SKIP_TESTS:-}" ]; then
timeout -k 10 400 python -u -m pytest tests/test_gpu.py tests/test_gpu_scale.py -x -q -m gpu \
    -k "search or selfplay or noise or c3 or c2 or c5" --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/${TAG}_tests.log; [ $rc -ne 0 ] && exit $rc
if [ -z "${TEST_LIB:-}" ]; then  # (the smoke checks that the product build is the one loaded)
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc"; [ $rc -ne 0 ] && exit $rc
fi
fi
unset OAZ_LIB
NAMES="$NAMES" ROUNDS=${ROUNDS:-3} bash tools/tree_ab.sh > gpurun_out/${TAG}_ab.log 2>&1
rc=$?; echo "ab rc=$rc"; [ $rc -ne 0 ] && exit $rc
for n in $NAMES; do
  OAZ_LIB=$L/libonitama_az_$n.so OUT=gpurun_out/${TAG}_pmc_$n SETS="FETCH_SIZE;WRITE_SIZE" bash tools/tree_pmc.sh > gpurun_out/${TAG}_pmc_$n.log 2>&1
  rc=$?; echo "pmc $n rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
