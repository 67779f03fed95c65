#!/bin/bash
# GPU parity suite (one process), then smoke. Stops at the first failure/crash/timeout.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-gpu}
timeout -k 10 1000 python -u -m pytest tests -x -v -m gpu --timeout 600 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_$TAG.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke_$TAG.log
exit $rc
