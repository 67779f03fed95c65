#!/bin/bash
# End-of-session check in one GPU call: parity suite + smoke (tools/gpu_tests.sh), the default bench
# with its rocprofv3 trace (tools/gpu_profile.sh), then the other modes' lines. Each step has its own
# time limit; the call stops at the first failure.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
TAG=${TAG:-final}
TAG=$TAG bash tools/gpu_tests.sh || exit $?
TAG=$TAG bash tools/gpu_profile.sh || exit $?
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t python bench.py "$@" > gpurun_out/${name}_$TAG.json 2> gpurun_out/${name}_$TAG.err; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
[ -n "$SKIP_MODES" ] && exit 0
run c5 600 --config c5
run c2 300 --config c2
run train 300 --mode train --cpu-seconds 10
run pure_mcts 300 --mode pure_mcts --steps 2 --warmup 1 --cpu-seconds 10
run arena 300 --mode arena --steps 1 --cpu-seconds 10
