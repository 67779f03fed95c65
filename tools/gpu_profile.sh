#!/bin/bash
# Full-size bench (its own PMC child passes included) + rocprofv3 kernel-trace stats of a short run
# of the same workload. Each step has its own timeout; stops at the first failure.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
TAG=${TAG:-prof}
mkdir -p gpurun_out/prof_$TAG
PY=$(command -v python3)  # absolute path after `--` (rocprofv3 must not exec a PATH lookup)
exec 3>&1  # step messages go to the script's stdout, not into a step's redirected output file
step() { local name=$1; shift; echo "== $name" >&3; "$@"; local rc=$?; echo "$name rc=$rc" >&3; if [ $rc -ne 0 ]; then exit $rc; fi; }
step bench timeout -k 10 900 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
tail -1 gpurun_out/bench_$TAG.json | cut -c1-600
step trace timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG/trace -o run -- "$PY" bench.py --steps 2 --no-cpu-baseline --no-allgather --no-pmc --no-exact ${PROF_ARGS:-} > gpurun_out/prof_$TAG/trace.log 2>&1
find gpurun_out/prof_$TAG -name "*kernel_stats.csv" | head
# the last 2 plies: bench.py ends with the single-stream roofline leg (2 timed plies, one part), whose
# NN launches are the roofline's; the --stats summary also averages every earlier launch
T=$(find gpurun_out/prof_$TAG -name "*kernel_trace.csv" | head -1)
[ -n "$T" ] && python tools/trace_steady.py "$T" $((2 * ${SIMS:-400})) --union k_nn_ --parts 1 > gpurun_out/prof_$TAG/steady_kernel_stats.csv
