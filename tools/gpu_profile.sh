#!/bin/bash
# Full-size bench + rocprofv3 kernel stats + PMC traffic passes (each its own timeout; stop on crash).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
mkdir -p gpurun_out/prof
PY=$(command -v python3)  # absolute path after `--` (rocprofv3 must not exec a PATH lookup)
step() { local name=$1; shift; echo "== $name"; "$@"; local rc=$?; echo "$name rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step bench timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench_full.log 2>&1
tail -1 gpurun_out/bench_full.log | cut -c1-400
step trace timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/trace -o run -- "$PY" bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-allgather --no-pmc ${PROF_ARGS:-} > gpurun_out/prof_trace.log 2>&1
step pmc_fetch timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof/pmc_fetch -o run -- "$PY" bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-allgather --no-pmc --games 8192 --sims 8 > gpurun_out/prof_fetch.log 2>&1
step pmc_write timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof/pmc_write -o run -- "$PY" bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-allgather --no-pmc --games 8192 --sims 8 > gpurun_out/prof_write.log 2>&1
find gpurun_out/prof -name "*.csv" | head -20
