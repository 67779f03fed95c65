#!/bin/bash
# Training-step bench (bench.py --mode train) + rocprofv3 kernel stats of the same command.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
mkdir -p gpurun_out/prof_train
PY=$(command -v python3)
step() { local name=$1; shift; echo "== $name"; "$@"; local rc=$?; echo "$name rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step train_bench timeout -k 10 300 python bench.py --mode train ${TRAIN_ARGS:-} --steps 200 --warmup 20 --cpu-seconds 10 > gpurun_out/train_bench.log 2>&1
tail -1 gpurun_out/train_bench.log | cut -c1-600
step train_trace timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_train/trace -o run -- "$PY" bench.py --mode train ${TRAIN_ARGS:-} --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/train_trace.log 2>&1
find gpurun_out/prof_train -name "*stats*.csv"
