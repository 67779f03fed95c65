#!/bin/bash
# NN parity tests on the product library, then same-box C3 and C5 bench A/Bs against a baseline library:
# LIBS="onitama-alphazero_amd/onitama_az/libonitama_az_prev.so onitama-alphazero_amd/onitama_az/libonitama_az.so"
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu.py tests/test_gpu_scale.py tests/test_gpu_precision.py -x -q -m gpu -k "nn or c3 or c5 or c2 or split16 or selfplay_matches or bitexact" --timeout 300 --timeout-method thread > gpurun_out/w128_tests.log 2>&1; rc=$?; tail -2 gpurun_out/w128_tests.log; [ $rc -eq 0 ] || exit $rc
LIBS="$LIBS" ROUNDS=${ROUNDS:-2} bash tools/lib_bench_ab.sh || exit $?
LIBS="$LIBS" ROUNDS=${ROUNDS:-2} BENCH_ARGS="--config c5" WARMUP=6 STEPS=3 bash tools/lib_bench_ab.sh
