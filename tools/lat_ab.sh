#!/bin/bash
# Same-box A/B of library builds on the Agent-API latency (one position, 400 playouts, tools/search_latency.py),
# each build first through the agent / one-launch / budget GPU tests:
# LIBS="onitama-alphazero_amd/onitama_az/libonitama_az_prev.so onitama-alphazero_amd/onitama_az/libonitama_az.so" tools/lat_ab.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
mkdir -p gpurun_out/lat_ab
for L in $LIBS; do
  n=$(basename $L .so)
  OAZ_LIB=$PWD/$L timeout -k 10 300 python -u -m pytest tests/test_gpu_agent.py tests/test_gpu.py -x -q -m gpu -k "agent or one_launch or time_budget" --timeout 250 --timeout-method thread > gpurun_out/lat_ab/tests_$n.log 2>&1; rc=$?; echo "$n tests: $(tail -1 gpurun_out/lat_ab/tests_$n.log)"; [ $rc -eq 0 ] || exit $rc
done
for r in 1 2; do for L in $LIBS; do
  n=$(basename $L .so)
  OAZ_LIB=$PWD/$L OAZ_LAT_G=1 OAZ_LAT_BUDGETS=0 timeout -k 10 300 python tools/search_latency.py 400 10 > gpurun_out/lat_ab/${n}_$r.json 2> gpurun_out/lat_ab/${n}_$r.err || { tail -3 gpurun_out/lat_ab/${n}_$r.err; exit 1; }
  echo "$n round $r: $(tail -c 400 gpurun_out/lat_ab/${n}_$r.json | tr '\n' ' ')"
done; done
