#!/bin/bash
# Same-box A/B of library builds on bench.py --mode pure_mcts, each build first through the pure-MCTS parity
# tests (trees byte-equal to the oracle):
# LIBS="onitama-alphazero_amd/onitama_az/libonitama_az_prev.so onitama-alphazero_amd/onitama_az/libonitama_az.so" tools/pure_mcts_ab.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
mkdir -p gpurun_out/pm_ab
for L in $LIBS; do
  n=$(basename $L .so)
  OAZ_LIB=$PWD/$L timeout -k 10 300 python -u -m pytest tests/test_pure_mcts.py -x -q -m gpu --timeout 250 --timeout-method thread > gpurun_out/pm_ab/tests_$n.log 2>&1; rc=$?; echo "$n tests: $(tail -1 gpurun_out/pm_ab/tests_$n.log)"; [ $rc -eq 0 ] || exit $rc
done
for r in $(seq 1 ${ROUNDS:-2}); do
  for L in $LIBS; do
    n=$(basename $L .so)
    OAZ_LIB=$PWD/$L timeout -k 10 300 python bench.py --mode pure_mcts --steps 2 --warmup 1 --no-cpu-baseline --no-pmc > gpurun_out/pm_ab/${n}_$r.json 2> gpurun_out/pm_ab/${n}_$r.err || { tail -3 gpurun_out/pm_ab/${n}_$r.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/pm_ab/${n}_$r.json').read().strip().splitlines()[-1]); print('$n', 'round $r', round(d['value']/1e6,1), 'M playouts/s', round(d['ms_per_step'],2), 'ms')"
  done
done
