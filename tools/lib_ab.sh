#!/bin/bash
# Same-box A/B of NN kernel builds: alternates tools/nn_ab.py over the given libraries (OAZ_LIB) for
# ROUNDS rounds; prints the median launch time per library and round.
# LIBS="onitama-alphazero_amd/onitama_az/libonitama_az_old.so onitama-alphazero_amd/onitama_az/libonitama_az.so" tools/lib_ab.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
mkdir -p gpurun_out/ab
for r in $(seq 1 ${ROUNDS:-3}); do
  for L in $LIBS; do
    n=$(basename $L .so)
    OAZ_LIB=$PWD/$L OAZ_NN_X6_V=${VAR:-0} timeout -k 10 120 python tools/nn_ab.py --blocks ${BLOCKS:-3} --precision ${PREC:-fp32h3} --x6-variants ${VAR:-0} --rounds 2 --reps ${REPS:-10} > gpurun_out/ab/lib_${n}_$r.json 2>&1 || { tail -3 gpurun_out/ab/lib_${n}_$r.json; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/ab/lib_${n}_$r.json')); print('$n', 'round $r', [round(v['median_ms'],4) for v in d.values()])"
  done
done
