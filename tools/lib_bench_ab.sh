#!/bin/bash
# Same-box A/B of whole library builds on the C3 bench (short, no baselines/PMC):
# LIBS="onitama-alphazero_amd/onitama_az/libonitama_az_prev.so onitama-alphazero_amd/onitama_az/libonitama_az.so" ROUNDS=2 tools/lib_bench_ab.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
mkdir -p gpurun_out/lib_bench_ab
for r in $(seq 1 ${ROUNDS:-2}); do
  for L in $LIBS; do
    n=$(basename $L .so)
    OAZ_LIB=$PWD/$L timeout -k 10 300 python bench.py --steps ${STEPS:-4} --warmup ${WARMUP:-14} --no-cpu-baseline --no-exact --no-pmc --no-allgather ${BENCH_ARGS:-} > gpurun_out/lib_bench_ab/${n}_$r.json 2> gpurun_out/lib_bench_ab/${n}_$r.err || { tail -3 gpurun_out/lib_bench_ab/${n}_$r.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/lib_bench_ab/${n}_$r.json').read().strip().splitlines()[-1]); print('$n', 'round $r', round(d['value']/1e6,3), 'M sims/s', round(d['ms_per_step'],2), 'ms', {k: (round(v,2) if v else v) for k,v in d['kernel_ms_per_step'].items()})"
  done
done
