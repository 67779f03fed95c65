#!/bin/bash
# Same-box A/B of the C3 bench (short, no baselines/PMC) over environment settings of the A/B build:
# ENVS="OAZ_TREE_FUSE=0 OAZ_TREE_FUSE=1" ROUNDS=3 tools/bench_ab.sh  -> value and ms_per_step per run
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
mkdir -p gpurun_out/bench_ab
export OAZ_LIB=$PWD/onitama-alphazero_amd/onitama_az/libonitama_az_ab.so
for r in $(seq 1 ${ROUNDS:-3}); do
  for E in $ENVS; do
    env $E timeout -k 10 300 python bench.py --steps ${STEPS:-4} --warmup ${WARMUP:-14} --no-cpu-baseline --no-exact --no-pmc --no-allgather ${BENCH_ARGS:-} > gpurun_out/bench_ab/${E}_$r.json 2> gpurun_out/bench_ab/${E}_$r.err || { tail -3 gpurun_out/bench_ab/${E}_$r.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/bench_ab/${E}_$r.json').read().strip().splitlines()[-1]); print('$E', 'round $r', round(d['value']/1e6,3), 'M sims/s', round(d['ms_per_step'],2), 'ms', {k: (round(v,2) if v else v) for k,v in d['kernel_ms_per_step'].items()})"
  done
done
