#!/bin/bash
# Same-box A/B of bench.py runs: AB="var:split var:split ..." (OAZ_NN_X6_V : OAZ_SPLIT_HALVES)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
for cfg in ${AB:-0:0 11:0}; do v=${cfg%%:*}; sp=${cfg##*:}
  OAZ_NN_X6_V=$v OAZ_SPLIT_HALVES=$sp timeout -k 10 240 python bench.py --no-cpu-baseline --no-pmc --no-allgather ${BENCH_ARGS:-} > gpurun_out/abb_${v}_${sp}.log 2>&1 || exit $?
  tail -1 gpurun_out/abb_${v}_${sp}.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v $sp', round(d['value']/1e6,3), round(d['roofline']['avg_launch_ms'],4), {k: round(x,1) for k,x in d['kernel_ms_per_step'].items()})"
done
