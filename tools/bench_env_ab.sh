#!/bin/bash
# Same-box A/B of runtime knobs of the A/B build (libonitama_az_ab.so, OAZ_AB=1) on a bench.py config:
# ROUNDS interleaved rounds over each setting in $SETTINGS (space-separated VAR=value[,VAR=value] lists), bench.py
# run with $BENCH_ARGS (default: --config c2, no side legs); one JSON summary line per run. OAZ_LIB=<path> in a
# setting picks another library.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
L=$PWD/onitama-alphazero_amd/onitama_az/libonitama_az_ab.so
for r in $(seq 1 ${ROUNDS:-3}); do
  for s in $SETTINGS; do
    env OAZ_LIB=$L $(echo "$s" | tr ',' ' ') timeout -k 10 300 python bench.py \
        ${BENCH_ARGS:---config c2 --no-cpu-baseline --no-exact --no-pmc --no-allgather} 2>/dev/null | tail -1 | python -c "
import json, sys
d = json.loads(sys.stdin.read())
k = d.get('kernel_ms_per_step', {})
print(json.dumps({'setting': '$s', 'round': $r, 'M': round(d['value'] / 1e6, 3), 'ms_per_step': round(d['ms_per_step'], 4),
                  'grp_ms': round(k.get('search_grp') or 0, 4), 'ok': d.get('checks', {}).get('ok')}))" || exit 1
  done
done
