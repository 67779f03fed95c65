#!/bin/bash
# Same-box A/B of builds on BASELINE C2 (bench.py --config c2, no side legs): ROUNDS interleaved rounds over
# onitama_az/libonitama_az_<name>.so for each name in $NAMES; one JSON summary line per run.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
L=$PWD/onitama-alphazero_amd/onitama_az
for r in $(seq 1 ${ROUNDS:-3}); do
  for n in $NAMES; do
    OAZ_LIB=$L/libonitama_az_$n.so timeout -k 10 300 python bench.py --config c2 --no-cpu-baseline --no-exact \
        --no-pmc --no-allgather ${C2_ARGS:-} 2>/dev/null | tail -1 | python -c "
import json, sys
d = json.loads(sys.stdin.read())
print(json.dumps({'lib': '$n', 'round': $r, 'Msims': round(d['value'] / 1e6, 3), 'ms_per_step': round(d['ms_per_step'], 4),
                  'grp_ms': round(d['kernel_ms_per_step'].get('search_grp') or 0, 4), 'ok': d['checks']['ok']}))" || exit 1
  done
done
