#!/bin/bash
# Same-box A/B of runtime knobs of the A/B build (libonitama_az_ab.so, OAZ_AB=1): bench.py --mode train
# (batch 512, 5 blocks), ROUNDS interleaved rounds over each setting in $SETTINGS (space-separated
# VAR=value[,VAR=value] lists; OAZ_LIB=<path> in a setting picks another library); test_train.py on the
# product library first (TESTS=1).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
L=$PWD/onitama-alphazero_amd/onitama_az
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 300 python -m pytest tests/test_train.py -x -q -m gpu --timeout 200 --timeout-method thread 2>&1 \
      | tail -1 | sed "s/^/product tests: /" || exit 1
fi
for r in $(seq 1 ${ROUNDS:-3}); do
  for s in $SETTINGS; do
    env OAZ_LIB=$L/libonitama_az_ab.so $(echo "$s" | tr ',' ' ') timeout -k 10 200 python bench.py --mode train \
        --steps 200 --warmup 20 --no-cpu-baseline 2>/dev/null | tail -1 | python -c "
import json, sys
d = json.loads(sys.stdin.read())
print(json.dumps({'setting': '$s', 'round': $r, 'ms_per_step': round(d['ms_per_step'], 4)}))" || exit 1
  done
done
