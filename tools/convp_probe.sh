#!/bin/bash
# Persistent-conv timing probe (A/B build): kernel stats of bench.py --mode train with the weight prologue
# skipped (OAZ_CONVP_DBG=1), the unit loop skipped (2), or neither (0). Timing-only: results are wrong
# under 1 and 2.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
PY=$(command -v python3)
L=$PWD/onitama-alphazero_amd/onitama_az/libonitama_az_ab.so
for d in ${DBGS:-0 1 2}; do
  OAZ_CONVP_DBG=$d OAZ_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv \
      -d gpurun_out/convp_probe/d$d -o run -- "$PY" bench.py --mode train --steps 50 --warmup 5 --no-cpu-baseline \
      > gpurun_out/convp_probe_d$d.log 2>&1 || exit 1
  python3 - "$d" <<'PY'
import csv, glob, sys
f = glob.glob(f"gpurun_out/convp_probe/d{sys.argv[1]}/**/run_kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'conv' in r['Name'] or 'wgrad<' in r['Name']:
        print(sys.argv[1], r['Name'][:40], r['Calls'], round(float(r['AverageNs']) / 1e3, 2), round(float(r['MinNs']) / 1e3, 2))
PY
done
