#!/bin/bash
# FETCH_SIZE and WRITE_SIZE passes (separate) over tools/pmc_cal/pmc_cal (built in-tree beforehand).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
B=$PWD/tools/pmc_cal/pmc_cal
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc_cal/$c -o cal -- $B > gpurun_out/pmc_cal_$c.log 2>&1 || exit 1
done
python3 tools/pmc_cal/analyse.py gpurun_out/pmc_cal
