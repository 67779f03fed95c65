#!/bin/bash
# Same-box A/B of the bf16 (C5) NN kernels of the A/B build: OAZ_NN_BF16_V1 values in VARS, 6-block
# random weights, parity vs the torch goldens + median per-launch ms. VARS="0 5" tools/bf16_ab.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
export OAZ_LIB=$PWD/onitama-alphazero_amd/onitama_az/libonitama_az_ab.so
for v in ${VARS:-0}; do
  OAZ_NN_BF16_V1=$v timeout -k 10 200 python tools/nn_ab.py --precision bf16 --blocks 6 --rounds ${ROUNDS:-2} > gpurun_out/bf16_$v.json 2>&1 || { tail -5 gpurun_out/bf16_$v.json; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/bf16_$v.json'))
print('bf16 v$v', [(k, round(x['median_ms'], 4), x['max_err_vs_torch']) for k, x in d.items()])"
done
