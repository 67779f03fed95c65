#!/bin/bash
# Same-box NN A/B over OAZ_NN_X6_V variants of the A/B build (parity vs the torch goldens + per-launch
# ms), then per-wave phase stamps of the given timing variants. VARS="0 23" PHASES="10 26" tools/stg_ab.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
export OAZ_LIB=$PWD/onitama-alphazero_amd/onitama_az/libonitama_az_ab.so
V=$(echo ${VARS:-0 23} | tr ' ' ',')
timeout -k 10 400 python tools/nn_ab.py --precision fp32h3 --x6-variants $V --rounds ${ROUNDS:-3} > gpurun_out/stg_ab.json 2>&1 || { tail -5 gpurun_out/stg_ab.json; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/stg_ab.json'))
for k,v in d.items(): print(k, round(v['median_ms'],4), round(v['min_ms'],4), v['max_err_vs_torch'])"
for p in ${PHASES:-}; do
  OAZ_NN_X6_V=$p timeout -k 10 120 python tools/nn_phases.py 65536 3 h3 > gpurun_out/phases_$p.json 2>&1 || { tail -5 gpurun_out/phases_$p.json; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/phases_$p.json')); print('phases $p', d['all_waves']); print({w: v for w, v in d['per_wave_mean_cycles'].items() if w in ('w0','w4')})"
done
