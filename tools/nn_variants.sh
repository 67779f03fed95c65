#!/bin/bash
# A/B of k_nn_h3 variants in the A/B build (make AB=1): per-launch time (nn_ab.py, interleaved rounds)
# and, for timing-build variants, the per-phase cycle breakdown (nn_phases.py).
# VARIANTS="0 40 41" PHASES="36" tools/nn_variants.sh  (the diagnostic variants: oaz_nn.hip launch_nn_forward)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
export OAZ_LIB=$PWD/onitama-alphazero_amd/onitama_az/libonitama_az_ab.so
mkdir -p gpurun_out/ab
V=$(echo ${VARIANTS:-0} | tr ' ' ',')
timeout -k 10 300 python tools/nn_ab.py --blocks ${BLOCKS:-3} --precision ${PREC:-fp32h3} --x6-variants $V --rounds ${ROUNDS:-5} > gpurun_out/ab/nn_ab.json 2>&1 || { cat gpurun_out/ab/nn_ab.json | tail -5; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/ab/nn_ab.json'))
for k,v in d.items(): print(k, round(v['median_ms'],4), round(v['min_ms'],4), v['max_err_vs_torch'])"
for p in ${PHASES:-}; do
  OAZ_NN_X6_V=$p timeout -k 10 120 python tools/nn_phases.py 65536 ${BLOCKS:-3} h3 > gpurun_out/ab/phases_$p.json 2>&1 || { tail -5 gpurun_out/ab/phases_$p.json; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/ab/phases_$p.json')); print('phases $p', d['per_wave_mean_cycles']['w0'], d['per_wave_mean_cycles']['w4'])"
done
