#!/bin/bash
# A/B of the bf16 NN kernel variants (OAZ_NN_BF16_V1): 0 = k_nn_bf16g<2>, 1 = k_nn_sq16<bf16>, 2 = k_nn_bf16g<4>
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
for v in 1 0 2; do
  OAZ_NN_BF16_V1=$v timeout -k 10 300 python tools/nn_ab.py --blocks 6 --precision bf16 --batch 65536 > gpurun_out/nn_bf16_v$v.json 2>&1 || exit 1
done
