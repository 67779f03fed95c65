# A/B: k_bn_bwd_apply rows per workgroup (A/B build OAZ_TRAIN_BWD_U=4 / 8: 16 / 32 rows, 800 / 400 workgroups
# at batch 512) against the product's 64 rows (200 workgroups). test_train.py on both first; 3 rounds.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
L=onitama-alphazero_amd/onitama_az
for u in 32; do
  OAZ_LIB=$L/libonitama_az_ab.so OAZ_TRAIN_BWD_U=$u timeout -k 10 300 python -u -m pytest tests/test_train.py -m gpu -x -q --timeout 120 --timeout-method thread >> gpurun_out/train_bwdu32_tests.log 2>&1 || exit 1
done
for r in 1 2 3; do
  for v in 16 32; do
    if [ $v = 16 ]; then lib=$L/libonitama_az.so; else lib=$L/libonitama_az_ab.so; fi
    echo "== round $r bwd_u=$v" >> gpurun_out/train_bwdu32_ab.log
    OAZ_LIB=$lib OAZ_TRAIN_BWD_U=$v timeout -k 10 200 python bench.py --mode train --steps 200 --warmup 20 --no-cpu-baseline >> gpurun_out/train_bwdu32_ab.log 2>&1 || exit 1
  done
done
