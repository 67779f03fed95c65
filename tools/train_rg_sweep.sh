cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
for rg in 1 2 4; do
  OAZ_CONV_RG=$rg timeout -k 10 200 python -m pytest tests/test_train.py -m gpu -x -q > gpurun_out/train_rg$rg.log 2>&1 || exit 1
  OAZ_CONV_RG=$rg timeout -k 10 200 python bench.py --mode train --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/train_bench_rg$rg.log 2>&1 || exit 1
done
