# A/B: training step, current build against the previous one (libonitama_az_prev.so); test_train.py on the
# current build first; 3 interleaved rounds at batch 512, 200 steps.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
L=onitama-alphazero_amd/onitama_az; T=${TAG:-prev_ab}
timeout -k 10 300 python -u -m pytest tests/test_train.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/train_${T}_tests.log 2>&1 || exit 1
for r in 1 2 3; do
  for v in prev cur; do
    if [ $v = prev ]; then lib=$L/libonitama_az_prev.so; else lib=$L/libonitama_az.so; fi
    echo "== round $r $v" >> gpurun_out/train_${T}.log
    OAZ_LIB=$lib timeout -k 10 200 python bench.py --mode train --steps 200 --warmup 20 --no-cpu-baseline >> gpurun_out/train_${T}.log 2>&1 || exit 1
  done
done
