# A/B: training step with the previous build (libonitama_az_prev.so), the current one, and the A/B build
# with the critical-path stream at the higher priority (OAZ_TRAIN_PRIO=1). Three interleaved rounds.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
L=onitama-alphazero_amd/onitama_az
timeout -k 10 300 python -u -m pytest tests/test_train.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/train_fin_tests.log 2>&1 || exit 1
OAZ_LIB=$L/libonitama_az_ab.so OAZ_TRAIN_PRIO=1 timeout -k 10 300 python -u -m pytest tests/test_train.py -m gpu -x -q --timeout 120 --timeout-method thread >> gpurun_out/train_fin_tests.log 2>&1 || exit 1
for r in 1 2 3; do
  for v in prev cur prio; do
    case $v in prev) lib=$L/libonitama_az_prev.so; p=;; cur) lib=$L/libonitama_az.so; p=;; prio) lib=$L/libonitama_az_ab.so; p=1;; esac
    echo "== round $r $v" >> gpurun_out/train_fin_ab.log
    OAZ_LIB=$lib OAZ_TRAIN_PRIO=$p timeout -k 10 200 python bench.py --mode train --steps 200 --warmup 20 --no-cpu-baseline >> gpurun_out/train_fin_ab.log 2>&1 || exit 1
  done
done
