# A/B: weight-gradient row splits per (tap, square): 2 (product) against 1 and 4 (-DOAZ_WSPLIT builds
# libonitama_az_ws{1,4}.so). test_train.py on both variants first; 3 interleaved rounds at batch 512.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
L=onitama-alphazero_amd/onitama_az
for w in 1 4; do
  OAZ_LIB=$L/libonitama_az_ws$w.so timeout -k 10 300 python -u -m pytest tests/test_train.py -m gpu -x -q --timeout 120 --timeout-method thread >> gpurun_out/train_wsplit_tests.log 2>&1 || exit 1
done
for r in 1 2 3; do
  for v in 2 1 4; do
    if [ $v = 2 ]; then lib=$L/libonitama_az.so; else lib=$L/libonitama_az_ws$v.so; fi
    echo "== round $r wsplit=$v" >> gpurun_out/train_wsplit_ab.log
    OAZ_LIB=$lib timeout -k 10 200 python bench.py --mode train --steps 200 --warmup 20 --no-cpu-baseline >> gpurun_out/train_wsplit_ab.log 2>&1 || exit 1
  done
done
