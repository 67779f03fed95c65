# A/B: BN finalisation on the consumer side. Product build: forward finalisation in k_bn_act_cfin. A/B build:
# OAZ_TRAIN_CFIN=0 restores the separate k_bn_fwd_fin + k_bn_act launches; OAZ_TRAIN_CFIN_BWD=1 adds the
# backward one (k_bn_bwd_apply_cfin). test_train.py on the backward variant first; 3 interleaved rounds.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
L=onitama-alphazero_amd/onitama_az
OAZ_LIB=$L/libonitama_az_ab.so OAZ_TRAIN_CFIN_BWD=1 timeout -k 10 300 python -u -m pytest tests/test_train.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/train_cfin2_tests.log 2>&1 || exit 1
for r in 1 2 3; do
  for v in sep cfin both; do
    echo "== round $r $v" >> gpurun_out/train_cfin2_ab.log
    case $v in
      sep) OAZ_LIB=$L/libonitama_az_ab.so OAZ_TRAIN_CFIN=0 timeout -k 10 200 python bench.py --mode train --steps 200 --warmup 20 --no-cpu-baseline >> gpurun_out/train_cfin2_ab.log 2>&1 || exit 1;;
      cfin) OAZ_LIB=$L/libonitama_az.so timeout -k 10 200 python bench.py --mode train --steps 200 --warmup 20 --no-cpu-baseline >> gpurun_out/train_cfin2_ab.log 2>&1 || exit 1;;
      both) OAZ_LIB=$L/libonitama_az_ab.so OAZ_TRAIN_CFIN_BWD=1 timeout -k 10 200 python bench.py --mode train --steps 200 --warmup 20 --no-cpu-baseline >> gpurun_out/train_cfin2_ab.log 2>&1 || exit 1;;
    esac
  done
done
