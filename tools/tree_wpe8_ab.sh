cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q -m gpu -k "wide_roots or root_noise or one_launch or legacy or selfplay_matches or nn_trees" --timeout 200 --timeout-method thread > gpurun_out/t8_tests.log 2>&1; rc=$?; tail -3 gpurun_out/t8_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_scale.py -x -q -m gpu --timeout 250 --timeout-method thread > gpurun_out/t8_scale.log 2>&1; rc=$?; tail -3 gpurun_out/t8_scale.log; [ $rc -eq 0 ] || exit $rc
LIBS="onitama-alphazero_amd/onitama_az/libonitama_az_prev.so onitama-alphazero_amd/onitama_az/libonitama_az.so" ROUNDS=3 bash tools/lib_bench_ab.sh
