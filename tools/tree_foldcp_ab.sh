# A/B: the root noise fold by change points (-DOAZ_FOLD_CP=1, libonitama_az_cp.so) against the product's
# sequential fold: tree / noise / self-play parity tests on the variant, then tools/tree_noise_probe.py, 3 rounds.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
L=onitama-alphazero_amd/onitama_az
OAZ_LIB=$L/libonitama_az_cp.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "hash_trees or selfplay or noise or scale" > gpurun_out/tree_foldcp_tests.log 2>&1 || exit 1
for r in 1 2 3; do
  for v in seq cp; do
    if [ $v = seq ]; then lib=$L/libonitama_az.so; else lib=$L/libonitama_az_cp.so; fi
    echo "== round $r $v" >> gpurun_out/tree_foldcp_ab.log
    OAZ_LIB=$lib timeout -k 10 200 python tools/tree_noise_probe.py 65536 400 >> gpurun_out/tree_foldcp_ab.log 2>&1 || exit 1
  done
done
