#!/bin/bash
# Same-box A/B of tree-kernel builds (onitama_az/libonitama_az_<name>.so for each name in $NAMES):
# tools/tree_noise_probe.py (single-stream C3, noise on / off) over ROUNDS interleaved rounds.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
for r in $(seq 1 ${ROUNDS:-3}); do
  for n in $NAMES; do
    OAZ_LIB=$PWD/onitama-alphazero_amd/onitama_az/libonitama_az_$n.so timeout -k 10 200 python tools/tree_noise_probe.py 2>/dev/null | sed "s/^/$n /" || exit 1
  done
done
