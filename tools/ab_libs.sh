#!/bin/bash
# Same-box A/B of NN kernel builds: fp16x3 3-block, then bf16 6-block, ROUNDS interleaved rounds over
# the libraries named (basenames under onitama_az/) in $NAMES; log in gpurun_out/ab_$TAG.log.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
L=onitama-alphazero_amd/onitama_az
LIBS=""; for n in $NAMES; do LIBS="$LIBS $L/libonitama_az_$n.so"; done
{ PREC=fp32h3 BLOCKS=3 ROUNDS=${ROUNDS:-8} LIBS="$LIBS" bash tools/lib_ab.sh &&
  PREC=bf16 BLOCKS=6 ROUNDS=${ROUNDS:-8} LIBS="$LIBS" bash tools/lib_ab.sh; } > gpurun_out/ab_${TAG:-x}.log 2>&1
rc=$?; python tools/ab_summary.py gpurun_out/ab_${TAG:-x}.log; exit $rc
