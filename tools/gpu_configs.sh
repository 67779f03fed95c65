#!/bin/bash
# The other BASELINE configs through bench.py (C2, C5) and a 2-rank torchrun rehearsal of the
# multi-GPU path on one GPU (gloo collectives, OAZ_BENCH_REHEARSE=1; its timings mean nothing).
# Each step has its own time limit; stops at the first failure.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
TAG=${TAG:-cfg}
mkdir -p gpurun_out
step() { local name=$1 out=$2; shift 2; echo "== $name"; "$@" > gpurun_out/$out.json 2> gpurun_out/$out.err; local rc=$?; echo "$name rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step c2 bench_c2_$TAG timeout -k 10 600 python bench.py --config c2
step c5 bench_c5_$TAG timeout -k 10 900 python bench.py --config c5 ${C5_ARGS:-}
step rehearse2 rehearse2_$TAG env OAZ_BENCH_REHEARSE=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --games 16384 --steps 2 --warmup 2
for f in gpurun_out/bench_c2_$TAG.json gpurun_out/bench_c5_$TAG.json gpurun_out/rehearse2_$TAG.json; do
  python -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', round(d['value']/1e6,3), d['unit'], 'games/s', round(d.get('games_per_s',0)), 'checks', d.get('checks',{}).get('ok'))"
done
