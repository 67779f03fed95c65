#!/bin/bash
# Where k_nn_h3's L2 fills come from: FETCH_SIZE / WRITE_SIZE of the network kernel
# launched back to back on one engine (tools/nn_prof.py: 65 536 positions per launch, host copies between
# launches, no tree kernels) against the same kernel inside the C3 self-play loop (bench.py's PMC passes:
# the two game parts' tree kernels and the root-noise kernel run between its launches).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/nn_l2}; mkdir -p $OUT
PY=$(command -v python3)
i=0
for set in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-include-regex k_nn_ --output-format csv -d $OUT/p$i -o run \
      -- "$PY" tools/nn_prof.py 65536 3 fp32h3 6 > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; if [ $rc -ne 0 ]; then tail -5 $OUT/p$i.log; exit $rc; fi
done
OUT=$OUT python3 - <<'PY' > $OUT/summary.txt
import csv, glob, collections, os
acc = collections.defaultdict(list)
for f in glob.glob(os.environ["OUT"] + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        acc[r["Counter_Name"]].append((int(r.get("Dispatch_Id", 0) or 0), float(r["Counter_Value"])))
for k, v in sorted(acc.items()):
    v.sort()
    vals = [x for _, x in v]
    print(f"{k:16s} per launch: " + " ".join(f"{x:.0f}" for x in vals) + f"  (mean of launches 2..: {sum(vals[1:]) / max(1, len(vals) - 1):.0f})")
PY
cat $OUT/summary.txt
