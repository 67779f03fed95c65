#!/bin/bash
# SQ counter passes over the fused tree kernel k_backup_select_seg (tools/tree_prof.py, single stream,
# the launches of ply 3), one rocprofv3 run per pass; per-dispatch means in $OUT/summary.txt.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/tree_pmc}; mkdir -p $OUT
PY=$(command -v python3)
SIMS=${SIMS:-400}
R="[$((2 * SIMS + 1))-$((3 * SIMS - 1))]"
i=0
DEFAULT_SETS=("SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM" \
           "SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_WAVES SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum" )
if [ -n "${SETS:-}" ]; then IFS=';' read -r -a SETLIST <<< "$SETS"; else SETLIST=("${DEFAULT_SETS[@]}"); fi
# SETS="A B;C D" overrides the counter sets (one rocprofv3 pass per ';'-separated set)
for set in "${SETLIST[@]}"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $set --kernel-include-regex k_backup_select_seg --kernel-iteration-range "$R" \
      --output-format csv -d $OUT/p$i -o run -- "$PY" tools/tree_prof.py 65536 $SIMS 3 > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; if [ $rc -ne 0 ]; then tail -5 $OUT/p$i.log; exit $rc; fi
done
timeout -s KILL 180 rocprofv3 --kernel-trace --kernel-include-regex k_backup_select_seg --output-format csv -d $OUT/trace -o run -- "$PY" tools/tree_prof.py 65536 $SIMS 3 > $OUT/trace.log 2>&1 || exit $?
OUT=$OUT python3 - <<'PY' > $OUT/summary.txt
import csv, glob, collections, os
acc = collections.defaultdict(list)
for f in glob.glob(os.environ["OUT"] + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(acc.items()):
    print(f"{k:30s} {sum(v)/len(v):16.1f}  (n={len(v)})")
d = []
for f in glob.glob(os.environ["OUT"] + "/trace/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        d.append((int(r["Dispatch_Id"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3))
d.sort()
last = [x for _, x in d[-400:]]
print(f"trace: {len(d)} dispatches, last 400 mean {sum(last)/len(last):.1f} us")
PY
cat $OUT/summary.txt
