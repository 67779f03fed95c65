#!/bin/bash
# Where k_nn_h3's power goes: per-launch time (tools/nn_ab.py, interleaved rounds) and the clock it ran at
# (rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace: cycles / duration) of the A/B build's ablations
# (timing only, wrong results): 0 product body, 40 no conv A reads, 41 no conv B loads, 47 conv B loads
# of one step (L1 hits instead of L2), 49 conv A reads performed but discarded (stale MFMA operands).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
export OAZ_LIB=$PWD/onitama-alphazero_amd/onitama_az/libonitama_az_ab.so
OUT=gpurun_out/energy; mkdir -p $OUT
PY=$(command -v python3)
V=${VARIANTS:-0 40 41 47 49}
timeout -k 10 300 python tools/nn_ab.py --blocks 3 --precision fp32h3 --x6-variants $(echo $V | tr ' ' ',') --rounds ${ROUNDS:-6} > $OUT/nn_ab.json 2>&1 || { tail -5 $OUT/nn_ab.json; exit 1; }
for v in $V; do
  OAZ_NN_X6_V=$v timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace --kernel-include-regex k_nn_ --output-format csv -d $OUT/clk$v -o run -- "$PY" tools/nn_prof.py 65536 3 fp32h3 6 > $OUT/clk$v.log 2>&1
  rc=$?; if [ $rc -ne 0 ]; then echo "clock pass $v rc=$rc"; tail -5 $OUT/clk$v.log; exit $rc; fi
done
python3 - <<'PY'
import csv, glob, json, os
out = "gpurun_out/energy"
ab = json.load(open(f"{out}/nn_ab.json"))
for v in os.environ.get("VARIANTS", "0 40 41 47 49").split():
    g, d = {}, {}
    for f in glob.glob(f"{out}/clk{v}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == "GRBM_GUI_ACTIVE":
                g[int(r["Dispatch_Id"])] = g.get(int(r["Dispatch_Id"]), 0.0) + float(r["Counter_Value"])
    for f in glob.glob(f"{out}/clk{v}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            d[int(r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    ids = sorted(set(g) & set(d))[1:]  # the first launch is a warm-up
    cyc = sum(g[i] / 8 for i in ids) / len(ids)
    mhz = sum(g[i] / 8 / d[i] / 1e6 for i in ids) / len(ids)
    k = [x for x in ab if x.endswith(f"-v{v}")][0]
    print(f"variant {v:>3}: {ab[k]['median_ms']:.4f} ms (nn_ab median), cycles/launch {cyc/1e6:.3f} M, clock {mhz:.0f} MHz")
PY
