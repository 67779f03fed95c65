"""FETCH_SIZE / WRITE_SIZE (rocprofv3 CSVs of tools/pmc_cal/run.sh) against each calibration kernel's known bytes."""
import csv
import glob
import sys

N = 1 << 22
KNOWN = {  # bytes each kernel touches (every line once)
    "k_cal_stream16": ("read", 16 * N), "k_cal_rec32": ("read", 32 * N), "k_cal_run400": ("read", 400 * N // 16),
    "k_cal_rec24": ("read", 24 * N), "k_cal_word4": ("read", 4 * N), "k_cal_word8": ("read", 8 * N),
    "k_cal_coal4": ("read", 4 * N), "k_cal_seg64": ("read", 16 * N),
    "k_cal_wstream16": ("write", 16 * N), "k_cal_wrec12": ("write", 12 * N), "k_cal_wword4": ("write", 4 * N),
}
vals = {}
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = next((k for k in KNOWN if k in r["Kernel_Name"]), None)
        if k:
            vals[(k, r["Counter_Name"])] = vals.get((k, r["Counter_Name"]), 0.0) + float(r["Counter_Value"])
print(f"{'kernel':18s} {'known':>12s} {'FETCH_SIZE':>12s} {'ratio':>7s} {'WRITE_SIZE':>12s} {'ratio':>7s}")
for k, (kind, b) in KNOWN.items():
    fz, wz = vals.get((k, "FETCH_SIZE")), vals.get((k, "WRITE_SIZE"))
    fb = fz * 1024 if fz is not None else None
    wb = wz * 1024 if wz is not None else None
    print(f"{k:18s} {b:12d} {fb if fb is not None else float('nan'):12.0f} {(fb / b) if fb else float('nan'):7.3f} "
          f"{wb if wb is not None else float('nan'):12.0f} {(wb / b) if wb else float('nan'):7.3f}   ({kind})")
