"""Per-kernel statistics of a rocprofv3 --kernel-trace CSV over the LAST n dispatches of each kernel
(the bench's timed plies: after the warm-up plies, whose staggered starts leave slots idle and, with
leaf compaction, the NN launches short). Same columns as rocprofv3's kernel_stats.csv.
Usage: python tools/trace_steady.py run_kernel_trace.csv N_LAST > steady_kernel_stats.csv"""
import csv
import sys
from collections import defaultdict

import numpy as np

rows = defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    rows[r["Kernel_Name"]].append((int(r["Dispatch_Id"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
n = int(sys.argv[2])
w = csv.writer(sys.stdout, quoting=csv.QUOTE_NONNUMERIC)
w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "MinNs", "MaxNs", "StdDev", "Window"])
for k, v in sorted(rows.items(), key=lambda kv: -sum(d for _, d in kv[1][-n:])):
    d = np.array([x for _, x in sorted(v)][-n:], dtype=np.float64)
    w.writerow([k, len(d), int(d.sum()), float(d.mean()), int(d.min()), int(d.max()), float(d.std()),
                f"last {n} dispatches of {len(v)}"])
