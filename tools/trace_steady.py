"""Per-kernel statistics of a rocprofv3 --kernel-trace CSV over the LAST n dispatches of each kernel
(the bench's timed plies: after the warm-up plies, whose staggered starts leave slots idle and, with
leaf compaction, the NN launches short). Same columns as rocprofv3's kernel_stats.csv, plus one
"union" row per kernel family given with --union: the NN launches of the game parts (one stream
each) overlap, so a simulation step's NN time is the union of its parts' intervals; AverageNs of
that row is the union per simulation step (last n dispatches / parts steps), the number bench.py's
roofline uses (busy_ms_per_sim_step).
Usage: python tools/trace_steady.py run_kernel_trace.csv N_LAST [--union k_nn_ --parts 2]"""
import argparse
import csv
import sys
from collections import defaultdict

import numpy as np

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("n", type=int)
ap.add_argument("--union", default="")
ap.add_argument("--parts", type=int, default=1)
a = ap.parse_args()
rows = defaultdict(list)
for r in csv.DictReader(open(a.trace)):
    rows[r["Kernel_Name"]].append((int(r["Dispatch_Id"]), int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
w = csv.writer(sys.stdout, quoting=csv.QUOTE_NONNUMERIC)
w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "MinNs", "MaxNs", "StdDev", "Window"])
for k, v in sorted(rows.items(), key=lambda kv: -sum(e - s for _, s, e in kv[1][-a.n:])):
    d = np.array([e - s for _, s, e in sorted(v)][-a.n:], dtype=np.float64)
    w.writerow([k, len(d), int(d.sum()), float(d.mean()), int(d.min()), int(d.max()), float(d.std()),
                f"last {a.n} dispatches of {len(v)}"])
if a.union:
    iv = sorted(x for k, v in rows.items() if a.union in k for x in sorted(v)[-a.n:])
    iv = sorted((s, e) for _, s, e in iv)
    total, lo, hi = 0, None, None
    for s, e in iv:
        if hi is None or s > hi:
            if hi is not None:
                total += hi - lo
            lo, hi = s, e
        else:
            hi = max(hi, e)
    if hi is not None:
        total += hi - lo
    steps = max(1, len(iv) // a.parts)
    w.writerow([f"union of {a.union}* dispatches per simulation step ({a.parts} game parts)", steps, total,
                total / steps, 0, 0, 0.0, f"last {a.n} dispatches of each matching kernel"])
