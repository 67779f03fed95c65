"""Per-kernel statistics from a rocprofv3 SQLite output (`-d DIR -o NAME` writes DIR/NAME_results.db on this
ROCm): name, calls, total / mean / min / max duration (us), share. Experiment tool, not a test.
usage: python tools/rocpd_stats.py DB [--last N] [--grid]   (--last: only the last N dispatches)"""
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
rows = list(db.execute("select dispatch_id, name, duration, grid_x, grid_y, grid_z from kernels order by dispatch_id"))
if "--last" in sys.argv:
    rows = rows[-int(sys.argv[sys.argv.index("--last") + 1]):]
by_grid = "--grid" in sys.argv
acc = {}
for _, name, dur, gx, gy, gz in rows:
    key = name.split("(")[0][:70] + (f" [{gx}x{gy}x{gz}]" if by_grid else "")
    acc.setdefault(key, []).append(dur * 1e-3)
tot = sum(sum(v) for v in acc.values())
print(f"{'kernel':80s} {'calls':>6s} {'total_us':>10s} {'mean_us':>8s} {'min':>7s} {'max':>7s} {'pct':>5s}")
for k, v in sorted(acc.items(), key=lambda kv: -sum(kv[1])):
    print(f"{k:80s} {len(v):6d} {sum(v):10.1f} {sum(v)/len(v):8.2f} {min(v):7.2f} {max(v):7.2f} {100*sum(v)/tot:5.1f}")
print(f"dispatches {len(rows)}, kernel time {tot:.1f} us")
