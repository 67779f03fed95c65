"""Summarise a tools/ab_libs.sh log: mean / median / min per-launch ms per library and precision block."""
import collections
import re
import statistics as st
import sys

d = collections.defaultdict(list)
blk, seen = 0, set()
for line in open(sys.argv[1]):
    m = re.match(r"(\S+) round (\d+) \[([\d.]+)\]", line)
    if not m:
        continue
    key = (m.group(1), int(m.group(2)))
    if key in seen:  # the second precision's rounds start
        blk, seen = blk + 1, set()
    seen.add(key)
    d[(blk, m.group(1))].append(float(m.group(3)))
for (b, name), v in sorted(d.items()):
    print(f"{['fp16x3 3-block', 'bf16 6-block'][b] if b < 2 else b:>15} {name:28} mean {st.mean(v):.4f} "
          f"median {st.median(v):.4f} min {min(v):.4f} n {len(v)}")
