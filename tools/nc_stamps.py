#!/usr/bin/env python3
"""Summarise the LDS candidate pass's per-workgroup stamps (SYZCOV_NC_DBG=8,
100 MHz clock) of the last launch in a stamp file."""
import sys
from collections import defaultdict

blocks, cur = [], []
for line in open(sys.argv[1]):
    if line.startswith("--"):
        blocks.append(cur)
        cur = []
    else:
        cur.append([int(x) for x in line.split()])
b = blocks[-1]
t0 = min(r[1] for r in b)
span = (max(r[3] for r in b) - t0) / 100
print(f"workgroups {len(b)}  span {span:.1f} us")
st = sorted((r[2] - r[1]) / 100 for r in b)
du = sorted((r[3] - r[2]) / 100 for r in b)
pct = lambda a, p: a[min(len(a) - 1, int(p * len(a)))]  # noqa: E731
print("staging+first step us: p10 %.1f p50 %.1f p90 %.1f max %.1f" % tuple(pct(st, p) for p in (.1, .5, .9, 1)))
print("loop us:               p10 %.1f p50 %.1f p90 %.1f max %.1f" % tuple(pct(du, p) for p in (.1, .5, .9, 1)))
rows = [r[4] & 0xFFFFFF for r in b]
tot_rows = sum(rows)
print(f"rows {tot_rows}, per WG p50 {sorted(rows)[len(rows)//2]}, max {max(rows)}")
per_row = sorted(((r[3] - r[2]) / 100) / max(1, r[4] & 0xFFFFFF) for r in b if (r[4] & 0xFFFFFF) > 256)
print("loop us per row (WGs > 256 rows): p10 %.3f p50 %.3f p90 %.3f" % tuple(pct(per_row, p) for p in (.1, .5, .9)))
# concurrency over time
ev = sorted([(r[1], 1) for r in b] + [(r[3], -1) for r in b])
c, mx, acc, last = 0, 0, 0.0, ev[0][0]
for t, d in ev:
    acc += c * (t - last)
    last = t
    c += d
    mx = max(mx, c)
print(f"concurrent WGs: max {mx}, mean {acc / (last - ev[0][0]):.1f}")
# time when 90% of WGs done
ends = sorted((r[3] - t0) / 100 for r in b)
print("WG end times us: p50 %.1f p90 %.1f p99 %.1f max %.1f" % tuple(pct(ends, p) for p in (.5, .9, .99, 1)))
byq = defaultdict(list)
for r in b:
    byq[(r[4] >> 24) & 0xFF].append((r[3] - r[1]) / 100)
print("per range: " + ", ".join(f"q{q}: n={len(v)} avg {sum(v)/len(v):.1f}us" for q, v in sorted(byq.items())))
# per-CU concurrency: (xcc, se, cu-field)
cu = defaultdict(list)
for r in b:
    key = ((r[4] >> 48) & 15, (r[4] >> 40) & 7, (r[4] >> 32) & 0xFF)
    cu[key].append((r[1], r[3]))
mx = 0
for key, iv in cu.items():
    ev = sorted([(a, 1) for a, _ in iv] + [(z, -1) for _, z in iv])
    c = 0
    for _, d in ev:
        c += d
        mx = max(mx, c)
print(f"distinct (xcc, se, cu) ids: {len(cu)}, max concurrent per id: {mx}, "
      f"xccs: {sorted(set(k[0] for k in cu))}")
