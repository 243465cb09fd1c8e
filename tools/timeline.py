#!/usr/bin/env python3
"""Analyse a rocprofv3 kernel trace of tools/seq_timeline.py: the window between the two spin
kernels; per stream (queue) busy time, GPU-wide idle gaps, and per-kernel totals.
    python3 tools/timeline.py <kernel_trace.csv>"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
qcol = next((c for c in ("Stream_Id", "Queue_Id") if c in rows[0]), None)
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0].replace("void ", ""),
             r.get(qcol, "?")) for r in rows)
spins = [e for e in ev if "spin" in e[2] or "sleep" in e[2].lower()]
if len(spins) >= 2:
    lo, hi = spins[-2][1], spins[-1][0]
    ev = [e for e in ev if e[0] >= lo and e[1] <= hi]
t0 = ev[0][0]
wall = (ev[-1][1] - t0) / 1e3
# union busy
busy, cur_s, cur_e = 0, None, None
gaps = []
prev_name = None
for s, e, n, q in ev:
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            busy += cur_e - cur_s
            if s - cur_e > 20_000:
                gaps.append(((cur_e - t0) / 1e3, (s - cur_e) / 1e3, prev_name, n))
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
    prev_name = n if e >= (cur_e or 0) else prev_name
busy += cur_e - cur_s
print(f"window {wall:.2f} ms, GPU busy (union) {busy / 1e6:.2f} ms, idle {wall - busy / 1e3:.2f} ms, launches {len(ev)}")
perq = defaultdict(float)
names = defaultdict(set)
for s, e, n, q in ev:
    perq[q] += (e - s) / 1e3
    names[q].add(n.split("<")[0].replace("vo::", ""))
for q, v in sorted(perq.items(), key=lambda kv: -kv[1]):
    print(f"  queue {q}: kernel time {v:9.2f} ms  ({', '.join(sorted(names[q]))[:150]})")
print(f"idle gaps > 20 us: {len(gaps)}, total {sum(g[1] for g in gaps):.2f} ms")
for g in sorted(gaps, key=lambda g: -g[1])[:25]:
    print(f"  at {g[0]:9.2f} ms idle {g[1]:8.1f} us after {g[2][:40]} before {g[3][:40]}")
tot = defaultdict(lambda: [0.0, 0])
for s, e, n, q in ev:
    tot[n][0] += (e - s) / 1e3
    tot[n][1] += 1
print("per kernel (ms in window, launches):")
for n, (v, c) in sorted(tot.items(), key=lambda kv: -kv[1][0])[:30]:
    print(f"  {n[:60]:60s} {v:9.3f} {c:6d}")
