#!/usr/bin/env python3
"""Per-stream occupancy of the pipelined SIFT loop from a rocprofv3 kernel trace of
tools/prof_run.py (N back-to-back calls, then one synchronised call): for the back-to-back
window, each queue's busy time (union of its kernels), its idle gaps and the kernels that
bracket the largest ones -- which stream is the critical path, and what the other waits on.
    python3 tools/stream_busy.py <kernel_trace.csv> [skip_first_calls]"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
qcol = next(c for c in ("Stream_Id", "Queue_Id") if c in rows[0])
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0].replace("void ", ""),
             r[qcol]) for r in rows if "vo::" in r["Kernel_Name"])
# window: from the first k_blur_base after `skip` calls to the start of the last k_blur_base
# (the synchronised call), so the warm-up call and the serialised call stay out
skip = int(sys.argv[2]) if len(sys.argv) > 2 else 1
bases = [e for e in ev if "k_blur_stream<5, 5" in e[2] or "k_blur_base" in e[2]]
lo, hi = bases[skip][0], bases[-1][0]
ev = [e for e in ev if e[0] >= lo and e[1] <= hi]
wall = (hi - lo) / 1e3
calls = len(bases) - 1 - skip
print(f"window {wall:.1f} us over {calls} calls ({wall / max(calls, 1):.1f} us per call)")
byq = defaultdict(list)
for e in ev:
    byq[e[3]].append(e)
for q, es in sorted(byq.items(), key=lambda kv: -len(kv[1])):
    es.sort()
    busy, gaps = 0, []
    cs, ce, prev = es[0][0], es[0][1], es[0][2]
    for s, e, n, _ in es[1:]:
        if s > ce:
            busy += ce - cs
            gaps.append(((s - ce) / 1e3, prev, n))
            cs, ce = s, e
        else:
            ce = max(ce, e)
        prev = n
    busy += ce - cs
    tot_gap = sum(g[0] for g in gaps)
    names = defaultdict(float)
    for s, e, n, _ in es:
        names[n.split("<")[0]] += (e - s) / 1e3
    top = ", ".join(f"{k} {v / max(calls, 1):.0f}" for k, v in sorted(names.items(), key=lambda kv: -kv[1])[:6])
    print(f"queue {q}: {len(es)} launches, busy {busy / 1e3:.1f} us ({100 * busy / 1e3 / wall:.1f} %), "
          f"gaps {tot_gap:.1f} us in {len(gaps)}; per call: {top}")
    for g, a, b in sorted(gaps, reverse=True)[:5]:
        print(f"    gap {g:8.1f} us after {a[:40]} before {b[:40]}")
