"""Kernel-trace overlap analysis: for every launch of the kernels named on the command line,
its duration and the time-weighted share of each other kernel running concurrently.
    python3 tools/overlap.py <kernel_trace.csv> <name-prefix> [...]"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0].replace("void ", "")) for r in rows]
ev.sort()
for pref in sys.argv[2:]:
    tgt = [e for e in ev if e[2].startswith(pref) or pref in e[2]]
    print(f"== {pref}: {len(tgt)} launches, mean {sum(e[1]-e[0] for e in tgt)/max(len(tgt),1)/1e3:.1f} us")
    share = defaultdict(float)
    slow = sorted(tgt, key=lambda e: -(e[1] - e[0]))[:6]
    for s, e, n in tgt:
        for s2, e2, n2 in ev:
            if (s2, e2, n2) == (s, e, n) or e2 <= s or s2 >= e:
                continue
            share[n2] += (min(e, e2) - max(s, s2)) / 1e3
    tot = sum(e[1] - e[0] for e in tgt) / 1e3
    for n2, v in sorted(share.items(), key=lambda kv: -kv[1])[:10]:
        print(f"   overlapped by {n2[:50]:50s} {v:9.1f} us ({v / tot:.0%} of its time)")
    for s, e, n in slow:
        co = sorted({n2.split('<')[0] for s2, e2, n2 in ev if not (e2 <= s or s2 >= e) and (s2, e2, n2) != (s, e, n)})
        print(f"   slow launch {n[:40]} {(e - s) / 1e3:8.1f} us with {co}")
