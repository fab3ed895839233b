"""Kernel timeline of the batch-1 synthesis runs in a rocprofv3 kernel trace (bench_synth.py --steps 0
--b1-runs N): splits the trace at host gaps > 200 us, reports the last full run's span, busy time, kernel count and
top kernels.  python tools/b1_trace.py <kernel_trace.csv>"""
import csv
import sys
from collections import Counter

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
segs, cur = [], [rows[0]]
for a, b in zip(rows, rows[1:]):
    if int(b["Start_Timestamp"]) - int(a["End_Timestamp"]) > 200_000:
        segs.append(cur)
        cur = []
    cur.append(b)
segs.append(cur)
big = [s for s in segs if len(s) > 100]
print(f"{len(segs)} segments, {len(big)} with > 100 kernels; sizes of the last 8: {[len(s) for s in segs[-8:]]}")
for s in big[-2:]:
    span = (int(s[-1]["End_Timestamp"]) - int(s[0]["Start_Timestamp"])) / 1e3
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in s) / 1e3
    gaps = [(int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3 for a, b in zip(s, s[1:])]
    print(f"run: {len(s)} kernels, span {span:.1f} us, busy {busy:.1f} us, gaps {sum(g for g in gaps if g > 0):.1f} us"
          f" (> 20 us: {sorted((round(g, 1) for g in gaps if g > 20), reverse=True)[:8]})")
    t, c = Counter(), Counter()
    for r in s:
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
        k = k.split("(")[0][:90]
        t[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        c[k] += 1
    for k, v in t.most_common(25):
        print(f"  {v:8.1f} us  n={c[k]:3d}  {k}")
if len(sys.argv) > 2 and sys.argv[2] == "--seq":  # ordered kernel sequence of the last run (fusion census)
    s = big[-1]
    t0 = int(s[0]["Start_Timestamp"])
    prev = t0
    for r in s:
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:80]
        st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        print(f"{(st - t0) / 1e3:9.1f} {(en - st) / 1e3:7.1f} gap {(st - prev) / 1e3:6.1f}  {k}")
        prev = en
