#!/usr/bin/env python
"""Per-stream view of the last training steps in a rocprofv3 kernel trace (weight gradients on the
side stream): per step, the busy time of each stream, the time both run together, and how long the
optimizer waited at the join for the side stream after the main stream's last backward kernel.

Usage: python tools/stream_split.py <kernel_trace.csv> [--last 5]"""
import argparse
import csv
import re
from collections import defaultdict


def short(n):
    n = n.replace("(anonymous namespace)::", "").replace("void ", "")
    m = re.match(r"([\w:]+(?:<[^()]*?>)?)", n)
    return (m.group(1) if m else n)[:48]


def union(iv):
    tot, cur = 0, None
    for s, e in sorted(iv):
        if cur is None or s > cur[1]:
            if cur:
                tot += cur[1] - cur[0]
            cur = [s, e]
        else:
            cur[1] = max(cur[1], e)
    if cur:
        tot += cur[1] - cur[0]
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--last", type=int, default=5)
    ap.add_argument("--tail", type=int, default=0, help="print the last N kernels (both streams) before Adam")
    ap.add_argument("--detail", action="store_true", help="per-stream top kernels and the kernels after main-stream gaps")
    ap.add_argument("--gaps", type=int, default=0,
                    help="print the N largest main-stream gaps: kernels around them and the side-stream kernel "
                         "that ended last before the gap closed (an event wait ends with it)")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    skey = "Stream_Id" if "Stream_Id" in rows[0] else "Queue_Id"
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r.get(skey, "0")) for r in rows)
    ends = [i for i, k in enumerate(ks) if re.search(r"adam(_img)?_kernel", k[2])]
    steps = list(zip(ends[:-1], ends[1:]))[-a.last:]
    print(f"stream key: {skey}")
    for i0, i1 in steps:
        t0, t1 = ks[i0][1], ks[i1][1]
        seg = ks[i0 + 1:i1 + 1]
        per = defaultdict(list)
        for s, e, n, q in seg:
            per[q].append((s, e))
        main_q = ks[i1][3]
        busy = {q: union(v) / 1e6 for q, v in per.items()}
        allu = union([(s, e) for s, e, _, _ in seg]) / 1e6
        both = sum(busy.values()) - allu
        side = [q for q in per if q != main_q]
        # the optimizer (adam) start vs the last main-stream kernel before it and the last side kernel
        adam_s = ks[i1][0]
        main_prev = max((e for s, e, n, q in seg[:-1] if q == main_q), default=t0)
        side_last = max((e for s, e, n, q in seg if q in side), default=t0)
        print(f"span {(t1 - t0) / 1e6:7.3f} ms  union {allu:7.3f}  overlap {both:6.3f}  "
              + "  ".join(f"q{q}:{busy[q]:7.3f}({len(per[q])})" for q in sorted(per))
              + f"  | main-idle-before-adam {(adam_s - main_prev) / 1e6:6.3f}  side-ends-before-adam {(adam_s - side_last) / 1e6:6.3f}")
        # main-stream idle gaps inside the step (waiting for host or for the side stream)
        if a.tail:
            for s_, e_, n, q in seg[-a.tail:]:
                print(f"   {(s_ - t0) / 1e3:9.1f} .. {(e_ - t0) / 1e3:9.1f} us  q{q}  {short(n)}")
        mk = sorted((s, e, n) for s, e, n, q in seg if q == main_q)
        gaps = [((mk[i + 1][0] - mk[i][1]) / 1e3, mk[i + 1][2]) for i in range(len(mk) - 1)]
        print(f"   main-stream gaps: total {sum(g for g, _ in gaps if g > 0) / 1e3:.3f} ms, "
              f">20us: {sum(1 for g, _ in gaps if g > 20)}")
        if a.gaps:
            gi = sorted(range(len(mk) - 1), key=lambda i: -(mk[i + 1][0] - mk[i][1]))[:a.gaps]
            sk = sorted((s, e, n) for s, e, n, q in seg if q != main_q)
            for i in sorted(gi):
                g0, g1 = mk[i][1], mk[i + 1][0]
                ended = [x for x in sk if g0 <= x[1] <= g1]
                last_side = max(ended, key=lambda x: x[1]) if ended else None
                running = sum(1 for x in sk if x[0] < g1 and x[1] > g0)
                print(f"   gap {(g1 - g0) / 1e3:7.1f} us at {(g0 - t0) / 1e3:8.1f}: {short(mk[i][2])} -> {short(mk[i + 1][2])}"
                      + (f"  | side ended {(g1 - last_side[1]) / 1e3:6.1f} us before close: {short(last_side[2])}"
                         if last_side else "") + f"  side kernels overlapping {running}")
        if a.detail:
            by = defaultdict(float)
            for g, n in gaps:
                if g > 0:
                    by[short(n)] += g
            print("   gap before (us): " + ", ".join(f"{k} {v:.0f}" for k, v in sorted(by.items(), key=lambda x: -x[1])[:8]))
            for q in sorted(per):
                tot = defaultdict(float)
                for s_, e_, n, qq in seg:
                    if qq == q:
                        tot[short(n)] += (e_ - s_) / 1e3
                print(f"   q{q} top: " + ", ".join(f"{k} {v:.0f}" for k, v in sorted(tot.items(), key=lambda x: -x[1])[:10]))


if __name__ == "__main__":
    main()
