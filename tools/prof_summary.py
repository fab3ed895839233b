#!/usr/bin/env python
"""Summarise a rocprofv3 kernel trace: per-kernel totals + GPU idle gaps.

usage: prof_summary.py <run_kernel_stats.csv> [<run_kernel_trace.csv>]
"""
import csv
import re
import sys


def short(n):
    n = n.replace("void ", "").replace("(anonymous namespace)::", "").replace("at::native::", "")
    return n.split("(")[0][:70]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
    print(f"total kernel time {tot / 1e6:.1f} ms")
    for r in rows[:25]:
        print(f'{float(r["TotalDurationNs"]) / 1e6:9.2f} ms {100 * float(r["TotalDurationNs"]) / tot:5.1f}% '
              f'n={r["Calls"]:>5} {r["Name"][:100]}')
    if len(sys.argv) > 2:
        tr = list(csv.DictReader(open(sys.argv[2])))
        ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in tr)
        if not ev:
            return
        busy = 0
        gaps = []
        cur_end = ev[0][0]
        for s, e, n in ev:
            if s > cur_end:
                gaps.append((s - cur_end, n))
            busy += max(0, e - max(s, cur_end))
            cur_end = max(cur_end, e)
        span = cur_end - ev[0][0]
        idle = span - busy
        print(f"trace span {span / 1e6:.1f} ms, GPU busy {busy / 1e6:.1f} ms, idle {idle / 1e6:.1f} ms "
              f"({100 * idle / max(span, 1):.1f}%), {len(ev)} kernels")
        gaps.sort(reverse=True)
        big = [g for g in gaps if g[0] > 1e6]
        print(f"gaps > 1 ms: {len(big)} totalling {sum(g[0] for g in big) / 1e6:.1f} ms; "
              f"gaps <= 1 ms total {sum(g[0] for g in gaps if g[0] <= 1e6) / 1e6:.1f} ms")
        for g, n in gaps[:8]:
            print(f"  gap {g / 1e6:8.3f} ms before {n[:80]}")
        # steady-state window: between the last two optimizer (adam) launches = one training step
        adam = [i for i, e in enumerate(ev) if re.search(r"adam(_img)?_kernel", e[2])]
        if len(adam) >= 2:
            i0, i1 = adam[-2], adam[-1]
            win = ev[i0 + 1:i1 + 1]
            t0, t1 = ev[i0][1], ev[i1][1]
            wb, cur, sg = 0, t0, {}
            for s, e, n in win:
                if s > cur:
                    key = short(n)
                    sg[key] = sg.get(key, 0) + (s - cur)
                wb += max(0, e - max(s, cur))
                cur = max(cur, e)
            print(f"last step: {(t1 - t0) / 1e6:.2f} ms wall, GPU busy {wb / 1e6:.2f} ms, "
                  f"{len(win)} kernels, idle {(t1 - t0 - wb) / 1e6:.2f} ms; idle before (top):")
            for k, v in sorted(sg.items(), key=lambda kv: -kv[1])[:12]:
                print(f"    {v / 1e3:8.1f} us  {k}")
            per = {}
            for s, e, n in win:
                key = short(n)
                per[key] = per.get(key, 0) + (e - s)
            print("  kernel time in that step (top):")
            for k, v in sorted(per.items(), key=lambda kv: -kv[1])[:14]:
                print(f"    {v / 1e3:8.1f} us  {k}")


if __name__ == "__main__":
    main()
