#!/usr/bin/env python
"""Per-step GPU timeline of a training run from a rocprofv3 kernel trace.

Steps are delimited by the fused Adam kernel.  For each step: span (end of the previous Adam kernel
to the end of this one), busy (union of kernel intervals), idle = span - busy, kernel count, and
the largest idle gaps with the kernel that followed them.  The totals over the last ``--last``
steps show whether the bench's ms/step is GPU work or GPU idle (host pacing / syncs).

Usage: python tools/step_timeline.py <kernel_trace.csv> [--last 10] [--gaps 12]"""
import argparse
import csv
import re
from collections import defaultdict


def short(n):
    n = n.replace("(anonymous namespace)::", "")
    m = re.match(r"(?:void )?([\w:]+(?:<[^()]*?>)?)", n)
    return (m.group(1) if m else n)[:64]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--last", type=int, default=10)
    ap.add_argument("--gaps", type=int, default=12)
    ap.add_argument("--top", type=int, default=60, help="per-(kernel, grid) table rows")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    def grid(r):
        return "x".join(str(r.get(k, "")) for k in ("Grid_Size_X", "Grid_Size_Y", "Grid_Size_Z"))

    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]), grid(r))
                 for r in rows))
    ends = [i for i, k in enumerate(ks) if re.search(r"adam(_img)?_kernel", k[2])]
    steps = list(zip(ends[:-1], ends[1:]))[-a.last:]
    tot_span = tot_busy = 0.0
    gap_by_next = defaultdict(float)
    print(f"{'step':>4} {'span_ms':>8} {'busy_ms':>8} {'idle_ms':>8} {'kernels':>7}")
    for si, (i0, i1) in enumerate(steps):
        t_prev = ks[i0][1]
        span = (ks[i1][1] - t_prev) / 1e6
        busy = 0.0
        cur_end = t_prev
        for s, e, n, _ in ks[i0 + 1:i1 + 1]:
            if s > cur_end:
                gap_by_next[n] += (s - cur_end) / 1e3
                busy += (e - s) / 1e6
                cur_end = e
            elif e > cur_end:
                busy += (e - cur_end) / 1e6
                cur_end = e
        tot_span += span
        tot_busy += busy
        print(f"{si:4d} {span:8.3f} {busy:8.3f} {span - busy:8.3f} {i1 - i0:7d}")
    n = max(1, len(steps))
    print(f"mean span {tot_span / n:.3f} ms, busy {tot_busy / n:.3f} ms, idle {(tot_span - tot_busy) / n:.3f} ms "
          f"({100 * (1 - tot_busy / max(tot_span, 1e-9)):.1f} %) over {len(steps)} steps")
    print("idle before kernel (us per step, summed over steps / n):")
    for k, v in sorted(gap_by_next.items(), key=lambda x: -x[1])[:a.gaps]:
        print(f"  {v / n:8.1f}  {k}")
    per = defaultdict(lambda: [0, 0.0])
    per_name = defaultdict(lambda: [0, 0.0])
    for i0, i1 in steps:
        for s, e, nm, gr in ks[i0 + 1:i1 + 1]:
            per[(nm, gr)][0] += 1
            per[(nm, gr)][1] += (e - s) / 1e3
            per_name[nm][0] += 1
            per_name[nm][1] += (e - s) / 1e3
    print("per kernel (us per step, launches per step):")
    for nm, (c, t) in sorted(per_name.items(), key=lambda x: -x[1][1])[:a.top]:
        print(f"  {t / n:9.1f} {c / n:6.1f}  {nm}")
    print("per kernel and grid (us per step, launches per step, us per launch):")
    for (nm, gr), (c, t) in sorted(per.items(), key=lambda x: -x[1][1])[:a.top]:
        print(f"  {t / n:9.1f} {c / n:6.1f} {t / max(c, 1):8.1f}  {nm}  grid={gr}")


if __name__ == "__main__":
    main()
