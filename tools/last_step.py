#!/usr/bin/env python
"""Per-kernel time of the LAST training step in a rocprofv3 kernel trace (steps delimited by the
Adam kernel): the steady-state breakdown, free of the warm-up steps' clock ramp.
Usage: python tools/last_step.py <kernel_trace.csv> [top]"""
import csv
import re
import sys
from collections import defaultdict


def short(n):
    n = n.replace("(anonymous namespace)::", "")
    m = re.match(r"(?:void )?([\w:]+(?:<[^()]*?>)?)", n)
    return (m.group(1) if m else n)[:72]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ends = [i for i, r in enumerate(rows) if re.search(r"adam(_img)?_kernel", r["Kernel_Name"])]
    a, b = ends[-2] + 1, ends[-1] + 1
    step = rows[a:b]
    agg = defaultdict(lambda: [0, 0.0])
    for r in step:
        k = agg[short(r["Kernel_Name"])]
        k[0] += 1
        k[1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    busy = sum(v[1] for v in agg.values())
    wall = (int(step[-1]["End_Timestamp"]) - int(step[0]["Start_Timestamp"])) / 1e3
    print(f"last step: wall {wall / 1e3:.2f} ms, kernels {len(step)}, busy {busy / 1e3:.2f} ms")
    for n, (c, t) in sorted(agg.items(), key=lambda x: -x[1][1])[:top]:
        print(f"{t:9.1f} us {c:4d}  {n}")


if __name__ == "__main__":
    main()
