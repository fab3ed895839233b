#!/usr/bin/env python
"""Host vs device timeline of the LAST training step from a rocprofv3 run with --kernel-trace and
--hip-runtime-trace (CSV): per kernel, the lead of its launch call over the kernel start (< ~20 us:
the GPU was waiting for the host), idle gaps attributed to the host calls issued in them, and any
synchronising / allocating HIP calls inside the step.
Usage: python tools/host_gap.py <kernel_trace.csv> <hip_api_trace.csv>"""
import csv
import re
import sys
from collections import Counter


def main():
    kt = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    api = sorted(csv.DictReader(open(sys.argv[2])), key=lambda r: int(r["Start_Timestamp"]))
    ends = [i for i, r in enumerate(kt) if re.search(r"adam(_img)?_kernel", r["Kernel_Name"])]
    a, b = ends[-2] + 1, ends[-1] + 1
    step = kt[a:b]
    t0, t1 = int(step[0]["Start_Timestamp"]), int(step[-1]["End_Timestamp"])
    launches = [r for r in api if "Launch" in r["Function"] or "launch" in r["Function"]]
    by_corr = {r.get("Correlation_Id"): r for r in launches}
    idle = 0
    waits = Counter()
    prev_end = None
    lead_small = 0
    for r in step:
        s = int(r["Start_Timestamp"])
        lr = by_corr.get(r.get("Correlation_Id"))
        lead = (s - int(lr["End_Timestamp"])) / 1e3 if lr else None
        if prev_end is not None and s > prev_end:
            gap = (s - prev_end) / 1e3
            idle += gap
            if gap > 20:
                waits[re.sub(r"\(anonymous namespace\)::", "", r["Kernel_Name"]).split("(")[0][:70]] += gap
        if lead is not None and lead < 20:
            lead_small += 1
        prev_end = max(prev_end or 0, int(r["End_Timestamp"]))
    if len(sys.argv) > 3:  # compact per-kernel timeline of the step: name, start, end, launch-call end (us)
        with open(sys.argv[3], "w") as f:
            f.write("name,start_us,end_us,launch_end_us\n")
            for r in step:
                lr = by_corr.get(r.get("Correlation_Id"))
                nm = re.sub(r"\(anonymous namespace\)::", "", r["Kernel_Name"]).split("(")[0][:70].replace(",", ";")
                le = (int(lr["End_Timestamp"]) - t0) / 1e3 if lr else -1
                f.write(f"{nm},{(int(r['Start_Timestamp']) - t0) / 1e3:.1f},{(int(r['End_Timestamp']) - t0) / 1e3:.1f},{le:.1f}\n")
    print(f"last step: wall {(t1 - t0) / 1e6:.2f} ms, kernels {len(step)}, idle {idle / 1e3:.2f} ms, "
          f"kernels launched < 20 us before they started: {lead_small}")
    calls = Counter()
    dur = Counter()
    for r in api:
        s = int(r["Start_Timestamp"])
        if t0 - 5_000_000 <= s <= t1:
            calls[r["Function"]] += 1
            dur[r["Function"]] += (int(r["End_Timestamp"]) - s) / 1e3
    print("HIP API calls in [step start - 5 ms, step end] (count, total us):")
    for f, n in calls.most_common(25):
        print(f"  {n:6d} {dur[f]:10.1f}  {f}")
    print("idle > 20 us before (kernel: total us):")
    for k, v in waits.most_common(15):
        print(f"  {v:8.1f}  {k}")


if __name__ == "__main__":
    main()
