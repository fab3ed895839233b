#!/usr/bin/env python
"""Which HIP API call enqueued each __amd_rocclr_copyBuffer kernel of the last step (rocprofv3 --hip-trace
--kernel-trace CSVs), and the main-stream idle time before the next kernel.
Usage: python tools/copy_origin.py DIR"""
import csv
import glob
import os
import sys


def main(d):
    kt = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    ht = glob.glob(os.path.join(d, "**", "*hip_api_trace.csv"), recursive=True)
    ks = sorted(csv.DictReader(open(kt)), key=lambda r: int(r["Start_Timestamp"]))
    api = {}
    if ht:
        for r in csv.DictReader(open(ht[0])):
            api[r.get("Correlation_Id")] = r
    adam = [i for i, r in enumerate(ks) if "adam" in r["Kernel_Name"]]
    lo = adam[-2] if len(adam) > 1 else 0
    seg = ks[lo + 1:adam[-1] + 1]
    for i, r in enumerate(seg):
        if "copyBuffer" not in r["Kernel_Name"]:
            continue
        nxt = seg[i + 1] if i + 1 < len(seg) else None
        a = api.get(r.get("Correlation_Id"), {})
        gap = (int(nxt["Start_Timestamp"]) - int(r["End_Timestamp"])) / 1e3 if nxt else 0
        print(f"copyBuffer corr={r.get('Correlation_Id')} stream={r.get('Stream_Id')} dur="
              f"{(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3:.1f}us gap_after={gap:.1f}us "
              f"api={a.get('Function', '?')} args={a.get('Args', '')[:160]}")
    # host timeline around the copies: API calls (host clock = kernel clock in rocprofv3)
    cps = [r for r in seg if "copyBuffer" in r["Kernel_Name"]]
    if cps and api:
        c0 = int(cps[0]["Correlation_Id"]) - 3
        c1 = int(cps[-1]["Correlation_Id"]) + 25
        kby = {r.get("Correlation_Id"): r for r in seg}
        t_ref = int(cps[0]["Start_Timestamp"])
        for c in range(c0, c1):
            a = api.get(str(c))
            if not a:
                continue
            k = kby.get(str(c))
            kt = f" -> GPU {(int(k['Start_Timestamp']) - t_ref) / 1e3:9.1f}us {k['Kernel_Name'][:40]}" if k else ""
            print(f"  api {c} host {(int(a['Start_Timestamp']) - t_ref) / 1e3:9.1f}us "
                  f"dur {(int(a['End_Timestamp']) - int(a['Start_Timestamp'])) / 1e3:7.1f}us {a['Function']}{kt}")


if __name__ == "__main__":
    main(sys.argv[1])
