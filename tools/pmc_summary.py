#!/usr/bin/env python
"""Aggregate rocprofv3 --pmc counter CSVs per kernel (tools/gpu.sh pmc / synthpmc output).

For each run directory: per kernel name (top by SQ_WAVE_CYCLES or FETCH_SIZE), dispatches,
MFMA busy / GRBM_GUI_ACTIVE (per-dispatch average, ~fraction of the time the matrix cores were
busy, summed over CUs -> divide by the CU count for a per-CU utilisation), the wave-state
split (wait / issue-stall / active), LDS bank-conflict cycles / LDS cycles, and bytes fetched
from HBM (FETCH_SIZE is KiB; on gfx950 it reports half of a wide streaming read, MI355X_MICROARCH.md).
"""
import collections
import csv
import glob
import os
import sys


def load(d):
    fs = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not fs:
        return None
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(fs[0])):
        k = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:58]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
    return agg, disp


def main(root):
    for d in sorted(glob.glob(os.path.join(root, "*"))):
        if not os.path.isdir(d):
            continue
        got = load(d)
        if got is None:
            continue
        agg, disp = got
        print(f"== {os.path.basename(d)}")
        sq = any("SQ_WAVE_CYCLES" in v for v in agg.values())
        key = "SQ_WAVE_CYCLES" if sq else "FETCH_SIZE"
        tot = sum(v.get(key, 0) for v in agg.values()) or 1
        for k, v in sorted(agg.items(), key=lambda kv: -kv[1].get(key, 0))[:18]:
            n = len(disp[k])
            gui = v.get("GRBM_GUI_ACTIVE", 0) or 1
            if sq:
                wc = v.get("SQ_WAVE_CYCLES", 0) or 1
                print(f"  {k:58s} n={n:4d} share={100 * v[key] / tot:5.1f}% mfma_busy/gui={v.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / gui:7.2f} "
                      f"wait={v.get('SQ_WAIT_ANY', 0) / wc:.2f} stall={v.get('SQ_WAIT_INST_ANY', 0) / wc:.2f} "
                      f"active={v.get('SQ_ACTIVE_INST_ANY', 0) / wc:.2f} "
                      f"lds_conf={v.get('SQ_LDS_BANK_CONFLICT', 0) / max(v.get('SQ_LDS_IDX_ACTIVE', 0), 1):.3f}")
            else:
                print(f"  {k:58s} n={n:4d} share={100 * v[key] / tot:5.1f}% fetch_MiB/disp={2 * v[key] / n / 1024:9.1f} "
                      f"(x2 gfx950 streaming correction)")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc_step")
