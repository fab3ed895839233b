"""Per (kernel, grid, LDS) time of the last training step in a rocprofv3 kernel-trace CSV: tells the
shapes apart behind one kernel template (e.g. which conv_gemm_big64 launches cost the most).
Usage: python tools/grid_census.py <kernel_trace.csv> [--top N] [--match SUBSTR]"""
import argparse
import csv
import re
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--match", default="")
    ap.add_argument("--all", action="store_true", help="the whole trace (synthesis: no optimizer-step marker)")
    a = ap.parse_args()
    kt = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    ends = [i for i, r in enumerate(kt) if re.search(r"adam(_img)?_kernel", r["Kernel_Name"])]
    step = kt if (a.all or len(ends) < 2) else kt[ends[-2] + 1: ends[-1] + 1]
    agg = defaultdict(lambda: [0, 0.0])
    for r in step:
        n = r["Kernel_Name"]
        if a.match and a.match not in n:
            continue
        n = n.replace("void ", "").replace("(anonymous namespace)::", "")
        n = re.sub(r"\(.*", "", n)
        key = (n[:60], r.get("Grid_Size_X", r.get("Grid_Size", "?")), r.get("Grid_Size_Y", "1"),
               r.get("LDS_Block_Size", r.get("Lds_Size", "?")), r.get("Stream_Id", "?"))
        e = agg[key]
        e[0] += 1
        e[1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    tot = sum(v[1] for v in agg.values())
    print(f"{'whole trace' if step is kt else 'last step'}: {len(step)} kernels, {tot:.1f} us kernel time (both streams)")
    print(f"{'us':>9} {'n':>4} {'us/launch':>9}  q  gridX x gridY  lds  kernel")
    for (n, gx, gy, lds, q), (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:a.top]:
        print(f"{t:9.1f} {c:4d} {t / c:9.1f}  {q}  {gx:>7} x {gy:<3} {lds:>6}  {n}")


if __name__ == "__main__":
    main()
