#!/bin/bash
set -o pipefail
R="$(cd "$(dirname "$0")/.." && pwd)"
cd "$R"; mkdir -p gpurun_out/pmc
[ -n "$REBUILD" ] && { python csrc/build.py > gpurun_out/build.log 2>&1 || exit 1; }
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --pmc ${COUNTERS:-SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE} --output-format csv -d "$R/gpurun_out/pmc" -o p1 -- python "$R/${PMC_TARGET:-tools/pmc_target.py}" > "$R/gpurun_out/pmc1.log" 2>&1 || { tail -20 "$R/gpurun_out/pmc1.log"; exit 1; }
cd "$R"
python - <<'PY'
import csv, glob, collections
f = glob.glob("gpurun_out/pmc/**/*counter_collection.csv", recursive=True)
print(f)
rows = list(csv.DictReader(open(f[0])))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(set)
for r in rows:
    k = r["Kernel_Name"][:60]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    cnt[k].add(r["Dispatch_Id"])
for k, d in agg.items():
    n = len(cnt[k])
    wc = d.get("SQ_WAVE_CYCLES", 0) or 1
    print(f"{k} dispatches={n}")
    print("   " + "  ".join(f"{c}={v/n:.3g}" for c, v in sorted(d.items())))
    if "SQ_WAIT_ANY" in d:
        print(f"   wait_any {d['SQ_WAIT_ANY']/wc:.2f} wait_inst {d['SQ_WAIT_INST_ANY']/wc:.2f} active {d['SQ_ACTIVE_INST_ANY']/wc:.2f}"
              f" lds_conflict/lds_active {d['SQ_LDS_BANK_CONFLICT']/max(d['SQ_LDS_IDX_ACTIVE'],1):.3f}"
              f" mfma_busy/gui {d['SQ_VALU_MFMA_BUSY_CYCLES']/max(d['GRBM_GUI_ACTIVE'],1):.3f}")
PY
