#!/bin/bash
# Same-box per-kernel A/B: rocprofv3 kernel stats of a short training bench with the in-tree
# kernel library (B) and ab/libssamd_kernels_$BASE.so (A); prints the kernels matching $KPAT.
set -o pipefail
R="$(cd "$(dirname "$0")/.." && pwd)"
cd "$R"
mkdir -p gpurun_out/abprof
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
for v in A B; do
  lib=""
  [ $v = A ] && lib="$R/ab/libssamd_kernels_$BASE.so"
  cd /tmp
  SSAMD_KERNEL_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/abprof/$v" -o run -- python3 "$R/bench.py" --steps 5 --warmup 2 --synth-steps 0 --config ${CFG:-LJSpeech} > "$R/gpurun_out/abprof_$v.log" 2>&1 || { tail -20 "$R/gpurun_out/abprof_$v.log"; exit 1; }
  cd "$R"
done
python3 - <<'PY'
import csv, glob, re, os
from collections import defaultdict
pat = re.compile(os.environ.get("KPAT", "."))
def short(n):
    n = n.replace("(anonymous namespace)::", "")
    m = re.match(r"(?:void )?([\w:]+(?:<[^()]*?>)?)", n)
    return (m.group(1) if m else n)[:70]
def load(v, last=3):  # per-kernel time over the LAST `last` steps (Adam-delimited): steady state only
    f = glob.glob(f"gpurun_out/abprof/{v}/**/*kernel_trace.csv", recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    ends = [i for i, r in enumerate(rows) if "adam_kernel" in r["Kernel_Name"] or "adam_img_kernel" in r["Kernel_Name"]]
    out = defaultdict(lambda: [0, 0.0])
    for r in rows[ends[-last - 1] + 1: ends[-1] + 1]:
        k = out[short(r["Kernel_Name"])]
        k[0] += 1
        k[1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    return out
a, b = load("A"), load("B")
ta_all, tb_all = sum(v[1] for v in a.values()), sum(v[1] for v in b.values())
print(f"{'TOTAL (last 3 steps)':70s} A {ta_all:9.1f} us         B {tb_all:9.1f} us")
for n in sorted(set(a) | set(b), key=lambda n: -(b[n][1] if n in b else a[n][1])):
    if not pat.search(n):
        continue
    ca, ta = a[n] if n in a else (0, 0.0)
    cb, tb = b[n] if n in b else (0, 0.0)
    print(f"{n:70s} A {ta:9.1f} us ({ca:4d})  B {tb:9.1f} us ({cb:4d})")
PY
