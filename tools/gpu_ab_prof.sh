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
pat = re.compile(os.environ.get("KPAT", "."))
def load(v):
    f = glob.glob(f"gpurun_out/abprof/{v}/**/*kernel_stats.csv", recursive=True)[0]
    out = {}
    for r in csv.DictReader(open(f)):
        n = r["Name"].replace("(anonymous namespace)::", "")
        n = re.sub(r"\(.*", "", n)[:70]
        out[n] = (int(r["Calls"]), float(r["TotalDurationNs"]) / 1e3)
    return out
a, b = load("A"), load("B")
for n in sorted(set(a) | set(b), key=lambda n: -(b.get(n, a.get(n))[1])):
    if not pat.search(n):
        continue
    ca, ta = a.get(n, (0, 0.0)); cb, tb = b.get(n, (0, 0.0))
    print(f"{n:70s} A {ta:9.1f} us ({ca:4d})  B {tb:9.1f} us ({cb:4d})")
PY
