#!/bin/bash
# LJSpeech per-stream split: all CUs vs CU-masked side stream (50 % / 75 %).
set -o pipefail
R="$(cd "$(dirname "$0")/.." && pwd)"
cd "$R"; mkdir -p gpurun_out/ae
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
i=0
for m in "" "--side-cu-mask 0x55555555" "--side-cu-mask 0x77777777"; do
  i=$((i+1))
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/ae/$i" -o run -- python3 "$R/bench.py" --steps 4 --warmup 2 --synth-steps 0 $m > "$R/gpurun_out/ae_$i.log" 2>&1 || { tail -20 "$R/gpurun_out/ae_$i.log"; exit 1; }
  cd "$R"
  t=$(find gpurun_out/ae/$i -name "*kernel_trace.csv" | head -1)
  echo "=== ${m:-allCU}"
  python tools/stream_split.py "$t" --last 2 --detail || exit 1
  rm -rf gpurun_out/ae/$i
done
