#!/bin/bash
set -o pipefail
R="$(cd "$(dirname "$0")/.." && pwd)"
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_vocoder_oracle_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/oracle.log 2>&1 || { tail -40 gpurun_out/oracle.log; exit 1; }
tail -8 gpurun_out/oracle.log
for c in LJSpeech BC2013; do
  mkdir -p gpurun_out/tl_$c
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/tl_$c" -o tl -- python3 "$R/bench.py" --steps 10 --warmup 3 --synth-steps 0 --config $c > "$R/gpurun_out/tl_$c.log" 2>&1 || { tail -20 "$R/gpurun_out/tl_$c.log"; exit 1; }
  cd "$R"
  t=$(find gpurun_out/tl_$c -name "*kernel_trace.csv" | head -1)
  python tools/step_timeline.py "$t" --last 10 --gaps 15 --top 70 > gpurun_out/timeline_$c.txt
  rm -rf gpurun_out/tl_$c
  head -14 gpurun_out/timeline_$c.txt
done
