#!/bin/bash
# Per-(kernel, grid) census of one LJSpeech and one BC2013 training step (kernel trace only).
set -o pipefail
R="$(cd "$(dirname "$0")/.." && pwd)"
cd "$R"; mkdir -p gpurun_out/al
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
for c in LJSpeech BC2013; do
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/al/$c" -o run -- python3 "$R/bench.py" --config $c --steps 3 --warmup 2 --pool 1 --synth-steps 0 > "$R/gpurun_out/al_$c.log" 2>&1 || { tail -20 "$R/gpurun_out/al_$c.log"; exit 1; }
  cd "$R"
  t=$(find gpurun_out/al/$c -name "*kernel_trace.csv" | head -1)
  python tools/grid_census.py "$t" --top 60 > gpurun_out/al_census_$c.txt || exit 1
  python tools/stream_split.py "$t" --last 1 --detail >> gpurun_out/al_census_$c.txt || exit 1
  head -45 gpurun_out/al_census_$c.txt
  rm -rf gpurun_out/al/$c
done
