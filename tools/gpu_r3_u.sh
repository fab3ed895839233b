#!/bin/bash
# LJSpeech / BC2013 per-stream step split (main vs weight-gradient side stream) from a kernel trace;
# BC2013 bench at an HBM-sized per-GPU frame budget.
set -o pipefail
R="$(cd "$(dirname "$0")/.." && pwd)"
cd "$R"; mkdir -p gpurun_out/u
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
for c in LJSpeech BC2013; do
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/u/$c" -o run -- python3 "$R/bench.py" --config $c --steps 4 --warmup 2 --synth-steps 0 > "$R/gpurun_out/u_$c.log" 2>&1 || { tail -20 "$R/gpurun_out/u_$c.log"; exit 1; }
  cd "$R"
  t=$(find gpurun_out/u/$c -name "*kernel_trace.csv" | head -1)
  python tools/stream_split.py "$t" --last 2 --detail > gpurun_out/u_split_$c.txt 2>&1 || { tail -20 gpurun_out/u_split_$c.txt; exit 1; }
  cat gpurun_out/u_split_$c.txt
  rm -rf gpurun_out/u/$c
done
timeout -k 10 240 python bench.py --config BC2013 --synth-steps 0 --frames-per-gpu 200000 > gpurun_out/u_bc_budget.log 2>&1 || { tail -20 gpurun_out/u_bc_budget.log; exit 1; }
tail -1 gpurun_out/u_bc_budget.log
