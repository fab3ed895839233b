#!/bin/bash
# LJSpeech step tail: the last kernels of both streams before the optimizer.
set -o pipefail
R="$(cd "$(dirname "$0")/.." && pwd)"
cd "$R"; mkdir -p gpurun_out/af
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/af/1" -o run -- python3 "$R/bench.py" --steps 4 --warmup 2 --synth-steps 0 > "$R/gpurun_out/af_1.log" 2>&1 || { tail -20 "$R/gpurun_out/af_1.log"; exit 1; }
cd "$R"
t=$(find gpurun_out/af/1 -name "*kernel_trace.csv" | head -1)
python tools/stream_split.py "$t" --last 1 --tail 40 || exit 1
rm -rf gpurun_out/af/1
