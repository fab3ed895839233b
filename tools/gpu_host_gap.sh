#!/bin/bash
# Host/device timeline of the training step: rocprofv3 kernel + HIP runtime traces (no counters).
set -o pipefail
R="$(cd "$(dirname "$0")/.." && pwd)"
cd "$R"; mkdir -p gpurun_out/hostgap
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d "$R/gpurun_out/hostgap" -o h -- python3 "$R/bench.py" --steps 3 --warmup 2 --synth-steps 0 ${BENCHARGS} > "$R/gpurun_out/hostgap.log" 2>&1 || { tail -20 "$R/gpurun_out/hostgap.log"; exit 1; }
cd "$R"
k=$(find gpurun_out/hostgap -name "*kernel_trace.csv" | head -1)
h=$(find gpurun_out/hostgap -name "*hip_api_trace.csv" | head -1)
python tools/host_gap.py "$k" "$h" gpurun_out/hostgap_timeline.csv > gpurun_out/hostgap_summary.txt
rm -f "$k" "$h"
cat gpurun_out/hostgap_summary.txt
