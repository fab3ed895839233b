#!/bin/bash
# rocprofv3 kernel-trace + stats of bench_synth.py (pre-built tree).
set -o pipefail
R="$(cd "$(dirname "$0")/.." && pwd)"
cd "$R"
TAG=${TAG:-prof_synth}
mkdir -p gpurun_out/$TAG
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python bench_synth.py ${SYNTHARGS} > gpurun_out/${TAG}_bench.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench.log
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/$TAG" -o run -- python3 "$R/bench_synth.py" --steps 2 --warmup 1 ${SYNTHARGS} > "$R/gpurun_out/$TAG.log" 2>&1 || { tail -30 "$R/gpurun_out/$TAG.log"; exit 1; }
cd "$R"
f=$(find gpurun_out/$TAG -name "*kernel_stats.csv" | head -1)
t=$(find gpurun_out/$TAG -name "*kernel_trace.csv" | head -1)
python tools/prof_summary.py "$f" "$t" > gpurun_out/${TAG}_summary.txt
head -30 gpurun_out/${TAG}_summary.txt
