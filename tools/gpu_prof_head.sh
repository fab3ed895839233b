#!/bin/bash
# At-HEAD evidence (GPU box): rocprofv3 kernel-trace stats of the LJSpeech training step (TAG, bench
# args in BENCHARGS) -> gpurun_out/<TAG>_summary.txt + last steady-state step table.  Each GPU step
# has its own time limit; the script stops at the first failure.
set -o pipefail
R="$(cd "$(dirname "$0")/.." && pwd)"
cd "$R"
TAG=${TAG:-prof_head}
mkdir -p gpurun_out/$TAG
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/$TAG" -o run -- python3 "$R/bench.py" --steps 3 --warmup 2 --synth-steps 0 ${BENCHARGS} > "$R/gpurun_out/$TAG.log" 2>&1 || { tail -30 "$R/gpurun_out/$TAG.log"; exit 1; }
cd "$R"
f=$(find gpurun_out/$TAG -name "*kernel_stats.csv" | head -1)
t=$(find gpurun_out/$TAG -name "*kernel_trace.csv" | head -1)
python tools/prof_summary.py "$f" "$t" > gpurun_out/${TAG}_summary.txt
python tools/last_step.py "$t" 60 > gpurun_out/${TAG}_last_step.txt
cp "$f" gpurun_out/${TAG}_kernel_stats.csv
rm -f "$t"
head -3 gpurun_out/${TAG}_last_step.txt
