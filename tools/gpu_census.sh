#!/bin/bash
# GEMM census (tools/gemm_census.py) of the configs in $CONFIGS, then (PROF=1) a rocprofv3
# kernel-trace profile of the LJSpeech training step.  Each GPU step has its own time limit.
set -o pipefail
R="$(cd "$(dirname "$0")/.." && pwd)"
cd "$R"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for cfg in ${CONFIGS:-LJSpeech}; do
  timeout -k 10 400 python tools/gemm_census.py --config $cfg > gpurun_out/census_$cfg.jsonl 2> gpurun_out/census_$cfg.err || { tail -20 gpurun_out/census_$cfg.err; exit 1; }
  tail -1 gpurun_out/census_$cfg.jsonl
done
if [ -n "$PROF" ]; then
  TAG=${TAG:-prof_train}
  mkdir -p gpurun_out/$TAG
  export TMPDIR=/tmp
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/$TAG" -o run -- python3 "$R/bench.py" --steps 3 --warmup 2 --synth-steps 0 ${PROFARGS} > "$R/gpurun_out/$TAG.log" 2>&1 || { tail -30 "$R/gpurun_out/$TAG.log"; exit 1; }
  cd "$R"
  f=$(find gpurun_out/$TAG -name "*kernel_stats.csv" | head -1)
  t=$(find gpurun_out/$TAG -name "*kernel_trace.csv" | head -1)
  python tools/prof_summary.py "$f" "$t" > gpurun_out/${TAG}_summary.txt
  sed -n '/last step/,$p' gpurun_out/${TAG}_summary.txt | head -60
fi
