#!/bin/bash
# bench.py at the driver's default invocation, synth-only runs for both style configs,
# rocprofv3 kernel-trace stats of the synthesis path.  Pre-built tree; every GPU step
# has its own limit and the script stops at the first failure.
set -o pipefail
R="$(cd "$(dirname "$0")/.." && pwd)"
cd "$R"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python bench.py ${BENCHARGS:---steps 20 --warmup 5} > gpurun_out/bench_main.log 2>&1 || { tail -30 gpurun_out/bench_main.log; exit 1; }
tail -1 gpurun_out/bench_main.log
for cfg in ${SYNTHCFGS:-BC2013 BC2013_GST LJSpeech}; do
  timeout -k 10 300 python bench_synth.py --config $cfg > gpurun_out/synth_$cfg.log 2>&1 || { tail -30 gpurun_out/synth_$cfg.log; exit 1; }
  tail -1 gpurun_out/synth_$cfg.log
done
if [ -n "$PROF" ]; then
TAG=${TAG:-prof_synth}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/$TAG" -o run -- python3 "$R/bench_synth.py" --steps 2 --warmup 1 ${SYNTHARGS} > "$R/gpurun_out/$TAG.log" 2>&1 || { tail -30 "$R/gpurun_out/$TAG.log"; exit 1; }
cd "$R"
f=$(find gpurun_out/$TAG -name "*kernel_stats.csv" | head -1)
t=$(find gpurun_out/$TAG -name "*kernel_trace.csv" | head -1)
python tools/prof_summary.py "$f" "$t" > gpurun_out/${TAG}_summary.txt
head -45 gpurun_out/${TAG}_summary.txt
fi
