#!/bin/bash
# Baseline GPU session on a pre-built tree: GPU tests, training bench for each config,
# synthesis bench on the styled config, rocprofv3 kernel-trace stats of the training step.
# Every GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
R="$(cd "$(dirname "$0")/.." && pwd)"
cd "$R"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
if [ -z "$SKIPTEST" ]; then
timeout -k 10 900 python -u -m pytest tests/ -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -8 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
fi
for cfg in ${CONFIGS:-LJSpeech BC2013 BC2013_GST}; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --config $cfg ${BENCHARGS} > gpurun_out/bench_$cfg.log 2>&1 || { tail -30 gpurun_out/bench_$cfg.log; exit 1; }
  tail -1 gpurun_out/bench_$cfg.log
done
if [ -n "$SYNTH" ]; then
timeout -k 10 300 python bench_synth.py --config ${SYNTHCFG:-BC2013} --steps 3 --warmup 1 > gpurun_out/bench_synth.log 2>&1 || { tail -30 gpurun_out/bench_synth.log; exit 1; }
tail -1 gpurun_out/bench_synth.log
fi
if [ -n "$PROF" ]; then
TAG=${TAG:-prof_train}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/$TAG" -o run -- python3 "$R/bench.py" --steps 3 --warmup 2 ${PROFARGS} > "$R/gpurun_out/$TAG.log" 2>&1 || { tail -30 "$R/gpurun_out/$TAG.log"; exit 1; }
cd "$R"
f=$(find gpurun_out/$TAG -name "*kernel_stats.csv" | head -1)
t=$(find gpurun_out/$TAG -name "*kernel_trace.csv" | head -1)
python tools/prof_summary.py "$f" "$t" > gpurun_out/${TAG}_summary.txt
head -40 gpurun_out/${TAG}_summary.txt
fi
