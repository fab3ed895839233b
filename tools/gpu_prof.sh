#!/bin/bash
# GPU session: build, kernel tests, bench, rocprofv3 kernel-trace stats of a short bench.
set -o pipefail
R="$(cd "$(dirname "$0")/.." && pwd)"
cd "$R"
mkdir -p gpurun_out/prof
export HSA_ENABLE_IPC_MODE_LEGACY=0
python csrc/build.py > gpurun_out/build.log 2>&1 || { echo "build failed"; cat gpurun_out/build.log; exit 1; }
if [ -z "$SKIPTEST" ]; then
timeout -k 10 600 python -m pytest tests/ -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -25 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 600 python bench.py --steps ${STEPS:-8} --warmup 3 ${BENCHARGS} > gpurun_out/bench_hip.log 2>&1 || { tail -30 gpurun_out/bench_hip.log; exit 1; }
tail -2 gpurun_out/bench_hip.log
if [ -n "$PROF" ]; then
export TMPDIR=/tmp
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof" -o run -- python "$R/bench.py" --steps 3 --warmup 2 ${BENCHARGS} > "$R/gpurun_out/prof.log" 2>&1 || { tail -30 "$R/gpurun_out/prof.log"; exit 1; }
cd "$R"
f=$(find gpurun_out/prof -name "*kernel_stats.csv" | head -1)
t=$(find gpurun_out/prof -name "*kernel_trace.csv" | head -1)
echo "stats: $f"
python tools/prof_summary.py "$f" "$t"
fi
