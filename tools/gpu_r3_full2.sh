#!/bin/bash
# Remaining GPU tests (from the fidelity test on) + benches + timeline (round 3).
set -o pipefail
R="$(cd "$(dirname "$0")/.." && pwd)"
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q -s --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu2.log 2>&1 || { tail -60 gpurun_out/pytest_gpu2.log; exit 1; }
grep -E "loss hip|passed|failed" gpurun_out/pytest_gpu2.log
for c in LJSpeech BC2013 BC2013_GST; do
  timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 3 --synth-steps 0 > gpurun_out/b_$c.log 2>&1 || { tail -20 gpurun_out/b_$c.log; exit 1; }
  tail -1 gpurun_out/b_$c.log | python -c "import sys,json; r=json.loads(sys.stdin.read()); print(r['config']['model'], r['value'], r['ms_per_step'])"
done
mkdir -p gpurun_out/tl_LJ
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/tl_LJ" -o tl -- python3 "$R/bench.py" --steps 10 --warmup 3 --synth-steps 0 > "$R/gpurun_out/tl_LJ.log" 2>&1 || { tail -20 "$R/gpurun_out/tl_LJ.log"; exit 1; }
cd "$R"
t=$(find gpurun_out/tl_LJ -name "*kernel_trace.csv" | head -1)
python tools/step_timeline.py "$t" --last 10 --gaps 15 --top 60 > gpurun_out/timeline_LJSpeech.txt
rm -rf gpurun_out/tl_LJ
sed -n 11,45p gpurun_out/timeline_LJSpeech.txt
BENCHARGS="--config BC2013" timeout -k 10 400 bash tools/gpu_host_gap.sh > gpurun_out/hostgap_BC2013.txt 2>&1 || { tail -20 gpurun_out/hostgap_BC2013.txt; exit 1; }
head -30 gpurun_out/hostgap_BC2013.txt
