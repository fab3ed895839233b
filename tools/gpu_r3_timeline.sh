#!/bin/bash
# Round 3 measurements: (1) per-step GPU busy vs idle of the headline bench from a kernel trace,
# (2) host cost of the DP gradient path (1-rank RCCL, forced hooks/buckets) vs plain, phase times,
# (3) LibriTTS multi-speaker bench lines (config batch and a frame budget).
set -o pipefail
R="$(cd "$(dirname "$0")/.." && pwd)"
cd "$R"; mkdir -p gpurun_out/tl
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
B="${BENCHARGS:---config LJSpeech}"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/tl" -o tl -- python3 "$R/bench.py" --steps 10 --warmup 3 --synth-steps 0 $B > "$R/gpurun_out/tl.log" 2>&1 || { tail -20 "$R/gpurun_out/tl.log"; exit 1; }
cd "$R"
t=$(find gpurun_out/tl -name "*kernel_trace.csv" | head -1)
python tools/step_timeline.py "$t" --last 10 --gaps 25 > gpurun_out/timeline.txt
rm -f "$t"
cat gpurun_out/timeline.txt | tail -30
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --synth-steps 0 --phase-times > gpurun_out/ph_plain_$i.log 2>&1 || { tail -20 gpurun_out/ph_plain_$i.log; exit 1; }
  tail -1 gpurun_out/ph_plain_$i.log
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --synth-steps 0 --phase-times --force-buckets > gpurun_out/ph_force_$i.log 2>&1 || { tail -20 gpurun_out/ph_force_$i.log; exit 1; }
  tail -1 gpurun_out/ph_force_$i.log
done
timeout -k 10 300 python bench.py --config LibriTTS --steps 10 --warmup 3 --synth-steps 0 > gpurun_out/b_libritts.log 2>&1 || { tail -20 gpurun_out/b_libritts.log; exit 1; }
tail -1 gpurun_out/b_libritts.log
timeout -k 10 300 python bench.py --config LibriTTS --steps 10 --warmup 3 --synth-steps 0 --frames-per-gpu 160000 > gpurun_out/b_libritts_fb.log 2>&1 || { tail -20 gpurun_out/b_libritts_fb.log; exit 1; }
tail -1 gpurun_out/b_libritts_fb.log
