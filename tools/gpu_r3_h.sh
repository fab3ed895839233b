#!/bin/bash
# Round 3: length-bucketed vocoder -- GPU tests, RTF A/B (8 buckets vs padded), synth profile.
set -o pipefail
R="$(cd "$(dirname "$0")/.." && pwd)"
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_vocoder_oracle_gpu.py -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_voc.log 2>&1 || { tail -40 gpurun_out/pytest_voc.log; exit 1; }
tail -2 gpurun_out/pytest_voc.log
for vb in 8 1 4; do
  timeout -k 10 300 python bench_synth.py --vocoder-buckets $vb > gpurun_out/bs.log 2>&1 || { tail -20 gpurun_out/bs.log; exit 1; }
  tail -1 gpurun_out/bs.log | python -c "import sys,json; r=json.loads(sys.stdin.read()); print('buckets $vb', r['value'], r['wall_s'], r['audio_seconds'])"
done
timeout -k 10 300 python bench_synth.py --config BC2013 > gpurun_out/bs.log 2>&1 || { tail -20 gpurun_out/bs.log; exit 1; }
tail -1 gpurun_out/bs.log
TAG=r3_synth_gst bash tools/gpu_prof_synth.sh
