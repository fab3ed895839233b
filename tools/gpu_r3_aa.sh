#!/bin/bash
# Synthesis two-stream pipeline A/B (bench_synth.py, two repetitions) + vocoder GPU tests.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_vocoder_oracle_gpu.py tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "hifigan or vocod or whole_block or resblock or bucket" > gpurun_out/aa_pytest.log 2>&1 || { tail -30 gpurun_out/aa_pytest.log; exit 1; }
tail -1 gpurun_out/aa_pytest.log
for rep in 1 2; do
  for f in "" "--synth-serial"; do
    timeout -k 10 200 python bench_synth.py $f > gpurun_out/aa_s.log 2>&1 || { tail -20 gpurun_out/aa_s.log; exit 1; }
    tail -1 gpurun_out/aa_s.log | python -c "import sys,json; r=json.loads(sys.stdin.read()); print('synth', '${f:-pipelined}', r['value'], r['wall_s'], r['audio_seconds'])"
  done
done
timeout -k 10 240 python bench.py > gpurun_out/aa_bench.log 2>&1 || { tail -20 gpurun_out/aa_bench.log; exit 1; }
tail -1 gpurun_out/aa_bench.log
