set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests/test_ddp_gpu.py tests/test_train_gpu.py tests/test_graphs_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/vt2.log 2>&1 || { tail -30 gpurun_out/vt2.log; exit 1; }
tail -1 gpurun_out/vt2.log
for c in "--config LibriTTS" "--config BC2013 --batch 10" "--config BC2013_GST" ""; do
  timeout -k 10 300 python bench.py $c --steps 20 --warmup 5 --synth-steps 0 --synth-b1-runs 0 > gpurun_out/vb.log 2>&1 || { tail -20 gpurun_out/vb.log; exit 1; }
  echo "[$c] $(tail -1 gpurun_out/vb.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["host_enqueue_ms_per_step"])')"
done
