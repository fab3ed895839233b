set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
for rep in 1 2; do
for c in "--config LibriTTS" "--config BC2013 --batch 10"; do
  for m in auto 1 0; do
    SSAMD_EXPERIMENTAL=side_wgrad=$m timeout -k 10 300 python bench.py $c --steps 30 --warmup 5 --synth-steps 0 --synth-b1-runs 0 > gpurun_out/vb.log 2>&1 || { tail -20 gpurun_out/vb.log; exit 1; }
    echo "[$c side=$m] $(tail -1 gpurun_out/vb.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["host_enqueue_ms_per_step"])')"
  done
done; done
