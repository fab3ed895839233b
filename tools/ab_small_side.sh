set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() {
  timeout -k 10 300 python bench.py $2 --steps 30 --warmup 5 --synth-steps 0 --synth-b1-runs 0 > gpurun_out/abs.log 2>&1 || { tail -20 gpurun_out/abs.log; exit 1; }
  echo "$1 $(tail -1 gpurun_out/abs.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["host_enqueue_ms_per_step"])')"
}
for rep in 1 2; do
  run "LibriTTS side" "--config LibriTTS"
  run "LibriTTS noside" "--config LibriTTS --no-side-wgrad"
  run "BC2013b10 side" "--config BC2013 --batch 10"
  run "BC2013b10 noside" "--config BC2013 --batch 10 --no-side-wgrad"
done
