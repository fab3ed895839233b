set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$(pwd)
mkdir -p gpurun_out/hgprof
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/hgprof" -o run -- python3 "$R/tools/exp_hifigan_train.py" hip > "$R/gpurun_out/hgprof.log" 2>&1) || { tail -20 gpurun_out/hgprof.log; exit 1; }
f=$(find gpurun_out/hgprof -name "*kernel_stats.csv" | head -1); t=$(find gpurun_out/hgprof -name "*kernel_trace.csv" | head -1)
python tools/prof_summary.py "$f" "$t" > gpurun_out/r5_hifigan_train_prof.txt; rm -rf gpurun_out/hgprof
head -30 gpurun_out/r5_hifigan_train_prof.txt
TAG=r5lt BENCHARGS="--config LibriTTS" bash tools/gpu.sh prof || exit 1
for c in "BC2013" "BC2013_GST" "BC2013 --batch 10" "LibriTTS"; do
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 --synth-steps 0 --synth-b1-runs 0 > gpurun_out/cfg.log 2>&1 || { tail -20 gpurun_out/cfg.log; exit 1; }
  echo "$c: $(tail -1 gpurun_out/cfg.log)" >> gpurun_out/r5_cfg_bench.txt
done
cut -c1-300 gpurun_out/r5_cfg_bench.txt
