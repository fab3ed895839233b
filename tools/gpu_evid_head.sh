set -o pipefail
cd /root/repo
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python tools/exp_hifigan_train.py > gpurun_out/r2_v11_hifigan_train_ab.jsonl 2> gpurun_out/hg.err && \
TAG=r2_v11_train_LJSpeech timeout -k 10 400 bash tools/gpu_prof_head.sh && \
TAG=r2_v11_train_BC2013 BENCHARGS="--config BC2013" timeout -k 10 400 bash tools/gpu_prof_head.sh
