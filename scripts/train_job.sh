#!/bin/bash
# SLURM job: FastSpeech2 / speaking-style training on MI355X nodes, one process per GPU
# (counterpart of the reference's scripts/train_job.sh, which ran a single DataParallel process).
#
#   sbatch scripts/train_job.sh                                  # BC2013, 1 node x 8 GPUs
#   CONFIG=LJSpeech GPUS=8 NODES=2 sbatch --nodes=2 scripts/train_job.sh
#   bash scripts/train_job.sh                                    # same, outside SLURM (one node)
#
# Each rank drives one GCD through HIP; gradients are all-reduced with RCCL over xGMI
# (torch.distributed backend "nccl" is RCCL on ROCm).  `optimizer.batch_size` in train.yaml is the
# GLOBAL batch: every rank trains on batch_size / world of each group (train/loop.py).
#
#SBATCH --job-name=speakingstyle_amd
#SBATCH --partition=gpu
#SBATCH --nodes=1
#SBATCH --ntasks-per-node=1
#SBATCH --gres=gpu:8
#SBATCH --cpus-per-task=64
#SBATCH --time=24:00:00
#SBATCH --output=logs/slurm-%j.out
set -euo pipefail

CONFIG=${CONFIG:-BC2013}
GPUS=${GPUS:-8}
NODES=${NODES:-${SLURM_JOB_NUM_NODES:-1}}
PORT=${PORT:-29511}
RESTORE=${RESTORE:-0}
EXTRA=${EXTRA:-}

cd "${SLURM_SUBMIT_DIR:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p logs

# RCCL / HIP environment for multi-process GPU work on this image
export HSA_ENABLE_IPC_MODE_LEGACY=0          # dmabuf IPC (RCCL peer buffers, CUDA-tensor sharing)
export TORCH_NCCL_ASYNC_ERROR_HANDLING=1     # a failed collective aborts the job instead of hanging
export NCCL_DEBUG=${NCCL_DEBUG:-WARN}
export OMP_NUM_THREADS=${OMP_NUM_THREADS:-8}

# kernel library (in-tree, gfx950); a no-op when already built
[ -n "${SKIP_BUILD:-}" ] || python csrc/build.py

if [ "${NODES}" -gt 1 ]; then
  MASTER_ADDR=$(scontrol show hostnames "${SLURM_JOB_NODELIST}" | head -n 1)
  RDZV=(--nnodes="${NODES}" --rdzv-backend=c10d --rdzv-endpoint="${MASTER_ADDR}:${PORT}" --rdzv-id="${SLURM_JOB_ID}")
  LAUNCH=(srun --ntasks-per-node=1 python -m torch.distributed.run)
else
  RDZV=(--nnodes=1 --master-addr=127.0.0.1 --master-port="${PORT}")
  LAUNCH=(python -m torch.distributed.run)
fi

echo "job ${SLURM_JOB_ID:-local} on ${SLURM_JOB_NODELIST:-$(hostname)}: ${NODES} node(s) x ${GPUS} GPU(s), config ${CONFIG}"
date '+started %d/%m/%Y %H:%M:%S'
"${LAUNCH[@]}" "${RDZV[@]}" --nproc-per-node="${GPUS}" train.py \
  -p "config/${CONFIG}/preprocess.yaml" -m "config/${CONFIG}/model.yaml" -t "config/${CONFIG}/train.yaml" \
  --restore_step "${RESTORE}" ${EXTRA}
date '+finished %d/%m/%Y %H:%M:%S'
