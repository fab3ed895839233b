#!/bin/bash
set -o pipefail
R="$(cd "$(dirname "$0")/.." && pwd)"
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 200 python tools/exp_short_k.py 113000 2>&1 | tee gpurun_out/exp_short_k.jsonl
