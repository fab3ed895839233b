#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 200 python tools/dbg_side.py 2>&1 | grep -v Warn | tail -20
