#!/bin/bash
# rocprofv3 PMC counters of whole training / synthesis steps (one counter pass per run, kernel
# trace only -- no sys/runtime traces with --pmc).  Summaries: tools/pmc_summary.py.
set -o pipefail
R="$(cd "$(dirname "$0")/.." && pwd)"
cd "$R"; mkdir -p gpurun_out/pmc_step
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
SQ="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
MEM="FETCH_SIZE GRBM_GUI_ACTIVE"
run() {  # tag counters args...
  local tag=$1 ctr=$2; shift 2
  cd /tmp
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $ctr --output-format csv -d "$R/gpurun_out/pmc_step/$tag" -o p -- python3 "$@" > "$R/gpurun_out/pmc_step/$tag.log" 2>&1 || { tail -20 "$R/gpurun_out/pmc_step/$tag.log"; return 1; }
  cd "$R"
}
run train_sq "$SQ" "$R/bench.py" --steps 1 --warmup 1 --synth-steps 0 &&
run train_mem "$MEM" "$R/bench.py" --steps 1 --warmup 1 --synth-steps 0 &&
run synth_sq "$SQ" "$R/bench_synth.py" --steps 1 --warmup 0 --batch 64 &&
run synth_mem "$MEM" "$R/bench_synth.py" --steps 1 --warmup 0 --batch 64 &&
python tools/pmc_summary.py gpurun_out/pmc_step > gpurun_out/pmc_step/summary.txt && head -60 gpurun_out/pmc_step/summary.txt
