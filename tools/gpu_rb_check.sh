set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "resblock or hifigan" > gpurun_out/t_rb.log 2>&1; rc=$?; tail -2 gpurun_out/t_rb.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench_synth.py > gpurun_out/synth_rb.log 2>&1 || { tail -5 gpurun_out/synth_rb.log; exit 1; }
tail -1 gpurun_out/synth_rb.log | cut -c1-200
export TMPDIR=/tmp; R=$PWD; cd /tmp
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmc_rb/synth_sq -o p -- python3 $R/bench_synth.py --steps 1 --warmup 0 --batch 64 > $R/gpurun_out/pmc_rb.log 2>&1 || exit 1
cd $R; python tools/pmc_summary.py gpurun_out/pmc_rb | head -14
