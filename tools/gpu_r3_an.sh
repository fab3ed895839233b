#!/bin/bash
# Isolated BatchNorm fwd/bwd kernel times (PostNet shape [150000 x 512]) under rocprofv3 --stats.
set -o pipefail
R="$(cd "$(dirname "$0")/.." && pwd)"
cd "$R"; mkdir -p gpurun_out/an
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/an" -o bn -- python3 "$R/tools/exp_bn_bwd.py" > "$R/gpurun_out/an.log" 2>&1 || { tail -20 "$R/gpurun_out/an.log"; exit 1; }
cd "$R"
s=$(find gpurun_out/an -name "*kernel_stats.csv" | head -1)
python -c "
import csv,sys
for r in csv.DictReader(open('$s')):
    print('%-60s n=%5s avg_us=%8.1f' % (r['Name'][:60], r['Calls'], float(r['AverageNs'])/1e3))
" | head -20
find gpurun_out/an -name "*kernel_trace.csv" -delete
