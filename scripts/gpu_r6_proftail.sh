#!/bin/bash
# Kernel traces of the headline step with and without the BN finalize tail
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd /tmp
for v in 0 1; do
  DPA_BN_TAIL=$v timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/tail$v -o run -- python3 $R/bench.py --steps 20 --warmup 5 > $R/gpurun_out/tail$v.log 2>&1 || { tail -20 $R/gpurun_out/tail$v.log; exit 1; }
  f=$(find $R/gpurun_out/tail$v -name "*kernel_trace.csv" | head -1)
  python3 $R/tools/trace_step.py $f --step -3 > $R/gpurun_out/tail${v}_timeline.txt || exit 1
done
grep -E "bn_bwd|span" $R/gpurun_out/tail0_timeline.txt $R/gpurun_out/tail1_timeline.txt
