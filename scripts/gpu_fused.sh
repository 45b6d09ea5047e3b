# Fused per-bucket update: single-rank sync tests, then A/B benches (fused vs update-after-backward)
# with the null communicator and a forced 1-rank RCCL communicator, plus a kernel trace.
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "sync_modes or sgd" > gpurun_out/fused_tests.log 2>&1 || { tail -30 gpurun_out/fused_tests.log; exit 1; }
tail -1 gpurun_out/fused_tests.log
for cfg in "1 0" "0 0" "1 1" "0 1"; do
  set -- $cfg
  DPA_FUSED_STEP=$1 DPA_FORCE_COMM=$2 timeout -k 10 150 python bench.py --steps 50 --warmup 10 > gpurun_out/bench_f$1_c$2.log 2>&1
  echo "fused=$1 forcecomm=$2 $(grep -o '"value": [0-9.]*' gpurun_out/bench_f$1_c$2.log)"
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 > $R/gpurun_out/prof.log 2>&1
echo prof-ok
