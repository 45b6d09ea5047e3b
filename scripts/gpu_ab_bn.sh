# A/B of the BN backward reduce grid (DPA_BN_BWD_BLOCKS) on the headline bench, 2 interleaved rounds.
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_ops_gpu.py -x -q -k "bn" --timeout 100 --timeout-method thread > gpurun_out/ab_bn_tests.log 2>&1 || { tail -30 gpurun_out/ab_bn_tests.log; exit 1; }
tail -1 gpurun_out/ab_bn_tests.log
for r in 1 2; do
for nb in 1024 512 256; do
  DPA_BN_BWD_BLOCKS=$nb timeout -k 10 120 python bench.py --steps 100 --warmup 20 --diag-steps 0 > gpurun_out/ab_bn_$nb.log 2>&1
  echo "nb=$nb $(grep -o '"value": [0-9.]*' gpurun_out/ab_bn_$nb.log)"
done
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof2 -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --diag-steps 0 > $R/gpurun_out/prof2.log 2>&1
echo prof-ok
