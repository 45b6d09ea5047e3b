# ResNet-50 kernel-trace profile (8 steps) + the new wide BN backward test.
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -k "wide_geometry" -x -q --timeout 150 --timeout-method thread > gpurun_out/rp_tests.log 2>&1 || { tail -40 gpurun_out/rp_tests.log; exit 1; }
tail -1 gpurun_out/rp_tests.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/rn_prof -o run -- python $R/bench_resnet.py --steps 5 --warmup 3 > $R/gpurun_out/rn_prof.log 2>&1 || { tail -20 $R/gpurun_out/rn_prof.log; exit 1; }
echo prof-ok
