# Iteration check: selected GPU tests ($TESTS), then the headline bench twice and a kernel-trace profile.
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest ${TESTS:-tests/test_fused_gpu.py tests/test_parity256_gpu.py} -x -q --timeout 200 --timeout-method thread > gpurun_out/iter_tests.log 2>&1 || { tail -40 gpurun_out/iter_tests.log; exit 1; }
tail -1 gpurun_out/iter_tests.log
for r in 1 2; do
  timeout -k 10 120 python bench.py --steps 100 --warmup 20 > gpurun_out/iter_bench.log 2>&1 || { tail -20 gpurun_out/iter_bench.log; exit 1; }
  echo "bench $(grep -o '"value": [0-9.]*' gpurun_out/iter_bench.log)"
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_iter -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --diag-steps 0 > $R/gpurun_out/prof_iter.log 2>&1
echo prof-ok
