# Quick health check on one MI355X: smoke(), headline bench, kernel-trace profile of the bench.
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 150 python bench.py --steps 50 --warmup 10 > gpurun_out/bench_x3.log 2>&1 || { tail -20 gpurun_out/bench_x3.log; exit 1; }
tail -1 gpurun_out/bench_x3.log
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 > $R/gpurun_out/prof.log 2>&1
echo prof-ok
