# Kernel trace of the graph-replayed x3 step.
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/profg -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --graph on > $R/gpurun_out/profg.log 2>&1
tail -1 $R/gpurun_out/profg.log | cut -c1-200
echo prof-ok
