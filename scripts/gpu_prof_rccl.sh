# Kernel trace of the x3 step through a 1-rank RCCL communicator (the multi-GPU code path).
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
for f in auto 0; do
  DPA_FUSED_STEP=$f DPA_FORCE_COMM=1 timeout -k 10 150 python bench.py --steps 50 --warmup 10 > gpurun_out/rc.log 2>&1
  echo "rccl1 fused=$f $(grep -o '"value": [0-9.]*' gpurun_out/rc.log)"
done
cd /tmp
DPA_FORCE_COMM=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/profc -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 > $R/gpurun_out/profc.log 2>&1
echo prof-ok
