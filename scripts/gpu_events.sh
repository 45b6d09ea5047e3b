# Event-scope A/B: micro-benchmark of event records, then the x3 bench with torch (system-scope)
# vs device-scope events, fused per-bucket update on/off, null and forced 1-rank RCCL comm.
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 120 python tools/event_overhead.py > gpurun_out/event_overhead.log 2>&1
cat gpurun_out/event_overhead.log | tail -1
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "sync_modes or sgd" > gpurun_out/ev_tests.log 2>&1 || { tail -30 gpurun_out/ev_tests.log; exit 1; }
tail -1 gpurun_out/ev_tests.log
for cfg in "torch 0 0" "device 0 0" "nofence 0 0" "device 1 0" "torch 1 1" "device 1 1" "device 0 1"; do
  set -- $cfg
  DPA_EVENT_SCOPE=$1 DPA_FUSED_STEP=$2 DPA_FORCE_COMM=$3 timeout -k 10 150 python bench.py --steps 50 --warmup 10 > gpurun_out/bench_ev_$1_$2_$3.log 2>&1
  echo "scope=$1 fused=$2 forcecomm=$3 $(grep -o '"value": [0-9.]*' gpurun_out/bench_ev_$1_$2_$3.log)"
done
cd /tmp
DPA_FUSED_STEP=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 > $R/gpurun_out/prof.log 2>&1
echo prof-ok
