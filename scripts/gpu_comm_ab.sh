# 1-rank RCCL communicator slowdown hunt: wgrad priority x fused step x event scope.
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
run() {
  env "$@" DPA_FORCE_COMM=1 timeout -k 10 150 python bench.py --steps 50 --warmup 10 > gpurun_out/cab.log 2>&1
  echo "$* $(grep -o '"value": [0-9.]*' gpurun_out/cab.log)"
}
run DPA_WGRAD_PRIO=low DPA_FUSED_STEP=auto
run DPA_WGRAD_PRIO=normal DPA_FUSED_STEP=auto
run DPA_WGRAD_PRIO=normal DPA_FUSED_STEP=0
run DPA_WGRAD_PRIO=low DPA_FUSED_STEP=0
run DPA_WGRAD_PRIO=normal DPA_FUSED_STEP=auto DPA_EVENT_SCOPE=torch
run DPA_WGRAD_PRIO=normal DPA_FUSED_STEP=auto DPA_BN_BWD_BLOCK=1024
timeout -k 10 150 python bench.py --steps 50 --warmup 10 > gpurun_out/cab.log 2>&1
echo "null comm $(grep -o '"value": [0-9.]*' gpurun_out/cab.log)"
