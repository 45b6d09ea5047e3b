# Interleaved 1-rank RCCL A/B of environment switches on one box (same tree).
#   AB_ENVS="DPA_WATCHDOG=1|DPA_WATCHDOG=0" bash scripts/gpu_ab_env.sh
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
IFS='|' read -ra ENVS <<< "${AB_ENVS:-DPA_WATCHDOG=1|DPA_WATCHDOG=0}"
run() { tag=$1; shift; (env DPA_FORCE_COMM=${FORCE_COMM:-1} "$@" timeout -k 10 200 python bench.py --steps 100 --warmup 20 > $R/gpurun_out/abe_$tag.log 2>&1) || { tail -20 $R/gpurun_out/abe_$tag.log; exit 1; }; echo "$tag $* $(tail -1 $R/gpurun_out/abe_$tag.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], (d["comm_diag"] or {}).get("exposed_comm_ms"))')"; }
for r in 1 2 3; do
  i=0
  for e in "${ENVS[@]}"; do
    i=$((i+1))
    run r${r}_$i $e
  done
done
