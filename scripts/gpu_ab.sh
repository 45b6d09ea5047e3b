# Interleaved same-box A/B of environment settings on the headline bench (docs/PERF_NOTES.md: every
# lever below ~5 % is judged this way; pool boxes differ by several percent for the same commit).
#
#   AB_ENVS="DPA_BN_FUSED_MAX=0|DPA_BN_FUSED_MAX=2200000" bash scripts/gpu_ab.sh
#
# AB_ENVS   '|'-separated variants, each a space-separated list of VAR=value (empty = defaults)
# REPS      interleaved rounds (default 3)        STEPS / WARMUP  per run (default 100 / 20)
# BENCH     bench.py (default) or bench_resnet.py  ARGS  extra bench arguments (e.g. "--impl bf16")
# FORCE_COMM=1  route the step through a 1-rank RCCL communicator (the multi-GPU code path)
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
IFS='|' read -ra ENVS <<< "${AB_ENVS:-}"
[ ${#ENVS[@]} -gt 0 ] || ENVS=("")
BENCH=${BENCH:-bench.py}
run() {
  tag=$1; shift
  (env DPA_FORCE_COMM=${FORCE_COMM:-0} $@ timeout -k 10 200 python $BENCH --steps ${STEPS:-100} --warmup ${WARMUP:-20} ${ARGS:-} \
     > gpurun_out/ab_$tag.log 2>&1) || { tail -20 gpurun_out/ab_$tag.log; exit 1; }
  echo "$tag [$*] $(tail -1 gpurun_out/ab_$tag.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
}
for r in $(seq ${REPS:-3}); do
  i=0
  for e in "${ENVS[@]}"; do
    i=$((i+1))
    run r${r}_v$i $e
  done
done
