# A/B on the single-GPU (null communicator) step, 3 interleaved rounds.
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
run() { env "$@" timeout -k 10 120 python bench.py --steps 100 --warmup 20 --diag-steps 0 > gpurun_out/abn.log 2>&1 || { tail -20 gpurun_out/abn.log; exit 1; }; echo "$* $(grep -o '"value": [0-9.]*' gpurun_out/abn.log)"; }
for r in 1 2 3; do
  run DPA_FUSED_STEP=auto
  run DPA_FUSED_STEP=1
  run DPA_WGRAD_STREAM=0
done
