# A/B of the communicator-path options on a 1-rank RCCL communicator (collectives are no-ops, so
# this measures the overhead the comm path adds to the step), 2 interleaved rounds.
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
run() { env DPA_FORCE_COMM=1 "$@" timeout -k 10 120 python bench.py --steps 100 --warmup 20 $BARGS > gpurun_out/abc.log 2>&1 || { tail -20 gpurun_out/abc.log; exit 1; }; echo "$* $BARGS $(grep -o '"value": [0-9.]*' gpurun_out/abc.log) $(grep -o '"exposed_comm_ms": [0-9.]*' gpurun_out/abc.log)"; }
for r in 1 2; do
  run DPA_FUSED_STEP=auto
  run DPA_FUSED_STEP=0
  run DPA_BUF_BCAST=pre
  BARGS="--bucket-mb 40" run DPA_FUSED_STEP=auto
  BARGS="--bucket-mb 20" run DPA_FUSED_STEP=auto
  BARGS="--bucket-mb 20" run DPA_FUSED_STEP=0
done
timeout -k 10 120 python bench.py --steps 100 --warmup 20 > gpurun_out/abc.log 2>&1 && echo "null-comm $(grep -o '"value": [0-9.]*' gpurun_out/abc.log)"
