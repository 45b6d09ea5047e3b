# Interleaved 1-rank RCCL A/B: per-bucket fused SGD inside backward (DPA_FUSED_STEP=1) against one
# SGD after backward (DPA_FUSED_STEP=0), DDP and per-tensor all-reduce modes.
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
run() { tag=$1; shift; (env DPA_FORCE_COMM=1 "$@" timeout -k 10 200 python bench.py --steps 150 --warmup 20 $BARGS > $R/gpurun_out/abf_$tag.log 2>&1) || { tail -20 $R/gpurun_out/abf_$tag.log; exit 1; }; echo "$tag $* $BARGS $(tail -1 $R/gpurun_out/abf_$tag.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], (d["comm_diag"] or {}).get("exposed_comm_ms"))')"; }
for r in 1 2 3 4; do
  BARGS="" run ddp_f1_$r DPA_FUSED_STEP=1
  BARGS="" run ddp_f0_$r DPA_FUSED_STEP=0
done
for r in 1 2; do
  BARGS="--mode allreduce" run ar_f1_$r DPA_FUSED_STEP=1
  BARGS="--mode allreduce" run ar_f0_$r DPA_FUSED_STEP=0
done
