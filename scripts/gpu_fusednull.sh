# Null comm: per-bucket SGD on the wgrad stream during backward (DPA_FUSED_STEP=1) vs one SGD at the end.
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
DPA_FUSED_STEP=1 timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -k "wgrad_stream or graphed or trajectory" -x -q --timeout 150 --timeout-method thread > gpurun_out/fn_tests.log 2>&1 || { tail -30 gpurun_out/fn_tests.log; exit 1; }
tail -1 gpurun_out/fn_tests.log
run() { tag=$1; shift; env "$@" timeout -k 10 150 python bench.py --steps 100 --warmup 20 > $R/gpurun_out/fn_$tag.log 2>&1 || { tail -20 $R/gpurun_out/fn_$tag.log; exit 1; }; echo "$tag $(tail -1 $R/gpurun_out/fn_$tag.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"; }
for r in 1 2 3; do
  run fused$r DPA_FUSED_STEP=1
  run end$r DPA_FUSED_STEP=auto
done
