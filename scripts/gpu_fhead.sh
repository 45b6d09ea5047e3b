# Fused head (last BN + ReLU + pool inside the classifier kernel): engine tests, then A/B.
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py tests/test_parity256_gpu.py tests/test_kernels_gpu.py -k "fused_head or engine or step or parity or fc or head or trajectory" -x -q --timeout 200 --timeout-method thread > gpurun_out/fh_tests.log 2>&1 || { tail -40 gpurun_out/fh_tests.log; exit 1; }
tail -1 gpurun_out/fh_tests.log
run() { tag=$1; shift; (env "$@" timeout -k 10 200 python bench.py --steps 150 --warmup 20 > $R/gpurun_out/fh_$tag.log 2>&1) || { tail -20 $R/gpurun_out/fh_$tag.log; exit 1; }; echo "$tag $* $(tail -1 $R/gpurun_out/fh_$tag.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["final_loss"], d["param_checksum"])')"; }
for r in 1 2 3; do
  run on_$r DPA_FUSED_HEAD=1
  run off_$r DPA_FUSED_HEAD=0
done
