# SGD kernel with two elements in flight per thread: SGD tests, then A/B.
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py tests/test_parity256_gpu.py tests/test_kernels_gpu.py -k "sgd or fused_step or trajectory or parity or overlapped or wgrad_stream" -x -q --timeout 200 --timeout-method thread > gpurun_out/su_tests.log 2>&1 || { tail -40 gpurun_out/su_tests.log; exit 1; }
tail -1 gpurun_out/su_tests.log
run() { tag=$1; shift; (env "$@" timeout -k 10 200 python bench.py --steps 150 --warmup 20 > $R/gpurun_out/su_$tag.log 2>&1) || { tail -20 $R/gpurun_out/su_$tag.log; exit 1; }; echo "$tag $* $(tail -1 $R/gpurun_out/su_$tag.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["final_loss"], d["param_checksum"])')"; }
for r in 1 2 3; do
  run on_$r DPA_SGD_UNROLL=2
  run off_$r DPA_SGD_UNROLL=1
done
