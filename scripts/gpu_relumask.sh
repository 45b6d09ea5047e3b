# ResNet add+ReLU backward from the forward ReLU mask: layer tests, then interleaved A/B of DPA_BN_RELU_MASK.
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_layers_gpu.py tests/test_multirank_gpu.py -k "resnet or bn_act or bf16_activation or head" -x -q --timeout 200 --timeout-method thread > gpurun_out/rm_tests.log 2>&1 || { tail -40 gpurun_out/rm_tests.log; exit 1; }
tail -1 gpurun_out/rm_tests.log
run() { tag=$1; shift; (env "$@" timeout -k 10 200 python bench_resnet.py --steps 20 --warmup 5 > $R/gpurun_out/rm_$tag.log 2>&1) || { tail -20 $R/gpurun_out/rm_$tag.log; exit 1; }; echo "$tag $* $(tail -1 $R/gpurun_out/rm_$tag.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["final_loss"])')"; }
for r in 1 2 3; do
  run on_$r DPA_BN_RELU_MASK=1
  run off_$r DPA_BN_RELU_MASK=0
done
