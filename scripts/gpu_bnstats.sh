# Conv-epilogue BN partials: kernel/engine/layer tests, VGG A/B (DPA_CONV_BN_STATS), ResNet bench.
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_ops_gpu.py tests/test_layers_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "epilogue or halo or engine or sync_modes or resnet or bn or graphed" > gpurun_out/bnstats_tests.log 2>&1 || { tail -40 gpurun_out/bnstats_tests.log; exit 1; }
tail -1 gpurun_out/bnstats_tests.log
for i in 1 2; do
  for v in 1 0; do
    DPA_CONV_BN_STATS=$v timeout -k 10 150 python bench.py --steps 50 --warmup 10 > gpurun_out/ab_bns_$v.log 2>&1
    echo "x3 bnstats=$v $(grep -o '"value": [0-9.]*' gpurun_out/ab_bns_$v.log)"
  done
done
for v in 1 0; do
  DPA_CONV_BN_STATS=$v timeout -k 10 200 python bench_resnet.py --batch 128 > gpurun_out/rn_bns_$v.log 2>&1
  echo "resnet bnstats=$v $(grep -o '"value": [0-9.]*' gpurun_out/rn_bns_$v.log)"
done
