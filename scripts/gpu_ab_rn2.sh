# BN backward geometry by size: ResNet-50 and VGG-11 benches, BN/layer GPU tests.
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
run() { tag=$1; shift; timeout -k 10 200 "$@" > $R/gpurun_out/abrn_$tag.log 2>&1 || { tail -20 $R/gpurun_out/abrn_$tag.log; exit 1; }; echo "$tag $(tail -1 $R/gpurun_out/abrn_$tag.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"; }
timeout -k 10 300 python -u -m pytest tests/test_layers_gpu.py tests/test_kernels_gpu.py -k "bn or resnet or BatchNorm or layer" -x -q --timeout 200 --timeout-method thread > gpurun_out/abrn_tests.log 2>&1 || { tail -40 gpurun_out/abrn_tests.log; exit 1; }
tail -1 gpurun_out/abrn_tests.log
run auto python bench_resnet.py --batch 128 --steps 20 --warmup 5
DPA_BN_BWD_BLOCK=256 run small python bench_resnet.py --batch 128 --steps 20 --warmup 5
run vgg python bench.py --steps 50 --warmup 10
run auto2 python bench_resnet.py --batch 128 --steps 20 --warmup 5
run vgg2 python bench.py --steps 50 --warmup 10
