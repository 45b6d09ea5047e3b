# ResNet path: generic layer tests, ResNet-50 bench and its kernel-trace profile.
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_layers_gpu.py tests/test_kernels_gpu.py -k "not conv_x3_fprop and not conv_x3_wgrad and not conv_fprop and not conv_wgrad" -x -q --timeout 200 --timeout-method thread > gpurun_out/rn_tests.log 2>&1 || { tail -40 gpurun_out/rn_tests.log; exit 1; }
tail -1 gpurun_out/rn_tests.log
timeout -k 10 200 python bench_resnet.py --batch 128 > gpurun_out/rn_bench.log 2>&1 || { tail -20 gpurun_out/rn_bench.log; exit 1; }
tail -1 gpurun_out/rn_bench.log
timeout -k 10 300 python bench_resnet.py --batch 128 --steps 5 --warmup 3 --profile --profile-dir $R/gpurun_out/prof_rn > gpurun_out/rn_prof.log 2>&1 || { tail -20 gpurun_out/rn_prof.log; exit 1; }
echo prof-ok
