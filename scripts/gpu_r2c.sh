# Full GPU suite + ResNet-50 bench + its kernel-trace profile (through bench_resnet.py --profile).
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r2c_gpu_tests.log 2>&1 || { tail -40 gpurun_out/r2c_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r2c_gpu_tests.log
timeout -k 10 200 python bench_resnet.py --batch 128 > gpurun_out/r2c_resnet.log 2>&1 || { tail -20 gpurun_out/r2c_resnet.log; exit 1; }
tail -1 gpurun_out/r2c_resnet.log
timeout -k 10 300 python bench_resnet.py --batch 128 --steps 5 --warmup 3 --profile --profile-dir $R/gpurun_out/prof_rn > gpurun_out/r2c_resnet_prof.log 2>&1 || { tail -20 gpurun_out/r2c_resnet_prof.log; exit 1; }
echo prof-ok
