# Whole-tree validation on one MI355X: GPU suite, smoke(), bench (default + 1-rank RCCL),
# ResNet-50 bench, rocprofv3 kernel stats of the headline bench.  SKIP_TESTS=1: benches only.
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
if [ "${SKIP_TESTS:-0}" != 1 ]; then
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/val_gpu_tests.log 2>&1 || { tail -40 gpurun_out/val_gpu_tests.log; exit 1; }
tail -1 gpurun_out/val_gpu_tests.log
fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/val_smoke.log 2>&1 || { tail -20 gpurun_out/val_smoke.log; exit 1; }
tail -1 gpurun_out/val_smoke.log
timeout -k 10 150 python bench.py --steps 50 --warmup 10 > gpurun_out/val_bench.log 2>&1 || { tail -20 gpurun_out/val_bench.log; exit 1; }
tail -1 gpurun_out/val_bench.log
timeout -k 10 150 python bench.py --steps 20 --warmup 5 > gpurun_out/val_bench_driver.log 2>&1 || { tail -20 gpurun_out/val_bench_driver.log; exit 1; }
tail -1 gpurun_out/val_bench_driver.log
timeout -k 10 300 python bench.py --steps 50 --warmup 10 --torch-baseline 30 > gpurun_out/val_bench_torch.log 2>&1 || { tail -20 gpurun_out/val_bench_torch.log; exit 1; }
tail -1 gpurun_out/val_bench_torch.log
DPA_FORCE_COMM=1 timeout -k 10 150 python bench.py --steps 50 --warmup 10 > gpurun_out/val_bench_rccl1.log 2>&1 || { tail -20 gpurun_out/val_bench_rccl1.log; exit 1; }
tail -1 gpurun_out/val_bench_rccl1.log
timeout -k 10 200 python bench_resnet.py --steps 20 --warmup 5 > gpurun_out/val_resnet.log 2>&1 || { tail -20 gpurun_out/val_resnet.log; exit 1; }
tail -1 gpurun_out/val_resnet.log
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/val_prof -o val -- python $R/bench.py --steps 30 --warmup 5 > $R/gpurun_out/val_prof.log 2>&1 || { tail -20 $R/gpurun_out/val_prof.log; exit 1; }
tail -1 $R/gpurun_out/val_prof.log
