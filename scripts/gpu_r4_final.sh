# round-4 validation: full GPU suite, smoke, driver-style VGG bench, ResNet bench, VGG kernel stats
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4v_tests.log 2>&1; rc=$?; echo "gpu tests rc=$rc"; tail -3 gpurun_out/r4v_tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4v_smoke.log 2>&1; echo "smoke rc=$?"; tail -1 gpurun_out/r4v_smoke.log
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r4v_bench.json 2> gpurun_out/r4v_bench.err; echo "bench rc=$?"; tail -1 gpurun_out/r4v_bench.json | cut -c1-200
timeout -k 10 200 python bench_resnet.py --steps 20 --warmup 5 > gpurun_out/r4v_resnet.json 2> gpurun_out/r4v_resnet.err; echo "resnet rc=$?"; tail -1 gpurun_out/r4v_resnet.json | cut -c1-200
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r4v_prof -o vgg -- python bench.py --steps 20 --warmup 5 > gpurun_out/r4v_prof.log 2>&1; echo "prof rc=$?"
