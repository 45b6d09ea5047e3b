export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r4_full_tests.log 2>&1; echo "gpu tests rc=$?"; tail -3 gpurun_out/r4_full_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4_smoke.log 2>&1; echo "smoke rc=$?"; tail -1 gpurun_out/r4_smoke.log
timeout -k 10 200 python bench_resnet.py --steps 20 --warmup 5 > gpurun_out/r4_resnet.log 2>&1; echo "resnet rc=$?"; tail -1 gpurun_out/r4_resnet.log | cut -c1-250
