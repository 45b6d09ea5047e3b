export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_multirank_gpu.py tests/test_rccl_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4_t5.log 2>&1; echo "multirank+rccl rc=$?"; tail -3 gpurun_out/r4_t5.log
AB_ENVS="DPA_FORCE_COMM=0|DPA_FORCE_COMM=1 DPA_TAIL_HERE=0|DPA_FORCE_COMM=1 DPA_TAIL_HERE=1" REPS=3 STEPS=100 WARMUP=20 timeout -k 10 500 bash scripts/gpu_ab.sh
