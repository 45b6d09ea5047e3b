export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 100 python tools/ipc_probe.py > gpurun_out/r4_ipc_probe.log 2>&1; echo ipc_rc=$?; tail -1 gpurun_out/r4_ipc_probe.log
timeout -k 10 400 python -u -m pytest tests/test_bnin_gpu.py tests/test_bn_gpu.py -x -q --timeout 120 --timeout-method thread -k "bn_on_load or residency or timeout_sets or fused_forward or geometry" > gpurun_out/r4_t1.log 2>&1; echo "tests rc=$?"; tail -5 gpurun_out/r4_t1.log
timeout -k 10 300 python -u -m pytest tests/test_multirank_gpu.py -x -q --timeout 120 --timeout-method thread -k "ipc_allreduce" > gpurun_out/r4_t2.log 2>&1; echo "ipc tests rc=$?"; tail -5 gpurun_out/r4_t2.log
DPA_FORCE_COMM=1 DPA_RCCL_CHANNELS=8 timeout -k 10 120 python bench.py --steps 20 --warmup 5 > gpurun_out/r4_rcclch.log 2>&1; echo "rcclch rc=$?"; tail -1 gpurun_out/r4_rcclch.log | cut -c1-200
AB_ENVS="DPA_BN_ON_LOAD=0|DPA_BN_ON_LOAD=1" REPS=3 STEPS=100 WARMUP=20 timeout -k 10 400 bash scripts/gpu_ab.sh
