export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_bnin_gpu.py tests/test_bn_gpu.py -x -q --timeout 120 --timeout-method thread -k "bn_on_load or bn_bwd_on_load or residency or timeout_sets or fused_forward or geometry" > gpurun_out/r4_t3.log 2>&1; echo "tests rc=$?"; tail -5 gpurun_out/r4_t3.log
AB_ENVS="DPA_BN_ON_LOAD=0|DPA_BN_ON_LOAD=1|DPA_BN_ON_LOAD=1 DPA_BN_BWD_ON_LOAD=1|DPA_BN_BWD_ON_LOAD=1" REPS=2 STEPS=100 WARMUP=20 timeout -k 10 400 bash scripts/gpu_ab.sh
VARIANTS="1" DPA_BN_BWD_ON_LOAD=1 timeout -k 10 250 bash scripts/gpu_r4_prof.sh
