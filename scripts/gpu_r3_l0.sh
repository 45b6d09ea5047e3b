# Layer-0 recompute + one-launch BN (batched merge, fewer row blocks): kernel tests, parity, A/B.
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_bn_gpu.py tests/test_layer0_gpu.py tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/l0_tests.log 2>&1 || { tail -40 gpurun_out/l0_tests.log; exit 1; }
tail -2 gpurun_out/l0_tests.log
timeout -k 10 300 python -u -m pytest tests/test_parity256_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/l0_parity.log 2>&1 || { tail -40 gpurun_out/l0_parity.log; exit 1; }
tail -2 gpurun_out/l0_parity.log
cp gpurun_out/parity256_errors.json gpurun_out/l0_parity256_errors.json
AB_ENVS="DPA_L0_RECOMPUTE=0 DPA_BN_FUSED_MAX=0|DPA_BN_FUSED_MAX=0|DPA_BN_FUSED_BWD_MAX=0|DPA_BN_FUSED_MAX=2200000" REPS=3 bash scripts/gpu_ab.sh
TAG=l0 bash scripts/gpu_profile.sh
for gr in off on; do
  timeout -k 10 200 python bench_resnet.py --steps 20 --warmup 5 --graph $gr > gpurun_out/l0_resnet_$gr.log 2>&1 || { tail -20 gpurun_out/l0_resnet_$gr.log; exit 1; }
  echo "resnet graph=$gr $(tail -1 gpurun_out/l0_resnet_$gr.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["final_loss"])')"
done
