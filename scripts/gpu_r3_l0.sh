# Layer-0 recompute + one-launch BN v2 + head split: kernel tests, parity, A/B, profile, ResNet graph.
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_bn_gpu.py tests/test_gemm_gpu.py tests/test_layer0_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/l0_tests.log 2>&1 || { tail -40 gpurun_out/l0_tests.log; exit 1; }
tail -2 gpurun_out/l0_tests.log
timeout -k 10 400 python -u -m pytest tests/test_parity256_gpu.py -q --timeout 200 --timeout-method thread > gpurun_out/l0_parity.log 2>&1 || true
tail -5 gpurun_out/l0_parity.log
cp gpurun_out/parity256_errors.json gpurun_out/l0_parity256_errors.json || true
AB_ENVS="DPA_L0_RECOMPUTE=0 DPA_BN_FUSED_MAX=0 DPA_HEAD_SIDE=0|DPA_BN_FUSED_MAX=0 DPA_HEAD_SIDE=0|DPA_BN_FUSED_MAX=0|DPA_BN_FUSED_BWD_MAX=0|" REPS=3 bash scripts/gpu_ab.sh
TAG=l0 bash scripts/gpu_profile.sh
for gr in off on; do
  timeout -k 10 200 python bench_resnet.py --steps 20 --warmup 5 --graph $gr > gpurun_out/l0_resnet_$gr.log 2>&1 || { tail -20 gpurun_out/l0_resnet_$gr.log; exit 1; }
  echo "resnet graph=$gr $(tail -1 gpurun_out/l0_resnet_$gr.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["final_loss"])')"
done
