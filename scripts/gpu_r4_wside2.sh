# side-stream wgrad A/B with the eager step (no HIP graph)
export TMPDIR=/tmp
mkdir -p gpurun_out
BENCH=bench_resnet.py STEPS=40 WARMUP=10 REPS=2 ARGS="--graph off" AB_ENVS="DPA_WGRAD_STREAM=0|DPA_WGRAD_STREAM=1" bash scripts/gpu_ab.sh || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r4p_rn_ws_eager -o rn -- python bench_resnet.py --steps 10 --warmup 5 --graph off > gpurun_out/r4p_rn_ws_eager.log 2>&1; echo "prof rc=$?"
