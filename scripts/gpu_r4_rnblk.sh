# ResNet-50: block count of the 1024-thread BN backward reduce
export TMPDIR=/tmp
mkdir -p gpurun_out
BENCH=bench_resnet.py STEPS=40 WARMUP=10 REPS=3 AB_ENVS="DPA_BN_BWD_WIDE_BLOCKS=256|DPA_BN_BWD_WIDE_BLOCKS=128|DPA_BN_BWD_WIDE_BLOCKS=192" bash scripts/gpu_ab.sh || exit 1
