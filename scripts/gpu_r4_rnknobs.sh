# ResNet-50 knob sweep: BN finalize channels per block, BN apply unroll
export TMPDIR=/tmp
mkdir -p gpurun_out
BENCH=bench_resnet.py STEPS=40 WARMUP=10 REPS=3 AB_ENVS="X=0|DPA_BN_FIN_CPB=4|DPA_BN_UNROLL=0" bash scripts/gpu_ab.sh || exit 1
