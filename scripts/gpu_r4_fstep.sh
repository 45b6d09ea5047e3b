# per-bucket SGD inside backward on the wgrad stream, one rank, null communicator
export TMPDIR=/tmp
mkdir -p gpurun_out
REPS=3 AB_ENVS="DPA_FUSED_STEP=0|DPA_FUSED_STEP=1" bash scripts/gpu_ab.sh || exit 1
