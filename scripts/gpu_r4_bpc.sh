# weight-gradient convs capped at b blocks per CU (DPA_WGRAD_BPC): room for the critical path's BN waves
export TMPDIR=/tmp
mkdir -p gpurun_out
REPS=3 AB_ENVS="X=0|DPA_WGRAD_BPC=2|DPA_WGRAD_BPC=1" bash scripts/gpu_ab.sh || exit 1
DPA_WGRAD_BPC=2 TAG=r4bpc2 bash scripts/gpu_profile.sh || exit 1
