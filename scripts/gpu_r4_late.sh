# weight gradient j waits for dgrad(j) to end (bsig[j-1]) instead of its start, per layer mask
export TMPDIR=/tmp
mkdir -p gpurun_out
REPS=3 AB_ENVS="X=0|DPA_WGRAD_LATE=0xFE|DPA_WGRAD_LATE=0x38|DPA_WGRAD_LATE=0x06" bash scripts/gpu_ab.sh || exit 1
DPA_WGRAD_LATE=0xFE TAG=r4late bash scripts/gpu_profile.sh || exit 1
