# Same-box A/B of the round-3 defaults (fused BN fwd <= 2.2M, bwd <= 0.6M, head weight gradient on
# the wgrad stream) against the round-2 configuration and two wider fused variants.
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
AB_ENVS="DPA_BN_FUSED_MAX=0 DPA_BN_FUSED_BWD_MAX=0 DPA_HEAD_SIDE=0|DPA_HEAD_SIDE=1|DPA_BN_FUSED_MAX=4300000|DPA_BN_FUSED_BWD_MAX=2200000" REPS=3 bash scripts/gpu_ab.sh
