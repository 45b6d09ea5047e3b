# ResNet-50: re-run the generic autotuner from an EMPTY table (every candidate, new halo tiles 22/23
# included), then A/B the committed and fresh tables
export TMPDIR=/tmp
mkdir -p gpurun_out
R=${GRAFT_REPO_ROOT:-$(pwd)}
echo '{}' > gpurun_out/generic_r4_fresh.json
DPA_GENERIC_TABLE=$R/gpurun_out/generic_r4_fresh.json timeout -k 10 900 python -u bench_resnet.py --autotune --steps 5 --warmup 2 > gpurun_out/r4_rntune.log 2>&1; echo "autotune rc=$?"; tail -1 gpurun_out/r4_rntune.log | cut -c1-150
BENCH=bench_resnet.py STEPS=40 WARMUP=10 REPS=3 AB_ENVS="X=0|DPA_GENERIC_TABLE=$R/gpurun_out/generic_r4_fresh.json" bash scripts/gpu_ab.sh || exit 1
