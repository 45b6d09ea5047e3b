# VGG-11 x3: fresh isolated autotune of every conv call (new halo tiles among the candidates) into
# gpurun_out, then an in-step A/B of the committed table against the fresh entries
export TMPDIR=/tmp
mkdir -p gpurun_out
R=${GRAFT_REPO_ROOT:-$(pwd)}
rm -f gpurun_out/vgg_x3_fresh.json
timeout -k 10 900 python -u tools/tune_convs.py --impls x3 --out $R/gpurun_out/vgg_x3_fresh.json > gpurun_out/r4_vggtune.log 2>&1; echo "tune rc=$?"; tail -2 gpurun_out/r4_vggtune.log
REPS=3 AB_ENVS="X=0|DPA_TUNING_EXTRA=$R/gpurun_out/vgg_x3_fresh.json" bash scripts/gpu_ab.sh || exit 1
