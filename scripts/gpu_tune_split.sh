# Step-level re-tune of the conv configs with one candidate per split-K count (tools/tune_step.py
# --per-split); the table is written under gpurun_out/ (copied back into tuning/ by hand).
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/tune
cp $R/distributed_pytorch_amd/tuning/mi355x.json $R/gpurun_out/tune/mi355x.json
timeout -k 10 700 python -u $R/tools/tune_step.py --per-split --kinds ${KINDS:-wgrad,dgrad,fprop} --out $R/gpurun_out/tune/mi355x.json > $R/gpurun_out/tune/tune_split.log 2>&1
tail -3 $R/gpurun_out/tune/tune_split.log
