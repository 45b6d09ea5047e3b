# Isolated conv-config sweep (tools/tune_convs.py) for selected calls, every candidate printed, the
# table written to gpurun_out/ (the tracked tuning table is replaced by hand after a step-level A/B).
#   ONLY="x3|fprop|256|2|,x3|dgrad|256|2|" bash scripts/gpu_tune.sh
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
DPA_TUNE_VERBOSE_ALL=1 timeout -k 10 ${TMO:-500} python -u tools/tune_convs.py --impls x3 --only "$ONLY" \
  --out gpurun_out/tune_${TAG:-small}.json > gpurun_out/tune_${TAG:-small}.log 2>&1
grep -v "^  cand" gpurun_out/tune_${TAG:-small}.log | tail -30
