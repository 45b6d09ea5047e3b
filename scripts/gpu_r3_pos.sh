# Position-major small-image conv kernel: unit tests, the isolated sweep of the small layers, then
# a same-box step A/B of the swept table against the tracked one.
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "pos" \
  > gpurun_out/pos_tests.log 2>&1 || { tail -40 gpurun_out/pos_tests.log; exit 1; }
tail -3 gpurun_out/pos_tests.log
ONLY="x3|fprop|256|2|,x3|dgrad|256|2|,x3|fprop|256|4|,x3|dgrad|256|4|" TAG=pos bash scripts/gpu_tune.sh
AB_ENVS="DPA_HEAD_SIDE=1|DPA_TUNING_EXTRA=gpurun_out/tune_pos.json" REPS=3 bash scripts/gpu_ab.sh
