# Two ranks on one GPU through gloo staging: every sync mode of the GPU engine path.
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_multirank_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/mr_tests.log 2>&1 || { tail -60 gpurun_out/mr_tests.log; exit 1; }
tail -6 gpurun_out/mr_tests.log
