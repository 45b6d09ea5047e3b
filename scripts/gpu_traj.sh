set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -k "trajectory" -x -v --timeout 250 --timeout-method thread > gpurun_out/traj.log 2>&1 || { tail -30 gpurun_out/traj.log; exit 1; }
tail -3 gpurun_out/traj.log
