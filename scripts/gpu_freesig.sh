# params_free via kernel-start signals: RCCL / sync tests and an interleaved 1-rank RCCL A/B.
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_rccl_gpu.py tests/test_ops_gpu.py tests/test_signal_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/fs_tests.log 2>&1 || { tail -40 gpurun_out/fs_tests.log; exit 1; }
tail -1 gpurun_out/fs_tests.log
run() { tag=$1; shift; env "$@" timeout -k 10 120 python bench.py --steps 100 --warmup 20 > $R/gpurun_out/fs_$tag.log 2>&1 || { tail -20 $R/gpurun_out/fs_$tag.log; exit 1; }; echo "$tag $(tail -1 $R/gpurun_out/fs_$tag.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["comm_diag"]["exposed_comm_ms"])')"; }
for r in 1 2; do
  run on$r DPA_FORCE_COMM=1
  run off$r DPA_FORCE_COMM=1 DPA_FREE_SIGNAL=0
  run unf$r DPA_FORCE_COMM=1 DPA_FUSED_STEP=0
done
run null
