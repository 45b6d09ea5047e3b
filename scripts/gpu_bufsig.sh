# Signal-ordered BN-buffer broadcast (DDP): multi-rank rehearsal + RCCL tests, 1-rank RCCL A/B.
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_multirank_gpu.py tests/test_rccl_gpu.py tests/test_ops_gpu.py -k "not wide_geometry" -x -q --timeout 150 --timeout-method thread > gpurun_out/bs_tests.log 2>&1 || { tail -40 gpurun_out/bs_tests.log; exit 1; }
tail -1 gpurun_out/bs_tests.log
run() { tag=$1; shift; env "$@" timeout -k 10 150 python bench.py --steps 100 --warmup 20 > $R/gpurun_out/bs_$tag.log 2>&1 || { tail -20 $R/gpurun_out/bs_$tag.log; exit 1; }; echo "$tag $(tail -1 $R/gpurun_out/bs_$tag.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"; }
for r in 1 2 3; do
  run sig$r DPA_FORCE_COMM=1 DPA_BUF_SIGNAL=1
  run ev$r DPA_FORCE_COMM=1 DPA_BUF_SIGNAL=0
done
