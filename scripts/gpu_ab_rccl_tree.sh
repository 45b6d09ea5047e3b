# 1-rank RCCL interleaved A/B of the in-tree build against ab_old/ (HEAD), after the rehearsal tests.
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_multirank_gpu.py tests/test_rccl_gpu.py tests/test_signal_gpu.py tests/test_ops_gpu.py -k "not wide_geometry" -x -q --timeout 150 --timeout-method thread > gpurun_out/abr_tests.log 2>&1 || { tail -40 gpurun_out/abr_tests.log; exit 1; }
tail -1 gpurun_out/abr_tests.log
run() { tag=$1; dir=$2; shift 2; (cd $dir && env DPA_FORCE_COMM=1 timeout -k 10 200 "$@" > $R/gpurun_out/abr_$tag.log 2>&1) || { tail -20 $R/gpurun_out/abr_$tag.log; exit 1; }; echo "$tag $(tail -1 $R/gpurun_out/abr_$tag.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["comm_diag"]["exposed_comm_ms"])')"; }
for r in 1 2 3; do
  run new$r $R python bench.py --steps 100 --warmup 20
  run old$r $R/ab_old python bench.py --steps 100 --warmup 20
done
