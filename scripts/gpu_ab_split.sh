# Overlapped-update tests, then interleaved A/B of DPA_SGD_SPLIT (0 = one SGD launch) with null comm
# and with a 1-rank RCCL communicator.
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -k "overlapped_update or wgrad_stream_matches or sync_modes_through_native" -x -q --timeout 150 --timeout-method thread > gpurun_out/abs_tests.log 2>&1 || { tail -40 gpurun_out/abs_tests.log; exit 1; }
tail -1 gpurun_out/abs_tests.log
run() { tag=$1; shift; (env "$@" timeout -k 10 200 python bench.py --steps 150 --warmup 20 > $R/gpurun_out/abs_$tag.log 2>&1) || { tail -20 $R/gpurun_out/abs_$tag.log; exit 1; }; echo "$tag $* $(tail -1 $R/gpurun_out/abs_$tag.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["final_loss"], d["param_checksum"])')"; }
for r in 1 2 3; do
  run n0_$r DPA_SGD_SPLIT=0
  run n3_$r DPA_SGD_SPLIT=3
  run n4_$r DPA_SGD_SPLIT=4
done
for r in 1 2; do
  run c0_$r DPA_FORCE_COMM=1 DPA_SGD_SPLIT=0
  run c3_$r DPA_FORCE_COMM=1 DPA_SGD_SPLIT=3
done
