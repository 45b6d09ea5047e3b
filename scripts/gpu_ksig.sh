# Kernel-start signals vs per-layer events in the two-stream backward: tests, interleaved A/B, profile.
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_signal_gpu.py tests/test_ops_gpu.py tests/test_parity256_gpu.py -k "signal or wait or wgrad_stream or graphed or parity or conv_call or loss or gradients or updates or layer0" -x -v --timeout 120 --timeout-method thread > gpurun_out/ksig_tests.log 2>&1 || { tail -40 gpurun_out/ksig_tests.log; exit 1; }
tail -1 gpurun_out/ksig_tests.log
run() { tag=$1; shift; env "$@" timeout -k 10 120 python bench.py --steps 100 --warmup 20 > $R/gpurun_out/ksig_$tag.log 2>&1 || { tail -20 $R/gpurun_out/ksig_$tag.log; exit 1; }; echo "$tag $(tail -1 $R/gpurun_out/ksig_$tag.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"; }
for r in 1 2; do
  run on$r DPA_KSIGNAL=1
  run off$r DPA_KSIGNAL=0
done
run rccl_on DPA_KSIGNAL=1 DPA_FORCE_COMM=1
run rccl_off DPA_KSIGNAL=0 DPA_FORCE_COMM=1
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/ksig_prof -o run -- python $R/bench.py --steps 20 --warmup 5 > $R/gpurun_out/ksig_prof.log 2>&1 || { tail -20 $R/gpurun_out/ksig_prof.log; exit 1; }
echo prof-ok
