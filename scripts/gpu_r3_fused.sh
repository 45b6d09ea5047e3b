# One-launch BN: kernel tests vs torch fp64 autograd, engine parity test, then an interleaved A/B of
# the step (DPA_BN_FUSED_MAX=0 = three-kernel BN everywhere) and a kernel trace of the new default.
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_bn_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/f_bn_tests.log 2>&1 || { tail -40 gpurun_out/f_bn_tests.log; exit 1; }
tail -2 gpurun_out/f_bn_tests.log
timeout -k 10 300 python -u -m pytest tests/test_parity256_gpu.py tests/test_multirank_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/f_parity.log 2>&1 || { tail -40 gpurun_out/f_parity.log; exit 1; }
tail -2 gpurun_out/f_parity.log
b() { tag=$1; shift; timeout -k 10 150 "$@" > gpurun_out/f_$tag.log 2>&1 || { tail -20 gpurun_out/f_$tag.log; exit 1; }; echo "$tag $(tail -1 gpurun_out/f_$tag.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"; }
for r in 1 2 3; do
  DPA_BN_FUSED_MAX=0 b off$r python bench.py --steps 100 --warmup 20
  b on$r python bench.py --steps 100 --warmup 20
  DPA_BN_FUSED_MAX=4300000 b big$r python bench.py --steps 100 --warmup 20
done
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/f_prof -o run -- python $R/bench.py --steps 30 --warmup 5 > $R/gpurun_out/f_prof.log 2>&1 || { tail -20 $R/gpurun_out/f_prof.log; exit 1; }
echo prof-ok
