# Round-2 (session 3) closing validation (after the fused head): GPU suite, smoke, benches,
# ResNet-50, and a kernel-trace profile of the default bench.
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/f5_gpu_tests.log 2>&1 || { tail -40 gpurun_out/f5_gpu_tests.log; exit 1; }
tail -1 gpurun_out/f5_gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/f5_smoke.log 2>&1 || { tail -20 gpurun_out/f5_smoke.log; exit 1; }
tail -1 gpurun_out/f5_smoke.log
b() { tag=$1; shift; timeout -k 10 150 "$@" > gpurun_out/f5_$tag.log 2>&1 || { tail -20 gpurun_out/f5_$tag.log; exit 1; }; echo "$tag $(tail -1 gpurun_out/f5_$tag.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"; }
b x3a python bench.py --steps 100 --warmup 20
b bf16 python bench.py --steps 100 --warmup 20 --impl bf16
b fp32 python bench.py --steps 100 --warmup 20 --impl fp32
b x3b python bench.py --steps 100 --warmup 20
DPA_FORCE_COMM=1 b rccl1 python bench.py --steps 100 --warmup 20
b resnet python bench_resnet.py --steps 20 --warmup 5
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/f5_prof -o run -- python $R/bench.py --steps 30 --warmup 5 > $R/gpurun_out/f5_prof.log 2>&1 || { tail -20 $R/gpurun_out/f5_prof.log; exit 1; }
echo prof-ok
