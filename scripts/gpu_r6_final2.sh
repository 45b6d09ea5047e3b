#!/bin/bash
# Round 6 final tree (per-chunk accumulation + layer-3 one-split forward): whole GPU suite, smoke, the
# driver-style bench twice, 1-rank RCCL, ResNet-50.
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=${OUT:-gpurun_out/val7}
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -q --maxfail 5 --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
tail -3 $O/gpu_tests.log; grep -E "^FAILED|^ERROR" $O/gpu_tests.log | head -10
[ $rc -le 1 ] || exit $rc
cp gpurun_out/parity256_errors.json gpurun_out/parity256_trained_errors.json $O/ 2>/dev/null
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for k in 1 2; do
timeout -k 10 150 python bench.py --steps 20 --warmup 5 > $O/bench_driver_$k.json 2> $O/bench_driver_$k.err || { tail -20 $O/bench_driver_$k.err; exit 1; }
tail -1 $O/bench_driver_$k.json | cut -c1-200
done
timeout -k 10 300 python bench.py --steps 50 --warmup 10 --torch-baseline 30 > $O/bench_torch.json 2> $O/bench_torch.err || { tail -20 $O/bench_torch.err; exit 1; }
tail -1 $O/bench_torch.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("50-step", d["value"], d["ms_per_step"], "torch", d.get("torch_eager_fp32_img_s"), d.get("vs_torch_eager_fp32"))'
DPA_FORCE_COMM=1 timeout -k 10 150 python bench.py --steps 50 --warmup 10 > $O/bench_rccl1.json 2> $O/bench_rccl1.err || { tail -20 $O/bench_rccl1.err; exit 1; }
tail -1 $O/bench_rccl1.json | cut -c1-200
timeout -k 10 200 python bench_resnet.py --steps 20 --warmup 5 > $O/resnet.json 2> $O/resnet.err || { tail -20 $O/resnet.err; exit 1; }
tail -1 $O/resnet.json | cut -c1-200
