#!/bin/bash
# Conv numerics, then an interleaved same-box bench A/B of two builds: v1 = ab_base/_C.so (the
# baseline build, run from a copy of the tree), v2 = the tree's own _C.so.
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out/kab
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "${KSEL:-x3 or halo or fp16 or split}" > gpurun_out/kab/kern.log 2>&1 || { tail -30 gpurun_out/kab/kern.log; exit 1; }
if [ "${PARITY:-1}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_parity256_gpu.py > gpurun_out/kab/par.log 2>&1 || { tail -30 gpurun_out/kab/par.log; exit 1; }
fi
B=/tmp/ab_base_tree
rm -rf $B && mkdir -p $B && cp -r bench.py distributed_pytorch_amd $B/ && cp ab_base/_C.so $B/distributed_pytorch_amd/_C.so
for r in $(seq ${REPS:-3}); do
  (cd $B && timeout -k 10 240 python bench.py --steps ${STEPS:-50} --warmup ${WARMUP:-10} ${ARGS:-}) > gpurun_out/kab/v1_$r.json 2> gpurun_out/kab/v1_$r.err || exit 1
  timeout -k 10 240 python bench.py --steps ${STEPS:-50} --warmup ${WARMUP:-10} ${ARGS:-} > gpurun_out/kab/v2_$r.json 2> gpurun_out/kab/v2_$r.err || exit 1
  for v in v1 v2; do echo "$r $v $(tail -1 gpurun_out/kab/${v}_$r.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"; done
done
