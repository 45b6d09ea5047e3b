# Streaming-GEMM tile (conv_x3.hip gemm_stream_kernel): kernel tests, then a conv autotune of every
# table entry missing from a work copy of the tuning table (WORK: the 1x1 / stride-1 entries removed
# beforehand), copied to gpurun_out/, and a same-box A/B of the tracked table against the work copy.
set -e
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "stream or epilogue or dgrad_with_addend" > gpurun_out/st_tests.log 2>&1 || { tail -30 gpurun_out/st_tests.log; exit 1; }
tail -1 gpurun_out/st_tests.log
T=$(pwd)/distributed_pytorch_amd/tuning
WORK=${WORK:-$T/generic_work.json}
DPA_GENERIC_TABLE=$WORK timeout -k 10 600 python bench_resnet.py --autotune --steps 5 --warmup 2 > gpurun_out/st_autotune.log 2>&1 || { tail -20 gpurun_out/st_autotune.log; exit 1; }
cp $WORK gpurun_out/generic_work.json
AB_ENVS="DPA_GENERIC_TABLE=$T/generic_mi355x.json|DPA_GENERIC_TABLE=$WORK" REPS=3 BENCH=bench_resnet.py STEPS=100 WARMUP=10 bash scripts/gpu_ab.sh
