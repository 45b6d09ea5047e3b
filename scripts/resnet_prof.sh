set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
timeout -k 10 600 python -m pytest tests/test_layers_gpu.py -x -q > gpurun_out/layers.log 2>&1 || { tail -30 gpurun_out/layers.log; exit 1; }
tail -1 gpurun_out/layers.log
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_rn -o run --output-format csv -- python3 $R/bench_resnet.py --batch 128 --steps 5 --warmup 2 > $R/gpurun_out/prof_rn.log 2>&1
echo prof-ok
cd $R
timeout -k 10 600 python tools/torch_baseline.py --model resnet50 --batch 128 --modes bf16_cl --steps 10 --warmup 5 2>&1 | grep img_per_s
