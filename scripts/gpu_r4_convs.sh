# per-shape ResNet-50 conv timings (ours / MIOpen / hipBLASLt), weight gradient separately
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u tools/resnet_conv_bench.py --iters 10 > gpurun_out/r4_rn_convs.jsonl 2> gpurun_out/r4_rn_convs.err; echo "rc=$?"; tail -2 gpurun_out/r4_rn_convs.jsonl
