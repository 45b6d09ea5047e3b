# call sites of the device copies in one eager ResNet-50 step
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/resnet_copies.py > gpurun_out/r4_resnet_copies.txt 2>&1; rc=$?; tail -30 gpurun_out/r4_resnet_copies.txt; exit $rc
