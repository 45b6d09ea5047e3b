# ResNet-50 per-kernel counters (eager step, one pass per counter group within the per-block limits).
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd /tmp
B="python3 $R/bench_resnet.py --steps 2 --warmup 1 --graph off"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT --kernel-trace --output-format csv -d $R/gpurun_out/rnp_A -o run -- $B > $R/gpurun_out/rnp_A.log 2>&1
echo A-ok
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVES --kernel-trace --output-format csv -d $R/gpurun_out/rnp_B -o run -- $B > $R/gpurun_out/rnp_B.log 2>&1
echo B-ok
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/rnp_C -o run -- $B > $R/gpurun_out/rnp_C.log 2>&1
echo C-ok
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/rnp_D -o run -- $B > $R/gpurun_out/rnp_D.log 2>&1
echo D-ok
