# Kernel trace of the headline step (timeline source for tools/trace_step.py) and, with PMC=1,
# the per-kernel counter passes on one stream (DPA_WGRAD_STREAM=0, counters not mixed by the
# weight-gradient stream; each pass within the per-block counter limits, its own run).
#   TAG=r3 PMC=1 bash scripts/gpu_profile.sh
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-prof}
mkdir -p $R/gpurun_out
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${TAG}_trace -o run -- python3 $R/bench.py --steps 30 --warmup 5 ${ARGS:-} > $R/gpurun_out/${TAG}_trace.log 2>&1 || { tail -20 $R/gpurun_out/${TAG}_trace.log; exit 1; }
echo trace-ok
if [ "${PMC:-0}" = 1 ]; then
  export DPA_WGRAD_STREAM=0
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT --kernel-trace --output-format csv -d $R/gpurun_out/${TAG}_pmcA -o run -- python3 $R/bench.py --steps 3 --warmup 2 ${ARGS:-} > $R/gpurun_out/${TAG}_pmcA.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVES --kernel-trace --output-format csv -d $R/gpurun_out/${TAG}_pmcB -o run -- python3 $R/bench.py --steps 3 --warmup 2 ${ARGS:-} > $R/gpurun_out/${TAG}_pmcB.log 2>&1
  echo pmc-ok
fi
