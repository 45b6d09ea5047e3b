# PMC pass (one stream) of the headline step with and without BN applied on load
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd /tmp
export DPA_WGRAD_STREAM=0
for v in 0 1; do
  DPA_BN_ON_LOAD=$v DPA_BN_BWD_ON_LOAD=$v timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_IFETCH SQ_INSTS_VALU --kernel-trace --output-format csv -d $R/gpurun_out/r4pmc_$v -o run -- python3 $R/bench.py --steps 3 --warmup 2 > $R/gpurun_out/r4pmc_$v.log 2>&1 || { echo "pmc $v failed"; tail -5 $R/gpurun_out/r4pmc_$v.log; exit 1; }
  echo "pmc $v ok"
done
