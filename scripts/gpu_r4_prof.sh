# kernel traces of the headline step with and without the consumer-side BN (DPA_BN_ON_LOAD)
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd /tmp
for v in ${VARIANTS:-0 1}; do
  DPA_BN_ON_LOAD=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r4p_bnin$v -o run -- python3 $R/bench.py --steps 30 --warmup 5 > $R/gpurun_out/r4p_bnin$v.log 2>&1 || { tail -20 $R/gpurun_out/r4p_bnin$v.log; exit 1; }
  echo "trace $v ok"
done
