# A/B: BN backward finalize geometry (DPA_BN_FIN_CPB) and wgrad-stream CU masks, interleaved.
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
run() { env "$@" timeout -k 10 120 python bench.py --steps 100 --warmup 20 --diag-steps 0 > gpurun_out/ab.log 2>&1 || { tail -20 gpurun_out/ab.log; exit 1; }; echo "$* $(grep -o '"value": [0-9.]*' gpurun_out/ab.log)"; }
for r in 1 2; do
  run DPA_BN_FIN_CPB=4
  run DPA_BN_FIN_CPB=8
  run DPA_WGRAD_CUS=mod8:7
  run DPA_WGRAD_CUS=div8:7
  run DPA_WGRAD_CUS=mod4:3
done
