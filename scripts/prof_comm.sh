set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
export DPA_FORCE_COMM=1
for args in "--no-overlap" "--bucket-mb 40" "--mode allreduce" "--comm torch"; do
  echo "== $args"; timeout -k 10 200 python bench.py --steps 30 --warmup 10 $args 2>&1 | grep metric | cut -c100-200
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_fc -o run -- python3 $R/bench.py --steps 20 --warmup 5 > $R/gpurun_out/prof_fc.log 2>&1
echo prof-ok
