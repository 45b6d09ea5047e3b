# Whole-step retune of every conv call (after schedule changes), then bench twice.
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 150 python bench.py --steps 100 --warmup 20 > gpurun_out/rt_bench0.log 2>&1 || { tail -20 gpurun_out/rt_bench0.log; exit 1; }
tail -1 gpurun_out/rt_bench0.log | cut -c1-200
timeout -k 10 900 python -u tools/tune_step.py --top 5 ${TUNE_ARGS:-} > gpurun_out/rt_tune.log 2>&1 || { tail -30 gpurun_out/rt_tune.log; exit 1; }
tail -2 gpurun_out/rt_tune.log
cp distributed_pytorch_amd/tuning/mi355x.json gpurun_out/rt_mi355x.json
for r in 1 2; do
timeout -k 10 150 python bench.py --steps 100 --warmup 20 > gpurun_out/rt_bench$r.log 2>&1 || { tail -20 gpurun_out/rt_bench$r.log; exit 1; }
tail -1 gpurun_out/rt_bench$r.log | cut -c1-200
done
