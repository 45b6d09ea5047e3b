# Round-3 start: x3 bench twice + a kernel-trace profile of the default bench (timeline source).
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
b() { tag=$1; shift; timeout -k 10 150 "$@" > gpurun_out/s_$tag.log 2>&1 || { tail -20 gpurun_out/s_$tag.log; exit 1; }; echo "$tag $(tail -1 gpurun_out/s_$tag.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"; }
b x3a python bench.py --steps 100 --warmup 20
b x3b python bench.py --steps 100 --warmup 20
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/s_prof -o run -- python $R/bench.py --steps 30 --warmup 5 > $R/gpurun_out/s_prof.log 2>&1 || { tail -20 $R/gpurun_out/s_prof.log; exit 1; }
echo prof-ok
