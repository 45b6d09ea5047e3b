# The driver's short bench (--steps 20 --warmup 5) against long runs (--steps 100 --warmup 20),
# interleaved on one box: is the short window systematically slower?
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
val() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" "$1" "$2"; }
for r in 1 2 3; do
  timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 ${ARGS:-} > gpurun_out/drv_$r.log 2>&1 || { tail -20 gpurun_out/drv_$r.log; exit 1; }
  val gpurun_out/drv_$r.log drv
  timeout -k 10 120 python bench.py --steps 100 --warmup 20 ${ARGS:-} > gpurun_out/long_$r.log 2>&1 || { tail -20 gpurun_out/long_$r.log; exit 1; }
  val gpurun_out/long_$r.log long
done
