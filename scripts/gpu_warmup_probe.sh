# Which part of the short driver window is slow: warmup length or timed-window length?
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
val() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" "$1" "$2"; }
for r in 1 2; do
  for cfg in "20 5" "20 20" "100 5" "20 60"; do
    set -- $cfg
    timeout -k 10 120 python bench.py --steps $1 --warmup $2 > gpurun_out/wp_$1_$2_$r.log 2>&1 || { tail -20 gpurun_out/wp_$1_$2_$r.log; exit 1; }
    val gpurun_out/wp_$1_$2_$r.log "steps=$1 warmup=$2"
  done
done
