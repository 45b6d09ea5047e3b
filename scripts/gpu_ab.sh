# Interleaved A/B of one env knob on the x3 (and bf16) bench, same box: gpu_ab.sh VAR valA valB [reps]
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
VAR=$1; A=$2; B=$3; REPS=${4:-3}
for i in $(seq $REPS); do
  for v in $A $B; do
    env $VAR=$v timeout -k 10 150 python bench.py --steps 50 --warmup 10 > gpurun_out/ab_$v.log 2>&1
    echo "x3 $VAR=$v $(grep -o '"value": [0-9.]*' gpurun_out/ab_$v.log)"
  done
done
for v in $A $B; do
  env $VAR=$v timeout -k 10 150 python bench.py --steps 50 --warmup 10 --impl bf16 > gpurun_out/ab_bf16_$v.log 2>&1
  echo "bf16 $VAR=$v $(grep -o '"value": [0-9.]*' gpurun_out/ab_bf16_$v.log)"
done
