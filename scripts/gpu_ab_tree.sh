# Interleaved A/B of the in-tree build against ab_old/ (HEAD, built in place): VGG and ResNet benches.
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 400 python -u -m pytest $TESTS -x -q --timeout 150 --timeout-method thread > gpurun_out/abt_tests.log 2>&1 || { tail -40 gpurun_out/abt_tests.log; exit 1; }
  tail -1 gpurun_out/abt_tests.log
fi
run() { tag=$1; dir=$2; shift 2; (cd $dir && timeout -k 10 200 "$@" > $R/gpurun_out/abt_$tag.log 2>&1) || { tail -20 $R/gpurun_out/abt_$tag.log; exit 1; }; echo "$tag $(tail -1 $R/gpurun_out/abt_$tag.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"; }
for r in 1 2; do
  run new_vgg$r $R python bench.py --steps 100 --warmup 20
  run old_vgg$r $R/ab_old python bench.py --steps 100 --warmup 20
  run new_rn$r $R python bench_resnet.py --steps 20 --warmup 5
  run old_rn$r $R/ab_old python bench_resnet.py --steps 20 --warmup 5
done
