# ResNet-50 A/B: round-1 tree (r1_old/, built in place) vs HEAD, and BN backward reduce geometry.
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
run() { tag=$1; shift; timeout -k 10 200 "$@" > $R/gpurun_out/abrn_$tag.log 2>&1 || { tail -20 $R/gpurun_out/abrn_$tag.log; exit 1; }; echo "$tag $(tail -1 $R/gpurun_out/abrn_$tag.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"; }
if [ -d r1_old ]; then (cd r1_old && run r1 python bench_resnet.py --batch 128 --steps 20 --warmup 5); fi
run head python bench_resnet.py --batch 128 --steps 20 --warmup 5
DPA_BN_BWD_BLOCKS=1024 run b1024 python bench_resnet.py --batch 128 --steps 20 --warmup 5
DPA_BN_BWD_BLOCKS=2048 run b2048 python bench_resnet.py --batch 128 --steps 20 --warmup 5
DPA_BN_BWD_BLOCK=1024 run wide python bench_resnet.py --batch 128 --steps 20 --warmup 5
run head2 python bench_resnet.py --batch 128 --steps 20 --warmup 5
