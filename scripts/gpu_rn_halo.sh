# ResNet-50: re-tune the 3x3/s1 conv calls with the halo tiles as candidates, then bench.
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 200 python bench_resnet.py --batch 128 > gpurun_out/bench_resnet_before.log 2>&1
echo "resnet before $(grep -o '"value": [0-9.]*' gpurun_out/bench_resnet_before.log)"
python - <<'PY'
import json
p = "distributed_pytorch_amd/tuning/generic_mi355x.json"
d = json.load(open(p))
drop = [k for k in d if k.endswith("|3|3|1|1")]
for k in drop:
    del d[k]
json.dump(d, open(p, "w"), indent=0, sort_keys=True)
print("re-tuning", len(drop), "3x3/s1 calls")
PY
timeout -k 10 500 python bench_resnet.py --batch 128 --autotune > gpurun_out/bench_resnet_tune.log 2>&1
echo "resnet tuned-run $(grep -o '"value": [0-9.]*' gpurun_out/bench_resnet_tune.log)"
cp distributed_pytorch_amd/tuning/generic_mi355x.json gpurun_out/generic_mi355x.json
timeout -k 10 200 python bench_resnet.py --batch 128 > gpurun_out/bench_resnet_after.log 2>&1
echo "resnet after $(grep -o '"value": [0-9.]*' gpurun_out/bench_resnet_after.log)"
