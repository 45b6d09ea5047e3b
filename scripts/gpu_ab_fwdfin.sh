mkdir -p gpurun_out
R=$(pwd)
run() { tag=$1; shift; (env "$@" timeout -k 10 200 python bench.py --steps 150 --warmup 20 > $R/gpurun_out/ff_$tag.log 2>&1) || { tail -20 $R/gpurun_out/ff_$tag.log; exit 1; }; echo "$tag $* $(tail -1 $R/gpurun_out/ff_$tag.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"; }
for r in 1 2 3; do run on_$r DPA_BN_FWD_FIN_CPB=2; run off_$r DPA_BN_FWD_FIN_CPB=4; done
DPA_BN_FWD_FIN_CPB=2 timeout -k 10 300 python -m pytest tests/test_ops_gpu.py -k "engine_step_matches_torch or bn" -x -q > gpurun_out/ff_t8.log 2>&1; echo "cpb2 tests rc=$?"
