set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
for impl in x3 bf16; do timeout -k 10 120 python tools/host_overhead.py --impl $impl 2>&1 | grep impl; done
DPA_FORCE_COMM=1 timeout -k 10 120 python bench.py --steps 50 --warmup 10 2>&1 | grep -o '"value": [0-9.]*'
