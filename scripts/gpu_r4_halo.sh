# EXPERIMENT: halo conv staging cost bounds (DPA_HALO_DBG)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/halo_staging_bound.py > gpurun_out/r4_halo_bound.jsonl 2>&1; echo "fprop rc=$?"; cat gpurun_out/r4_halo_bound.jsonl
timeout -k 10 200 python -u tools/halo_staging_bound.py --dgrad >> gpurun_out/r4_halo_bound.jsonl 2>&1; echo "dgrad rc=$?"; tail -5 gpurun_out/r4_halo_bound.jsonl
