# round-4 final tree: step trace + the two one-stream PMC passes (tools/pmc_summary.py)
TAG=r4f PMC=1 bash scripts/gpu_profile.sh
