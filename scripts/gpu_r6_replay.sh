#!/bin/bash
# Round-6 replay A/B: 4-process differential replay of the training step (tools/replay_check.py) under
# several engine switches; CFGS items "label|K=V,K=V" (empty env = default)
set -o pipefail
mkdir -p gpurun_out/replay
n=0
for cfg in ${CFGS:-"default|" "onestream|DPA_WGRAD_STREAM=0" "noconv0|DPA_FUSED_CONV0=0" "nosig|DPA_KSIGNAL=0"}; do
  lbl=${cfg%%|*}; e=${cfg#*|}; n=$((n+1))
  timeout -k 10 ${TMO:-200} python -u tools/replay_check.py --procs ${P:-4} --batch 64 --impl h2 --pairs 400 --seconds ${SECS:-40} --diag --env "$e" > gpurun_out/replay/$lbl.json 2> gpurun_out/replay/$lbl.err || { tail -30 gpurun_out/replay/$lbl.err; exit 1; }
  python -c 'import json,sys; d=json.load(open(sys.argv[1])); print("==", sys.argv[2], "bad_total", d["bad_pairs_total"], "pairs", sum(r["pairs"] for r in d["rows"])); [print(r["rank"], r["bad_pairs"], r["z0_bad_pairs"], r["z0_elems_differing"], r["z0_block_hits_by_xcd"], list(r["first_diffs"].values())[:2]) for r in d["rows"]]; [print("DIAG", r["rank"], json.dumps(x)[:1200]) for r in d["rows"] for x in r.get("diag", [])[:2]]' gpurun_out/replay/$lbl.json $lbl
done
