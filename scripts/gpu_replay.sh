#!/bin/bash
# Differential re-execution under multi-process load (tools/replay_check.py); CFGS items "procs:batch:impl:env"
set -o pipefail
mkdir -p gpurun_out/replay
n=0
for cfg in ${CFGS:-"4:64:h2:" "4:256:h2:"}; do
  IFS=: read -r p b i e <<< "$cfg"; n=$((n+1))
  timeout -k 10 ${TMO:-200} python -u tools/replay_check.py ${RARGS:-} --procs $p --batch $b --impl $i --pairs ${PAIRS:-400} --seconds ${SECS:-60} --env "$e" > gpurun_out/replay/r$n.json 2> gpurun_out/replay/r$n.err || { tail -30 gpurun_out/replay/r$n.err; exit 1; }
  echo "$cfg"; python -c 'import json,sys; d=json.load(open(sys.argv[1])); print("bad_total", d["bad_pairs_total"]); [print({k: v for k, v in r.items() if k not in ("first_diffs", "diag")}, list(r["first_diffs"].values())[:1]) for r in d["rows"]]; [print("DIAG", r["rank"], json.dumps(x)) for r in d["rows"] for x in r.get("diag", [])[:2]]' gpurun_out/replay/r$n.json
done
