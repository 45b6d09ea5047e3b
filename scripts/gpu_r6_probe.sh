#!/bin/bash
# Round-6 probe: torch-only and framework producer/consumer patterns under 4-process load, then the
# differential replay of the training step (tools/replay_check.py).
set -o pipefail
mkdir -p gpurun_out/mp gpurun_out/replay
timeout -k 10 300 python -u tools/mp_repro.py --procs 4 --seconds ${SECS:-10} --mode ${MODES:-fill,big,bigev,conv0,conv0alt,signal} > gpurun_out/mp/probe.jsonl 2> gpurun_out/mp/probe.err || { tail -20 gpurun_out/mp/probe.err; exit 1; }
python -c 'import json,sys
for l in open("gpurun_out/mp/probe.jsonl"):
    d=json.loads(l); print(d["mode"], "bad_total", d["bad_total"], [(r["iters"], r["bad"]) for r in d["rows"]])'
timeout -k 10 240 python -u tools/replay_check.py --procs 4 --batch 64 --impl h2 --pairs 400 --seconds ${RSECS:-45} --diag ${RARGS:-} > gpurun_out/replay/r1.json 2> gpurun_out/replay/r1.err || { tail -30 gpurun_out/replay/r1.err; exit 1; }
python -c 'import json,sys; d=json.load(open(sys.argv[1])); print("bad_total", d["bad_pairs_total"]); [print({k: v for k, v in r.items() if k not in ("diag",)}) for r in d["rows"]]; [print("DIAG", r["rank"], json.dumps(x)[:1500]) for r in d["rows"] for x in r.get("diag", [])[:1]]' gpurun_out/replay/r1.json
