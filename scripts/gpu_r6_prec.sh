#!/bin/bash
# precision report (tools/parity_report.py) at the random init and the torch-trained state, then the suite's trained-state test
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/parity_report.py > gpurun_out/r6_prec.log 2>&1 || { tail -20 gpurun_out/r6_prec.log; exit 1; }
cat gpurun_out/r6_prec.log
