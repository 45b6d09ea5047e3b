# driver-window transient: cold process vs GPU pre-busied for 0.3 s / 1.5 s before the warmup steps
export TMPDIR=/tmp
mkdir -p gpurun_out
for pw in 0 300 1500 0; do
  timeout -k 10 200 python tools/step_transient.py --steps 60 --warmup 5 --prewarm-ms $pw > gpurun_out/r4trans_$pw.txt 2>&1 || exit 1
  echo "prewarm $pw"; grep "^steps" gpurun_out/r4trans_$pw.txt
done
