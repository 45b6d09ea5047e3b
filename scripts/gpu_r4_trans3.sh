# driver-window transient: is it tied to steps since process start, or steps since the last sync?
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {
  tag=$1; shift
  timeout -k 10 200 python tools/step_transient.py --steps 60 "$@" > gpurun_out/r4trans3_$tag.txt 2>&1 || exit 1
  echo "$tag [$*]"; grep "^steps" gpurun_out/r4trans3_$tag.txt
}
run w5 --warmup 5
run w40 --warmup 40
run w100 --warmup 100
