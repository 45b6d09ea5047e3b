# driver-window transient: frozen weights (lr 0) and a memory-bound pre-busy
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {
  tag=$1; shift
  timeout -k 10 200 python tools/step_transient.py --steps 60 --warmup 5 "$@" > gpurun_out/r4trans2_$tag.txt 2>&1 || exit 1
  echo "$tag [$*]"; grep "^steps" gpurun_out/r4trans2_$tag.txt
}
run base
run lr0 --lr 0
run mem --prewarm-ms 1500 --prewarm-kind mem
run lr0mem --lr 0 --prewarm-ms 1500 --prewarm-kind mem
