# driver-window transient: kernel-argument placement and launch-path warm-up
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {
  tag=$1; shift
  timeout -k 10 200 python tools/step_transient.py --steps 40 --warmup 5 "$@" > gpurun_out/r4trans4_$tag.txt 2>&1 || exit 1
  echo "$tag [$*]"; grep "^steps" gpurun_out/r4trans4_$tag.txt
}
run base
export HIP_FORCE_DEV_KERNARG=0; run hostkarg
export HIP_FORCE_DEV_KERNARG=1; run devkarg; unset HIP_FORCE_DEV_KERNARG
run pre30k --prelaunch 30000
