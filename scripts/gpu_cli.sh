# CLI / checkpoint / smoke checks on one GPU
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
timeout -k 10 300 python __graft_entry__.py smoke 2>&1 | tail -1
timeout -k 10 300 python main.py --synthetic --train-size 12800 --test-size 2560 --max-iters 45 --checkpoint-dir /tmp/ck --checkpoint-every 40 > gpurun_out/cli_main.log 2>&1
tail -4 gpurun_out/cli_main.log
timeout -k 10 300 python main.py --synthetic --train-size 12800 --test-size 2560 --checkpoint-dir /tmp/ck --resume --no-eval --max-iters 5 > gpurun_out/cli_resume.log 2>&1
tail -2 gpurun_out/cli_resume.log
MASTER_ADDR=127.0.0.1 MASTER_PORT=29555 WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 LOCAL_WORLD_SIZE=1 timeout -k 10 300 python main_ddp.py --synthetic --train-size 5120 --test-size 1024 > gpurun_out/cli_ddp.log 2>&1
head -1 gpurun_out/cli_ddp.log; tail -2 gpurun_out/cli_ddp.log
