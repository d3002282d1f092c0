set -o pipefail
mkdir -p gpurun_out
export APNEAUQ_DIST_BACKEND=gloo
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 3 --warmup 1 > gpurun_out/rehearse2.log 2>&1 && \
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29532 bench.py --gpus 4 --steps 3 --warmup 1 > gpurun_out/rehearse4.log 2>&1
echo EXIT $?
tail -2 gpurun_out/rehearse2.log; tail -2 gpurun_out/rehearse4.log
