# Multi-rank rehearsal of bench.py on ONE card: gloo process group, ranks sharing the GPU
# (APNEAUQ_REHEARSE_SHARED_GPU), a smaller window set so N ranks' batch-BN activations fit.
# Exercises the launcher, rank-consistent chunking, SyncBN all-reduces and the DE member exchange.
set -o pipefail
mkdir -p gpurun_out
export APNEAUQ_DIST_BACKEND=gloo APNEAUQ_REHEARSE_SHARED_GPU=1
timeout -k 10 400 python bench.py --gpus 2 --windows 4096 --steps 3 --warmup 1 > gpurun_out/rehearse2.log 2>&1 && \
timeout -k 10 400 python bench.py --gpus 4 --windows 2048 --steps 3 --warmup 1 > gpurun_out/rehearse4.log 2>&1
rc=$?
echo EXIT $rc
tail -c 600 gpurun_out/rehearse2.log; echo; tail -c 600 gpurun_out/rehearse4.log
exit $rc
