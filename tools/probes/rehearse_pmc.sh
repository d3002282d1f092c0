# (1) 2-rank rehearsal of bench.py on one card (gloo; the SCALE code path: sharded batch-BN MCD with
#     SyncBN, member-parallel DE with all_to_all); (2) PMC counters of the x3 layer kernels
set -o pipefail
cd /root/repo
export PYTHONPATH=/root/repo TMPDIR=/tmp
APNEAUQ_DIST_BACKEND=gloo APNEAUQ_REHEARSE_SHARED_GPU=1 timeout -k 10 400 python3 bench.py --gpus 2 --windows 4096 --steps 3 --warmup 1 --no-secondary > gpurun_out/rehearse2.json 2> gpurun_out/rehearse2.err || { tail -30 gpurun_out/rehearse2.err; exit 1; }
cat gpurun_out/rehearse2.json
bash tools/probes/x3_pmc_tcp.sh > gpurun_out/pmc_r3.txt 2>&1; cat gpurun_out/pmc_r3.txt
