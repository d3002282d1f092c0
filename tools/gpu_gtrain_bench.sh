set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m bench.generic_train_micro > gpurun_out/gtrain_micro.json 2> gpurun_out/gtrain_micro.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_gtrain -o gtrain -- python3 -m bench.generic_train_micro --specs pooled --iters 10 --no-torch > gpurun_out/prof_gtrain.log 2>&1
echo EXIT $?
cat gpurun_out/gtrain_micro.json
find gpurun_out/prof_gtrain -name "*stats*"
