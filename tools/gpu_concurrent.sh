set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_train_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_conc.log 2>&1 && \
timeout -k 10 300 python -u -m bench.train_bench --members 8 --steps 20 --streams 1 > gpurun_out/train_bench_s1.json 2> gpurun_out/train_bench.err && \
timeout -k 10 300 python -u -m bench.train_bench --members 8 --steps 20 --streams 4 > gpurun_out/train_bench_s4.json 2>> gpurun_out/train_bench.err && \
PYTHONPATH=$PWD timeout -k 10 300 python -u tools/probes/multistream_train.py 8 > gpurun_out/multistream.json 2>> gpurun_out/train_bench.err
echo EXIT $?
tail -4 gpurun_out/pytest_conc.log
cat gpurun_out/train_bench_s1.json gpurun_out/train_bench_s4.json gpurun_out/multistream.json
