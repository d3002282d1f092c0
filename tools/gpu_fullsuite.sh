set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m "not gpu" -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_cpu_on_gpu.log 2>&1
echo EXIT $?
tail -15 gpurun_out/pytest_cpu_on_gpu.log
