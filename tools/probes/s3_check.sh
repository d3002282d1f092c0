set -o pipefail
bash tools/gpu_quick.sh sp1 "tests/test_train_gpu.py tests/test_deterministic_gpu.py" || exit 1
timeout -k 10 200 python -m bench.train_micro --steps 50 > gpurun_out/sp1_train.json 2>&1 && cat gpurun_out/sp1_train.json | tail -2
