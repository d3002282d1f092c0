set -e
export TMPDIR=/tmp PYTHONPATH=$PWD
mkdir -p gpurun_out/deprof
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/deprof/de -o run -- python3 bench/x3_micro.py --reps 2 --only de > gpurun_out/deprof/de.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/deprof/mcd -o run -- python3 bench/x3_micro.py --reps 2 --only mcd --passes 8 > gpurun_out/deprof/mcd.log 2>&1
tail -1 gpurun_out/deprof/de.log; tail -1 gpurun_out/deprof/mcd.log
