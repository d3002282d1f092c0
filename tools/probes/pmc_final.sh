set -o pipefail

bash tools/probes/pmc_run.sh mcd_s3 python3 $PWD/bench.py --steps 1 --warmup 1 --no-secondary --no-deviation > /dev/null 2>&1 || { echo MCD PMC FAILED; exit 1; }
head -40 gpurun_out/pmc_mcd_s3/summary.md
