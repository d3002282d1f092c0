# x3 epilogue A/B: mask drawn in the producer epilogue (library) vs in the consumer staging
# (APNEAUQ_X3_MASK_IN=1), with the DPP row sums (probes_so/dpp.so).  Numerics first, then 3 rounds.
set -o pipefail
cd /root/repo
export PYTHONPATH=/root/repo
APNEAUQ_X3_MASK_IN=1 APNEAUQ_SO_PATH=/root/repo/probes_so/dpp.so timeout -k 10 300 python -u -m pytest tests/test_x3_gpu.py tests/test_uq_fp32_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_x3_epi.log 2>&1 && tail -2 gpurun_out/t_x3_epi.log || { tail -30 gpurun_out/t_x3_epi.log; exit 1; }
for r in 1 2 3; do
  echo -n "lib mask0 r$r: "; timeout -k 10 200 python3 bench/x3_micro.py --reps 3 --only mcd,de,run || exit 1
  echo -n "lib mask1 r$r: "; APNEAUQ_X3_MASK_IN=1 timeout -k 10 200 python3 bench/x3_micro.py --reps 3 --only mcd,de,run || exit 1
  echo -n "dpp mask1 r$r: "; APNEAUQ_X3_MASK_IN=1 APNEAUQ_SO_PATH=/root/repo/probes_so/dpp.so timeout -k 10 200 python3 bench/x3_micro.py --reps 3 --only mcd,de,run || exit 1
done
