# x3 A/B: library vs DPP row sums (dpp.so) vs DPP + two chunks of loader prefetch (pf2.so).
set -o pipefail
cd /root/repo
export PYTHONPATH=/root/repo
APNEAUQ_SO_PATH=/root/repo/probes_so/pf2.so timeout -k 10 300 python -u -m pytest tests/test_x3_gpu.py tests/test_uq_fp32_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_x3_pf.log 2>&1 && tail -2 gpurun_out/t_x3_pf.log || { tail -30 gpurun_out/t_x3_pf.log; exit 1; }
for r in 1 2 3; do
  for v in default dpp pf2; do
    echo -n "$v r$r: "
    if [ $v = default ]; then timeout -k 10 200 python3 bench/x3_micro.py --reps 3 --only mcd,de || exit 1
    else APNEAUQ_SO_PATH=/root/repo/probes_so/$v.so timeout -k 10 200 python3 bench/x3_micro.py --reps 3 --only mcd,de || exit 1; fi
  done
done
