# block 3 output hand-off through LDS (library) vs direct epilogue stores (nooutlds.so)
set -o pipefail
cd /root/repo
export PYTHONPATH=/root/repo
timeout -k 10 300 python -u -m pytest tests/test_x3_gpu.py tests/test_uq_fp32_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_x3_ol.log 2>&1 && tail -2 gpurun_out/t_x3_ol.log || { tail -30 gpurun_out/t_x3_ol.log; exit 1; }
bash tools/probes/x3_abl.sh ol default probes_so/nooutlds.so > gpurun_out/abl_ol.txt 2>&1 && cat gpurun_out/abl_ol.txt
for r in 1 2; do
  echo -n "lib r$r: "; timeout -k 10 200 python3 bench/x3_micro.py --reps 3 --only mcd,de || exit 1
  echo -n "direct r$r: "; APNEAUQ_SO_PATH=/root/repo/probes_so/nooutlds.so timeout -k 10 200 python3 bench/x3_micro.py --reps 3 --only mcd,de || exit 1
done
