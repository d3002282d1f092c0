# chunk-order rotation per tile/workgroup (library, ROT=1) vs natural chunk order (rot0.so)
set -o pipefail
cd /root/repo
export PYTHONPATH=/root/repo
timeout -k 10 300 python -u -m pytest tests/test_x3_gpu.py tests/test_uq_fp32_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_x3_rot.log 2>&1 && tail -2 gpurun_out/t_x3_rot.log || { tail -30 gpurun_out/t_x3_rot.log; exit 1; }
bash tools/probes/x3_abl.sh rot default probes_so/rot0.so > gpurun_out/abl_rot.txt 2>&1 && cat gpurun_out/abl_rot.txt
for r in 1 2; do
  echo -n "rot1 r$r: "; timeout -k 10 200 python3 bench/x3_micro.py --reps 3 --only mcd || exit 1
  echo -n "rot0 r$r: "; APNEAUQ_SO_PATH=/root/repo/probes_so/rot0.so timeout -k 10 200 python3 bench/x3_micro.py --reps 3 --only mcd || exit 1
done
