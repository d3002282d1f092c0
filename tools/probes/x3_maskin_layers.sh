# per-layer kernel times: dropout masks drawn in the producer epilogue (0) vs the consumer loaders (1)
set -o pipefail
cd /root/repo
export PYTHONPATH=/root/repo
bash tools/probes/x3_abl.sh mask0 default > gpurun_out/abl_mask0.txt 2>&1 && cat gpurun_out/abl_mask0.txt
APNEAUQ_X3_MASK_IN=1 bash tools/probes/x3_abl.sh mask1 default > gpurun_out/abl_mask1.txt 2>&1 && cat gpurun_out/abl_mask1.txt
