# fused pooled kernel ablations (timing only): library vs probe builds given as arguments
set -o pipefail
cd /root/repo
export PYTHONPATH=/root/repo
for r in 1 2; do
  timeout -k 10 120 python3 tools/probes/pooled_time.py lib || exit 1
  for so in "$@"; do APNEAUQ_SO_PATH=/root/repo/$so timeout -k 10 120 python3 tools/probes/pooled_time.py $so || exit 1; done
done
