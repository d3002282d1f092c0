# single-model HIP training step vs batch size (what a member-batched launch could reach)
cd /root/repo
export PYTHONPATH=/root/repo
for b in 1024 2048 4096 8192; do
  timeout -k 10 120 python3 bench/train_micro.py --batch $b --steps 30 || exit 1
done
