#!/bin/bash
# Interleaved x3_micro rounds: the current tree, the round-3 final tree (probes_src/r3, built in-tree on the CPU side).   x3_r3_ab.sh <rounds>
set -e
R=$PWD
for r in $(seq 1 $1); do
  echo "== current round $r"; timeout -k 10 200 python3 bench/x3_micro.py --reps 3
  echo "== r3 round $r"; (cd $R/probes_src/r3 && PYTHONPATH=. timeout -k 10 200 python3 bench/x3_micro.py --reps 3)
done
