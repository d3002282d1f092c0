#!/bin/bash
# Training-step phase ablations (timing only; results garbage by construction): kernel traces of
# bench/train_prof.py with the library .so and each gpuprobe/abl_<v>.so variant.
#   tools/probes/train_abl.sh tag v1 v2 ...
set -o pipefail
tag=$1; shift
mkdir -p gpurun_out; export TMPDIR=/tmp
for v in lib "$@"; do
  for b in 1024 8192; do
    s=$([ $b = 1024 ] && echo 30 || echo 8)
    so=""; [ $v != lib ] && so=/root/repo/gpuprobe/abl_$v.so
    d=/root/repo/gpurun_out/${tag}_${v}_$b
    cd /tmp && APNEAUQ_SO_PATH=$so timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o p -- \
      python3 /root/repo/bench/train_prof.py --batch $b --steps $s > $d.log 2>&1 || { echo PROF FAILED $v $b; tail $d.log; exit 1; }
    cd /root/repo
    f=$(find $d -name "*kernel_stats.csv" | head -1)
    echo "== $v batch $b"; python tools/prof_summary.py $f 20 | grep -E "dgrad|wgrad_kernel|kernel \|"
  done
done
