#!/bin/bash
# Per-kernel times of x3 probe builds (rocprofv3 kernel trace, one run each):
#   tools/probes/x3_abl.sh <tag> <so...>   ("default" = the library build)
set -e
tag=$1; shift
R=/root/repo; export PYTHONPATH=$R TMPDIR=/tmp
OUT=$R/gpurun_out/abl_$tag; rm -rf $OUT; mkdir -p $OUT
for so in "$@"; do
  name=$(basename $so .so | tr '=,:/' '____')
  T=$R  # "tree:<dir>" = another whole checkout (e.g. probes_src/r3), its own package and bench
  E=()  # "env:VAR=VALUE" = the library build under that environment variable
  if [ "$so" = "default" ]; then unset APNEAUQ_SO_PATH
  elif [ "${so#env:}" != "$so" ]; then unset APNEAUQ_SO_PATH; E=("${so#env:}")
  elif [ "${so#tree:}" != "$so" ]; then unset APNEAUQ_SO_PATH; T=$R/${so#tree:}
  else export APNEAUQ_SO_PATH=$R/$so; fi
  env "${E[@]}" PYTHONPATH=$T timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$name -o run -- \
    python3 $T/bench/x3_micro.py --reps 1 --only mcd --passes 20 > $OUT/$name.log 2>&1
done
unset APNEAUQ_SO_PATH
python3 - "$OUT" <<'PY'
import csv, glob, os, sys
root = sys.argv[1]
rows = {}
for d in sorted(glob.glob(os.path.join(root, "*"))):
    if not os.path.isdir(d):
        continue
    f = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)
    if not f:
        continue
    for r in csv.DictReader(open(f[0])):
        if "layer_kernel" in r["Name"]:
            key = ",".join(r["Name"].split("<")[1].split(">")[0].split(",")[:3])  # Cin, Cout, k: the layer
            rows.setdefault(key, {})[os.path.basename(d)] = int(r["TotalDurationNs"]) / 1e6
names = sorted({n for v in rows.values() for n in v})
print("| layer_kernel<> | " + " | ".join(names) + " |")
print("|---|" + "---:|" * len(names))
for k, v in rows.items():
    print(f"| {k} | " + " | ".join(f"{v.get(n, 0):.2f}" for n in names) + " |")
print("| total | " + " | ".join(f"{sum(v.get(n, 0) for v in rows.values()):.2f}" for n in names) + " |")
PY
