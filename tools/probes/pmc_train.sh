#!/bin/bash
# SQ counters of the bf16 training step kernels (bench.train_micro --batch $1), one pass.
R=/root/repo; export PYTHONPATH=$R TMPDIR=/tmp
OUT=$R/gpurun_out/pmc_train_$1; rm -rf $OUT; mkdir -p $OUT
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --output-format csv -d $OUT -o run -- python3 -m bench.train_micro --batch ${1:-1024} --steps 5 > $OUT/run.log 2>&1 || exit 1
cd $R
python3 - "$OUT" <<'PY'
import csv, glob, collections, sys
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "train::" in k and "Lb0E" not in k and "false>" in k:
            agg[k.split("(")[0]][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in agg.items():
    g = v["GRBM_GUI_ACTIVE"] / 8
    print(f"{k}: MFMA busy {v['SQ_VALU_MFMA_BUSY_CYCLES']/1024/max(g,1)*100:.0f}%  VALU/MFMA {v['SQ_INSTS_VALU']/max(v['SQ_INSTS_MFMA'],1):.2f}  "
          f"LDS active {v['SQ_LDS_IDX_ACTIVE']/256/max(g,1)*100:.0f}%  bank-conflict/active {v['SQ_LDS_BANK_CONFLICT']/max(v['SQ_LDS_IDX_ACTIVE'],1)*100:.1f}%  "
          f"wait-LDS/wave {v['SQ_WAIT_INST_LDS']/max(v['SQ_WAVES'],1):.0f}")
PY
