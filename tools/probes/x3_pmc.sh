#!/bin/bash
# Vector-memory-path counters (TA / TD / TCP) of the x3 layer kernels (one rocprofv3 --pmc pass),
# plus an SQ pass for MFMA busy / clock.  Summaries per kernel to stdout.
R=$PWD; export PYTHONPATH=$R TMPDIR=/tmp
OUT=$R/gpurun_out/x3_tcp; rm -rf $OUT; mkdir -p $OUT
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc TA_BUSY_avr TA_DATA_STALLED_BY_TC_CYCLES_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE --output-format csv -d $OUT/p1 -o run -- python3 $R/bench/x3_micro.py --reps 1 --only mcd --passes 10 > $OUT/p1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $OUT/p2 -o run -- python3 $R/bench/x3_micro.py --reps 1 --only mcd --passes 10 > $OUT/p2.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE --output-format csv -d $OUT/p3 -o run -- python3 $R/bench/x3_micro.py --reps 1 --only mcd --passes 10 > $OUT/p3.log 2>&1 || echo "p3 failed"
cd $R
python3 - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float))
dur = collections.defaultdict(float)
for f in glob.glob("gpurun_out/x3_tcp/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "layer_kernel" in k:
            k = k.split("<")[1].split(">")[0]
            agg[k][r["Counter_Name"] + ("@p1" if "/p1/" in f else "@p3" if "/p3/" in f else "@p2")] += float(r["Counter_Value"])
for k, v in agg.items():
    g1 = v["GRBM_GUI_ACTIVE@p1"] / 8
    g2 = v["GRBM_GUI_ACTIVE@p2"] / 8
    print(f"{k}: TA busy {v['TA_BUSY_avr@p1']/max(g1,1)*100:.0f}%  TA stalled-by-TC {v['TA_DATA_STALLED_BY_TC_CYCLES_sum@p1']/256/max(g1,1)*100:.0f}%  "
          f"TD busy {v['TD_TD_BUSY_sum@p1']/256/max(g1,1)*100:.0f}%  TD TC-stall {v['TD_TC_STALL_sum@p1']/256/max(g1,1)*100:.0f}%  "
          f"L1 hit {100*(1 - v['TCP_TCC_READ_REQ_sum@p1']/max(v['TCP_TOTAL_CACHE_ACCESSES_sum@p1'],1)):.0f}%  "
          f"TCP pend-stall {v['TCP_PENDING_STALL_CYCLES_sum@p1']/256/max(g1,1)*100:.0f}%  "
          f"MFMA busy {v['SQ_VALU_MFMA_BUSY_CYCLES@p2']/1024/max(g2,1)*100:.0f}%  VALU/MFMA {v['SQ_INSTS_VALU@p2']/max(v['SQ_INSTS_MFMA@p2'],1):.2f}")
    g3 = v["GRBM_GUI_ACTIVE@p3"] / 8
    if g3:
        print(f"    LDS active {v['SQ_LDS_IDX_ACTIVE@p3']/256/g3*100:.0f}%  bank-conflict/active {v['SQ_LDS_BANK_CONFLICT@p3']/max(v['SQ_LDS_IDX_ACTIVE@p3'],1)*100:.1f}%  "
              f"LDS insts/MFMA {v['SQ_INSTS_LDS@p3']/max(v['SQ_INSTS_MFMA@p2'],1):.2f}  VMEM rd/MFMA {v['SQ_INSTS_VMEM_RD@p3']/max(v['SQ_INSTS_MFMA@p2'],1):.3f}  "
              f"wait-LDS/wave {v['SQ_WAIT_INST_LDS@p3']/max(v['SQ_WAVES@p2'],1):.0f}  active VALU {v['SQ_ACTIVE_INST_VALU@p3']/256/g3*100:.0f}%  active LDS {v['SQ_ACTIVE_INST_LDS@p3']/256/g3*100:.0f}%")
PY
