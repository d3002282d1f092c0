#!/bin/bash
# rocprofv3 PMC passes (one run per pass, kernel-trace only, csv) over a short GPU program.
#   $1 = tag, rest = the program after "--" (e.g. python3 -m bench.fused_micro --iters 2)
# Output: gpurun_out/pmc_<tag>/p<i>/...counter_collection.csv; summarise with tools/pmc_summary.py.
set -e
tag=$1; shift
R=$PWD; export PYTHONPATH=$R
OUT=$R/gpurun_out/pmc_$tag
rm -rf $OUT; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
PASSES=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
  "SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_COEXEC_CYCLES"
  "FETCH_SIZE TCC_HIT_sum GRBM_GUI_ACTIVE"
  "WRITE_SIZE TCC_MISS_sum TCC_REQ_sum"
)
i=0
for p in "${PASSES[@]}"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $p --output-format csv -d $OUT/p$i -o run -- "$@" > $OUT/p$i.log 2>&1
done
cd $R
python3 tools/pmc_summary.py $OUT > $OUT/summary.md
cat $OUT/summary.md
