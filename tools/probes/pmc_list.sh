#!/bin/bash
# List the PMC counters rocprofv3 offers on this box (gfx950) into gpurun_out/pmc_list.txt.
set -e
R=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $R/gpurun_out/pmc_list.txt 2>&1 || true
grep -o "SQ_[A-Z0-9_]*\|TA_[A-Z0-9_]*\|TD_[A-Z0-9_]*\|TCC_[A-Z0-9_]*\|TCP_[A-Z0-9_]*\|GRBM_[A-Z0-9_]*\|FETCH_SIZE\|WRITE_SIZE" $R/gpurun_out/pmc_list.txt | sort -u > $R/gpurun_out/pmc_names.txt || true
wc -l $R/gpurun_out/pmc_names.txt
