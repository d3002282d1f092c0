"""Summarise rocprofv3 ``--pmc`` passes (``tools/probes/pmc_run.sh``) into one Markdown table per kernel.

Reads every ``*counter_collection.csv`` under the given directory (one sub-directory per pass),
sums each counter over the dispatches of a kernel and derives:

* ``clk GHz``      = (GRBM_GUI_ACTIVE / 8 XCDs) / kernel time  -- sanity check of the normalisation;
* ``MFMA busy``    = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8): the fraction of
                     SIMD-cycles the matrix pipe was busy (the counter counts cycles per SIMD);
* ``MFMA/wave-cyc``, the wave-cycle split (active / waiting on a dependency or barrier / issue-stalled);
* ``LDS conflict`` = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE;
* ``L2 hit``       = TCC_HIT / (TCC_HIT + TCC_MISS);  ``HBM rd/wr GB/s`` from FETCH_SIZE / WRITE_SIZE (KB).
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def load(root):
    per = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))  # kernel -> counter -> pass -> sum
    durs = defaultdict(dict)                          # kernel -> (pass, dispatch) -> ns
    for path in sorted(glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)):
        pas = os.path.relpath(path, root).split(os.sep)[0]
        with open(path) as f:
            for r in csv.DictReader(f):
                k = r.get("Kernel_Name", "?")
                per[k][r["Counter_Name"]][pas] += float(r["Counter_Value"])
                key = (pas, r.get("Dispatch_Id", r.get("Correlation_Id")))
                try:
                    durs[k][key] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
                except (KeyError, ValueError):
                    pass
    # a counter collected in several passes (GRBM_GUI_ACTIVE): average over its passes
    vals = {k: {n: sum(v.values()) / len(v) for n, v in cs.items()} for k, cs in per.items()}
    return vals, durs


def main(root, top=12):
    vals, durs = load(root)
    rows = []
    for k, c in vals.items():
        # per-pass kernel time (each pass re-runs the program): use the pass that holds GRBM_GUI_ACTIVE
        by_pass = defaultdict(float)
        for (pas, _), ns in durs[k].items():
            by_pass[pas] += ns
        t_ns = max(by_pass.values()) if by_pass else 0.0
        rows.append((t_ns, k, c, by_pass))
    rows.sort(key=lambda r: -r[0])
    print(f"PMC summary of `{root}` (sums over all dispatches of a kernel; one program run per pass)\n")
    print("| kernel | time ms | clk GHz | MFMA busy | MFMA insts | VALU insts | wave cyc: active / wait / stall "
          "| LDS conflict | L2 hit | HBM rd GB/s | HBM wr GB/s |")
    print("|---|---:|---:|---:|---:|---:|---|---:|---:|---:|---:|")
    for t_ns, k, c, by_pass in rows[:top]:
        name = k if len(k) < 70 else k[:67] + "..."
        g = c.get("GRBM_GUI_ACTIVE", 0.0)
        g_pass = g
        t_s = t_ns / 1e9 if t_ns else float("nan")
        clk = g_pass / 8 / t_s / 1e9 if g_pass and t_ns else float("nan")
        mfma = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (1024 * g_pass / 8) if g_pass else float("nan")
        wc = c.get("SQ_WAVE_CYCLES", 0.0)
        act = c.get("SQ_ACTIVE_INST_ANY", 0.0) / wc if wc else float("nan")
        wait = c.get("SQ_WAIT_ANY", 0.0) / wc if wc else float("nan")
        stall = c.get("SQ_WAIT_INST_ANY", 0.0) / wc if wc else float("nan")
        lds = c.get("SQ_LDS_BANK_CONFLICT", 0.0) / c["SQ_LDS_IDX_ACTIVE"] if c.get("SQ_LDS_IDX_ACTIVE") else float("nan")
        hit, miss = c.get("TCC_HIT_sum", 0.0), c.get("TCC_MISS_sum", 0.0)
        l2 = hit / (hit + miss) if hit + miss else float("nan")
        rd = c.get("FETCH_SIZE", 0.0) * 1024 / t_s / 1e9 if t_ns else float("nan")
        wr = c.get("WRITE_SIZE", 0.0) * 1024 / t_s / 1e9 if t_ns else float("nan")
        print(f"| `{name}` | {t_ns / 1e6:.2f} | {clk:.2f} | {mfma:.1%} | {c.get('SQ_INSTS_MFMA', 0):.3g} | "
              f"{c.get('SQ_INSTS_VALU', 0):.3g} | {act:.0%} / {wait:.0%} / {stall:.0%} | {lds:.1%} | {l2:.1%} | "
              f"{rd:.0f} | {wr:.0f} |")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 12)
