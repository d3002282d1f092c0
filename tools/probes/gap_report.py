"""Busy vs idle time of the GPU over a rocprofv3 kernel trace (csv): per-kernel sums, the union of
kernel intervals and the gaps between consecutive dispatches (launch / graph-node overhead).

    python tools/probes/gap_report.py <kernel_trace.csv>
"""
import csv
import sys
from collections import defaultdict


def main(path):
    rows = list(csv.DictReader(open(path)))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    # keep the last half of the trace (steady state)
    ev = ev[len(ev) // 2:]
    t0, t1 = ev[0][0], max(e[1] for e in ev)
    busy, cur_s, cur_e = 0, None, None
    gaps = []
    for s, e, _ in ev:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
                gaps.append(s - cur_e)
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    per = defaultdict(lambda: [0, 0])
    for s, e, n in ev:
        per[n][0] += e - s
        per[n][1] += 1
    span = t1 - t0
    ksum = sum(e - s for s, e, _ in ev)
    print(f"kernel-time sum {ksum / 1e6:.3f} ms vs union {busy / 1e6:.3f} ms (concurrent {100 * (ksum - busy) / max(busy, 1):.1f} %)")
    print(f"span {span / 1e6:.3f} ms, busy {busy / 1e6:.3f} ms ({100 * busy / span:.1f} %), {len(ev)} dispatches, "
          f"{len(gaps)} gaps, mean gap {sum(gaps) / max(len(gaps), 1) / 1e3:.2f} us")
    for n, (t, c) in sorted(per.items(), key=lambda kv: -kv[1][0])[:30]:
        print(f"{t / 1e6:9.3f} ms {c:6d} x {t / c / 1e3:8.1f} us  {n[:90]}")


if __name__ == "__main__":
    main(sys.argv[1])
