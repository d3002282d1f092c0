"""Summarise fused-kernel phase stamps (tools/probes/fused_ablation.hip built with -DAPNEAUQ_STAMPS).

Per layer: K-loop issue time, barrier wait before the epilogue, epilogue time, trailing barrier.
Times in shader-clock cycles (s_memtime), medians over waves of the steady-state workgroups."""
import sys

import numpy as np

WG, W, N = 2048, 4, 32


def load(path):
    raw = open(path, "rb").read()
    cu = np.frombuffer(raw[: WG * 4], dtype=np.uint32)
    st = np.frombuffer(raw[WG * 4:], dtype=np.uint64).reshape(WG, W, N).astype(np.int64)
    return cu, st


def report(path):
    cu, st = load(path)
    sel = st[512:WG]  # skip the first dispatch rounds
    t0 = sel[:, :, 0:1]
    rel = sel - t0
    total = np.median(sel[:, :, 1] - sel[:, :, 0])
    print(f"== {path}: median tile time {total:.0f} cycles")
    rows = []
    prev_end = np.zeros_like(sel[:, :, 0])
    for l in range(6):
        ks, ke, es, ee = (sel[:, :, 2 + 4 * l + i] for i in range(4))
        start_gap = ks - (sel[:, :, 0] if l == 0 else sel[:, :, 5 + 4 * (l - 1)])
        kl = ke - ks
        bw = es - ke
        ep = (ee - es) if l < 5 else (sel[:, :, 1] - es)
        rows.append((l + 1, np.median(start_gap), np.median(kl), np.median(bw), np.median(ep)))
    print(f"{'layer':>5} {'pre(bar)':>9} {'K-loop':>8} {'bar-wait':>9} {'epilogue':>9}")
    for r in rows:
        print(f"{r[0]:>5} {r[1]:>9.0f} {r[2]:>8.0f} {r[3]:>9.0f} {r[4]:>9.0f}")
    s = np.array([r[1:] for r in rows]).sum(0)
    print(f"{'sum':>5} {s[0]:>9.0f} {s[1]:>8.0f} {s[2]:>9.0f} {s[3]:>9.0f}")
    # co-residency: two WGs on the same CU overlapping in time
    starts, ends = st[:, 0, 0], st[:, 0, 1]
    by_cu = {}
    for b in range(WG):
        by_cu.setdefault(int(cu[b]), []).append(b)
    ov = []
    for bs in by_cu.values():
        bs = sorted(bs, key=lambda b: starts[b])
        for i in range(len(bs) - 1):
            a, c = bs[i], bs[i + 1]
            if starts[c] < ends[a]:
                ov.append((starts[c] - starts[a]) / max(1, ends[a] - starts[a]))
    if ov:
        print(f"co-resident start offset (fraction of tile): median {np.median(ov):.2f}, p10 {np.percentile(ov, 10):.2f}, p90 {np.percentile(ov, 90):.2f}")


if __name__ == "__main__":
    for p in sys.argv[1:]:
        report(p)
