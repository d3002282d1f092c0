#!/usr/bin/env python3
"""Static instruction mix per basic block of one kernel in a gfx950 assembly listing.

    hipcc --offload-arch=gfx950 -O3 --cuda-device-only -S x.hip -o x.s
    python tools/isa_blocks.py x.s fwd_kernelILi2E [--all]
"""
import re
import sys


def main():
    path, pat = sys.argv[1], sys.argv[2]
    show_all = "--all" in sys.argv
    s = open(path).read()
    m = re.search(r"^(_Z\S*" + re.escape(pat) + r"\S*):", s, re.M)
    if not m:
        sys.exit(f"no kernel matching {pat}")
    i = m.start()
    j = s.index(".Lfunc_end", i)
    blocks, cur = [], ["entry", []]
    for line in s[i:j].splitlines():
        t = line.split(";")[0].strip()
        if not t:
            continue
        if re.match(r"^\.LBB\S+:$", t):
            blocks.append(cur)
            cur = [t[:-1], []]
        elif not t.startswith((".", "//")) and not t.endswith(":"):
            cur[1].append(t.split()[0])
    blocks.append(cur)
    tot = {"mfma": 0, "valu": 0, "ds": 0, "vmem": 0, "salu": 0}
    print(f"{m.group(1)}")
    print(f"{'block':14s} {'n':>5s} {'mfma':>5s} {'valu':>5s} {'ds':>4s} {'vmem':>4s} {'salu':>4s}  top valu ops")
    for lab, ins in blocks:
        mf = sum(x.startswith("v_mfma") for x in ins)
        va = [x for x in ins if x.startswith("v_") and not x.startswith("v_mfma")]
        ds = sum(x.startswith("ds_") for x in ins)
        vm = sum(x.startswith(("global_", "buffer_", "flat_")) for x in ins)
        sa = sum(x.startswith("s_") for x in ins)
        for k, v in (("mfma", mf), ("valu", len(va)), ("ds", ds), ("vmem", vm), ("salu", sa)):
            tot[k] += v
        if show_all or mf or len(va) > 40:
            hist = {}
            for x in va:
                hist[x] = hist.get(x, 0) + 1
            top = ", ".join(f"{k}:{v}" for k, v in sorted(hist.items(), key=lambda kv: -kv[1])[:6])
            print(f"{lab:14s} {len(ins):5d} {mf:5d} {len(va):5d} {ds:4d} {vm:4d} {sa:4d}  {top}")
    print("total (static):", tot)


if __name__ == "__main__":
    main()
