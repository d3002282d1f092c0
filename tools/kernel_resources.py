#!/usr/bin/env python3
"""Per-kernel register / spill / occupancy table of a HIP source for gfx950 (compile-only, no GPU).

    python tools/kernel_resources.py uncertaintyquantification_sleepapnea_1dcnn_amd/csrc/train_conv.hip [-DFOO=1 ...]
"""
import os
import re
import subprocess
import sys

CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                    "uncertaintyquantification_sleepapnea_1dcnn_amd", "csrc")


def main():
    src, extra = sys.argv[1], sys.argv[2:]
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-c", src, "-o", "/tmp/_kres.o", "-O3", "-std=c++17",
           f"-I{CSRC}", "-ffp-contract=fast", "-munsafe-fp-atomics", "-Rpass-analysis=kernel-resource-usage",
           *extra]
    r = subprocess.run(cmd, capture_output=True, text=True)
    rows, cur = [], None
    for line in r.stderr.splitlines():
        m = re.search(r"remark: ([A-Za-z /\[\]]+?): (.+?) \[-Rpass", line)
        if not m:
            continue
        k, v = m.group(1).strip(), m.group(2).strip()
        if k == "Function Name":
            cur = {"name": v}
            rows.append(cur)
        elif cur is not None:
            cur[k] = v
    if r.returncode != 0:
        print(r.stderr[-4000:])
        sys.exit(r.returncode)
    try:
        dem = subprocess.run(["c++filt"], input="\n".join(x["name"] for x in rows), capture_output=True,
                             text=True).stdout.splitlines()
    except OSError:
        dem = [x["name"] for x in rows]
    print(f"{'kernel':70s} {'VGPR':>5s} {'AGPR':>5s} {'spill':>5s} {'occ':>4s} {'LDS':>6s} {'scratch':>7s}")
    for x, d in zip(rows, dem):
        print(f"{d[:70]:70s} {x.get('VGPRs', '?'):>5s} {x.get('AGPRs', '?'):>5s} {x.get('VGPRs Spill', '?'):>5s} "
              f"{x.get('Occupancy [waves/SIMD]', '?'):>4s} {x.get('LDS Size [bytes/block]', '?'):>6s} "
              f"{x.get('ScratchSize [bytes/lane]', '?'):>7s}")


if __name__ == "__main__":
    main()
