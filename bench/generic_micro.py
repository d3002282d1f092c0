"""Micro-benchmark of the layer-wise HIP path (ops/generic.py) for non-reference architectures:
MC Dropout T passes over N windows, windows/s; ``--spec reference`` runs the reference
architecture through the generic kernels for comparison with the fused kernel (bench/fused_micro.py);
``pooled`` and ``single30`` take the fused multi-sample-tile kernels (csrc/fused_tiled.hip),
``*_layerwise`` the same models on the layer-wise kernels."""
import argparse
import dataclasses
import json
import time

import torch

from uncertaintyquantification_sleepapnea_1dcnn_amd.models import reference as R
from uncertaintyquantification_sleepapnea_1dcnn_amd.models.spec import DEFAULT_SPEC, BlockSpec, ModelSpec
from uncertaintyquantification_sleepapnea_1dcnn_amd.ops import generic

SPECS = {
    "reference": DEFAULT_SPEC,
    "pooled": dataclasses.replace(DEFAULT_SPEC, blocks=tuple(dataclasses.replace(b, pool=(i < 5))
                                                             for i, b in enumerate(DEFAULT_SPEC.blocks))),
    "single30": ModelSpec(30, 1, tuple(BlockSpec(f, k, r) for f, k, r in
                                       [(128, 7, 0.3), (192, 5, 0.3), (224, 3, 0.4), (96, 7, 0.2), (256, 9, 0.3),
                                        (96, 9, 0.5)])),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=16384)
    ap.add_argument("--T", type=int, default=50)
    ap.add_argument("--iters", type=int, default=3)
    a = ap.parse_args()
    res = {}
    runs = list(SPECS.items()) + [("pooled_layerwise", SPECS["pooled"]), ("single30_layerwise", SPECS["single30"])]
    for name, spec in runs:
        p = {k: v.cuda() for k, v in R.synthetic_params(spec, 1).items()}
        pk = generic.pack(spec, p)
        if name.endswith("_layerwise"):  # the layer-wise kernels on a spec a fused tiled kernel covers
            pk = {k: v for k, v in pk.items() if k != "tiled_blob"}
        x = torch.randn(a.n, spec.input_length, spec.input_channels, device="cuda").to(torch.bfloat16)
        fn = lambda: generic.forward(pk, spec, x, n_pass=a.T, dropout=True, seed=3)  # noqa: E731
        fn()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(a.iters):
            fn()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / a.iters
        res[name] = {"ms": dt * 1e3, "windows_per_s": a.n / dt,
                     "tflops_eff": a.n * a.T * 2 * spec.forward_macs() / dt / 1e12}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
