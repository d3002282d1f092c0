"""Reference-semantics comparator: the number ``bench.py``'s ``vs_baseline`` divides by.

The reference publishes no throughput, so we measure what its code does,
in plain eager fp32 PyTorch (``torch.nn`` Conv1d / BatchNorm1d / Dropout; MIOpen convs on ROCm):

* MC Dropout (``uncertainty_quantification/uq_techniques.py:12-24``): ``T`` full-test-set passes,
  each ``model(X, training=True)`` (dropout on, BN on batch statistics, running-stat side effect)
  and copied to host, stacked to (T, N, 1).
* Deep Ensemble (``uq_techniques.py:26-32``): ``m.predict(X)`` per member, Keras default batch 32,
  inference BN, no dropout, stacked to (M, N, 1).
* UQ metrics (``uq_techniques.py:40-112``): the per-window mean / variance / entropies / MI and the
  aggregates on the host with NumPy, as ``uq_evaluation_dist`` does.

One "step" = both methods over the same N windows, exactly like ``bench.py``'s step;
``windows/s = N / step time``.  ``--bn-mode running`` reruns MCD with BN on running statistics
(the semantics of ``bench.py``'s default MCD phase) for an apples-to-apples comparison.

    python -m bench.comparator --n 16384            # 1 x MI355X
    python -m bench.comparator --n 512 --device cpu # CPU
"""
from __future__ import annotations

import argparse
import json
import time

import numpy as np
import torch
from torch import nn

from uncertaintyquantification_sleepapnea_1dcnn_amd.models.reference import synthetic_params as _sp
from uncertaintyquantification_sleepapnea_1dcnn_amd.models.spec import DEFAULT_SPEC as SPEC
from uncertaintyquantification_sleepapnea_1dcnn_amd.uq import metrics as M


def synthetic_params(seed):
    return _sp(SPEC, seed)


class EagerCNN(nn.Module):
    """Plain ``torch.nn`` rendition of ``models/cnn_baseline_train.py:55-94`` (channels-last in)."""

    def __init__(self, spec=SPEC):
        super().__init__()
        layers = []
        cin = spec.input_channels
        for b in spec.blocks:
            layers += [nn.Conv1d(cin, b.filters, b.kernel_size, padding="same"), nn.ReLU(),
                       nn.BatchNorm1d(b.filters, eps=1e-3, momentum=0.01), nn.Dropout(b.dropout)]
            cin = b.filters
        self.body = nn.Sequential(*layers)
        self.dense = nn.Linear(cin, 1)

    def load_keras(self, p):
        convs = [m for m in self.body if isinstance(m, nn.Conv1d)]
        bns = [m for m in self.body if isinstance(m, nn.BatchNorm1d)]
        with torch.no_grad():
            for i, (c, b) in enumerate(zip(convs, bns), start=1):
                c.weight.copy_(p[f"conv1d_{i}/kernel"].permute(2, 1, 0))
                c.bias.copy_(p[f"conv1d_{i}/bias"])
                b.weight.copy_(p[f"batchnorm_{i}/gamma"])
                b.bias.copy_(p[f"batchnorm_{i}/beta"])
                b.running_mean.copy_(p[f"batchnorm_{i}/moving_mean"])
                b.running_var.copy_(p[f"batchnorm_{i}/moving_variance"])
            self.dense.weight.copy_(p["output_layer/kernel"].t())
            self.dense.bias.copy_(p["output_layer/bias"])
        return self

    def forward(self, x):
        h = self.body(x.transpose(1, 2))
        return torch.sigmoid(self.dense(h.mean(dim=2)))


def _sync(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize()


def mcd_reference(model, x, T, bn_mode):
    model.train()
    if bn_mode == "running":
        for m in model.modules():
            if isinstance(m, nn.BatchNorm1d):
                m.eval()
    with torch.no_grad():
        return np.stack([model(x).cpu().numpy() for _ in range(T)])


def de_reference(models, x, batch_size=32):
    outs = []
    with torch.no_grad():
        for m in models:
            m.eval()
            outs.append(torch.cat([m(x[i:i + batch_size]) for i in range(0, x.shape[0], batch_size)]).cpu().numpy())
    return np.stack(outs)


def uq_host(preds, y):
    return M.aggregates(M.per_window(preds), y)


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--n", type=int, default=16384)
    ap.add_argument("--passes", type=int, default=50)
    ap.add_argument("--members", type=int, default=8)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--bn-mode", choices=["batch", "running"], default="batch")
    ap.add_argument("--device", default="cuda" if torch.cuda.is_available() else "cpu")
    ap.add_argument("--seed", type=int, default=2025)
    a = ap.parse_args(argv)
    dev = torch.device(a.device)
    if dev.type == "cpu":
        torch.set_num_threads(max(1, torch.get_num_threads()))
    g = torch.Generator().manual_seed(a.seed)
    x = torch.randn(a.n, 60, 4, generator=g).to(dev)
    y = (torch.rand(a.n, generator=g) < 0.3).numpy().astype(np.int64)
    mcd_model = EagerCNN().load_keras(synthetic_params(a.seed)).to(dev)
    members = [EagerCNN().load_keras(synthetic_params(a.seed + 100 + m)).to(dev) for m in range(a.members)]

    def step():
        t = [time.perf_counter()]
        pm = mcd_reference(mcd_model, x, a.passes, a.bn_mode)
        t.append(time.perf_counter())
        am = uq_host(pm, y)
        t.append(time.perf_counter())
        pd = de_reference(members, x)
        t.append(time.perf_counter())
        ad = uq_host(pd, y)
        t.append(time.perf_counter())
        return np.diff(t), am, ad

    step()  # warmup (MIOpen kernel selection, allocator)
    _sync(dev)
    parts = np.zeros(4)
    for _ in range(a.steps):
        d, am, ad = step()
        parts += d
    parts /= a.steps
    total = parts.sum()
    res = {
        "what": "reference-semantics eager fp32 comparator (our measurement; the reference publishes none)",
        "device": torch.cuda.get_device_name(dev) if dev.type == "cuda" else "cpu",
        "n_windows": a.n, "passes": a.passes, "members": a.members, "bn_mode_mcd": a.bn_mode, "dtype": "fp32",
        "windows_per_s": a.n / total,
        "step_s": total,
        "mcd_forward_s": parts[0], "mcd_metrics_s": parts[1], "de_forward_s": parts[2], "de_metrics_s": parts[3],
        "mcd_windows_per_s": a.n / (parts[0] + parts[1]), "de_windows_per_s": a.n / (parts[2] + parts[3]),
        "mcd_mean_entropy": am["mean_total_pred_entropy"], "de_mean_mutual_info": ad["mean_mutual_info"],
    }
    print(json.dumps(res), flush=True)
    return res


if __name__ == "__main__":
    main()
