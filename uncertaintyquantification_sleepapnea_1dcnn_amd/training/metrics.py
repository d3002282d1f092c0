"""Keras-semantics training metrics: loss mean, binary accuracy and the 200-threshold AUC.

``model.compile(metrics=['accuracy', tf.keras.metrics.AUC(name='auc')])``
(``cnn_baseline_train.py:100-102``).  Keras ``AUC()`` defaults: 200 thresholds
``[-1e-7, 1/199, ..., 198/199, 1+1e-7]``, ROC curve, ``summation_method='interpolation'`` —
confusion counts at every threshold accumulated over the epoch, then the trapezoidal area.
On the GPU both metrics accumulate into device-resident int64 counters with one launch of the
K10 kernel per batch (``csrc/metrics.hip``: accuracy count + the 2 x 201 threshold-bucket
histograms), so an epoch's training loop never synchronises with the host for metrics; the
counters are read once when the result is needed (``flush``).  Elsewhere the same buckets come
from ``torch.bucketize`` + ``bincount``.
"""
from __future__ import annotations

import numpy as np
import torch

NUM_THRESHOLDS = 200


def keras_thresholds(num: int = NUM_THRESHOLDS) -> np.ndarray:
    eps = 1e-7
    inner = [(i + 1) * 1.0 / (num - 1) for i in range(num - 2)]
    return np.array([0.0 - eps] + inner + [1.0 + eps], dtype=np.float64)


def _device_counts(p: torch.Tensor, y: torch.Tensor, thr: torch.Tensor, counts):
    """Add one batch into the K10 device counters (allocated on first use); None if no HIP path."""
    if not p.is_cuda:
        return None
    from ..ops import _ext

    if not _ext.available():
        return None
    if counts is None:
        counts = torch.zeros(1 + 2 * (thr.numel() + 1), dtype=torch.int64, device=p.device)
    _ext.ops().metrics_update(p.reshape(-1).float().contiguous(), y.reshape(-1).float().contiguous(), thr, counts)
    return counts


class MeanMetric:
    def __init__(self):
        self.total = 0.0
        self.count = 0.0

    def update(self, value_sum: float, weight: float) -> None:
        self.total += float(value_sum)
        self.count += float(weight)

    def result(self) -> float:
        return self.total / self.count if self.count else 0.0


class BinaryAccuracy(MeanMetric):
    _THR = {}

    def __init__(self):
        super().__init__()
        self._counts = None

    def update_state(self, y: torch.Tensor, p: torch.Tensor) -> None:
        if p.is_cuda:
            thr = self._THR.get(p.device)
            if thr is None:
                thr = self._THR[p.device] = torch.tensor([0.5], dtype=torch.float32, device=p.device)
            c = _device_counts(p, y, thr, self._counts)
            if c is not None:
                self._counts = c
                self.count += float(y.numel())
                return
        correct = ((p.reshape(-1) > 0.5).float() == (y.reshape(-1) > 0.5).float()).float().sum()
        self.update(correct.item(), y.numel())

    def flush(self) -> None:
        """Move the device counter into ``total`` (one host read)."""
        if self._counts is not None:
            self.total += float(self._counts[0].item())
            self._counts = None

    def result(self) -> float:
        self.flush()
        return super().result()


class AUC:
    """Streaming ROC AUC with Keras' threshold set and interpolation rule."""

    def __init__(self, num_thresholds: int = NUM_THRESHOLDS):
        self.thresholds = keras_thresholds(num_thresholds)
        self._thr_t = {}
        self.reset_state()

    def reset_state(self) -> None:
        n = len(self.thresholds)
        self.pos_hist = np.zeros(n + 1, dtype=np.float64)
        self.neg_hist = np.zeros(n + 1, dtype=np.float64)
        self._counts = None

    def update_state(self, y: torch.Tensor, p: torch.Tensor) -> None:
        dev = p.device
        thr = self._thr_t.get(dev)
        if thr is None:
            thr = torch.tensor(self.thresholds, dtype=torch.float32, device=dev)
            self._thr_t[dev] = thr
        c = _device_counts(p, y, thr, self._counts)
        if c is not None:
            self._counts = c
            return
        p = p.reshape(-1).float()
        y = y.reshape(-1)
        # bucket b = number of thresholds strictly below p  (pred > thr  <=>  thr < p)
        b = torch.bucketize(p, thr, right=False)
        n = len(self.thresholds) + 1
        pos = torch.bincount(b[y > 0.5], minlength=n).double().cpu().numpy()
        neg = torch.bincount(b[y <= 0.5], minlength=n).double().cpu().numpy()
        self.pos_hist += pos
        self.neg_hist += neg

    def flush(self) -> None:
        """Move the device histograms into ``pos_hist`` / ``neg_hist`` (one host read)."""
        if self._counts is not None:
            h = self._counts.cpu().numpy().astype(np.float64)
            nb = self.pos_hist.size
            self.pos_hist += h[1: 1 + nb]
            self.neg_hist += h[1 + nb:]
            self._counts = None

    def confusion(self):
        self.flush()
        # tp[i] = #positives with pred > thr[i] = sum of buckets b > i
        pos_gt = np.cumsum(self.pos_hist[::-1])[::-1]
        neg_gt = np.cumsum(self.neg_hist[::-1])[::-1]
        tp = pos_gt[1:]
        fp = neg_gt[1:]
        fn = self.pos_hist.sum() - tp
        tn = self.neg_hist.sum() - fp
        return tp, fp, tn, fn

    def result(self) -> float:
        tp, fp, tn, fn = self.confusion()
        with np.errstate(divide="ignore", invalid="ignore"):
            tpr = np.where(tp + fn > 0, tp / (tp + fn), 0.0)
            fpr = np.where(fp + tn > 0, fp / (fp + tn), 0.0)
        heights = (tpr[:-1] + tpr[1:]) / 2.0
        return float(np.sum((fpr[:-1] - fpr[1:]) * heights))


def bce_from_logits(logits: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
    """Per-sample binary cross-entropy on logits (Keras' sigmoid-output logits path)."""
    return torch.nn.functional.binary_cross_entropy_with_logits(logits.reshape(-1), y.reshape(-1).float(),
                                                                reduction="none")
