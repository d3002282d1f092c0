"""``model.fit`` with Keras 2.12 semantics on a device-resident dataset.

Reference behaviour reproduced (``cnn_baseline_train.py:204-217``, ``train_deep_ensemble_cnns.py:150-165``):

* ``validation_split`` takes the LAST fraction of the arrays *before* shuffling
  (``split_at = int(n * (1 - validation_split))``);
* the training part is reshuffled every epoch; batches of ``batch_size`` with a partial tail;
* per step: forward in training mode (dropout on, BN on batch statistics + moving-average update),
  BCE on logits averaged over the batch, backward, Keras Adam;
* epoch logs: ``loss`` (batch-size-weighted mean), ``accuracy``, ``auc`` (200 thresholds) and the
  same ``val_*`` on the validation slice in inference mode; ``verbose=2`` prints one line per epoch;
* callbacks (EarlyStopping with restore_best_weights, History).

The whole dataset is copied to the GPU once (288 GB HBM makes this trivially affordable) and
batches are gathered on device, so there is no host->device traffic inside the epoch loop.
"""
from __future__ import annotations

import time
from typing import List, Optional

import numpy as np
import torch

from ..utils.faults import maybe_fail
from .callbacks import Callback, History
from ..parallel.data_parallel import split_batch
from .metrics import AUC, BinaryAccuracy, MeanMetric


def _sync_metrics(dp, loss_acc: torch.Tensor, acc_m, auc_m) -> None:
    """Sum the epoch's per-rank metric state over the data-parallel group."""
    dev = loss_acc.device
    acc_m.flush()
    auc_m.flush()
    buf = torch.tensor([acc_m.total, acc_m.count], dtype=torch.float64, device=dev)
    hist = torch.tensor(np.concatenate([auc_m.pos_hist, auc_m.neg_hist]), dtype=torch.float64, device=dev)
    dp.all_reduce_(loss_acc)
    dp.all_reduce_(buf)
    dp.all_reduce_(hist)
    acc_m.total, acc_m.count = float(buf[0]), float(buf[1])
    k = auc_m.pos_hist.size
    h = hist.cpu().numpy()
    auc_m.pos_hist, auc_m.neg_hist = h[:k].copy(), h[k:].copy()


def _to_device(a, device, dtype=torch.float32) -> torch.Tensor:
    if isinstance(a, torch.Tensor):
        return a.to(device=device, dtype=dtype)
    return torch.as_tensor(np.asarray(a), dtype=dtype, device=device)


def evaluate_arrays(model, x: torch.Tensor, y: torch.Tensor, batch_size: int = 1024):
    """Inference-mode loss / accuracy / AUC over (x, y) (device tensors)."""
    loss_m, acc_m, auc_m = MeanMetric(), BinaryAccuracy(), AUC()
    n = x.shape[0]
    loss_sum = torch.zeros((), dtype=torch.float64, device=x.device)
    with torch.no_grad():
        for s in range(0, n, batch_size):
            xb, yb = x[s: s + batch_size], y[s: s + batch_size]
            logits = model.logits(xb, training=False)
            l = torch.nn.functional.binary_cross_entropy_with_logits(logits.reshape(-1), yb.float(), reduction="sum")
            p = torch.sigmoid(logits)
            loss_sum += l
            acc_m.update_state(yb, p)
            auc_m.update_state(yb, p)
    loss_m.update(loss_sum.item(), n)
    return loss_m.result(), acc_m.result(), auc_m.result()


def fit(model, x, y, batch_size: int = 32, epochs: int = 1, verbose: int = 1, callbacks: Optional[List[Callback]] = None,
        validation_split: float = 0.0, validation_data=None, shuffle: bool = True, seed: Optional[int] = None,
        initial_epoch: int = 0, grad_allreduce=None) -> History:
    """Keras ``model.fit`` semantics (``cnn_baseline_train.py:210-217``); runs :func:`fit_steps` to the end."""
    it = fit_steps(model, x, y, batch_size, epochs, verbose, callbacks, validation_split, validation_data, shuffle,
                   seed, initial_epoch, grad_allreduce)
    while True:
        try:
            next(it)
        except StopIteration as stop:
            return stop.value


def fit_concurrent(models: List, x, y, streams: Optional[List] = None, batched: Optional[bool] = None,
                   **fit_kwargs) -> List[History]:
    """Train several independent models (ensemble members sharing one GPU) at the same time.

    ``batched`` (default: whenever ``ops/train_ops.py:ensemble_supported``): every round, the live
    members' next optimizer steps run as ONE member-batched HIP graph (``GraphedEnsembleStep``: each
    layer kernel launched once for all members).  Otherwise each model's :func:`fit_steps` runs on
    its own HIP stream and the host round-robins one optimizer step per model, so the kernels of
    different members overlap on the device (``profiles/multistream_train_r1.json``).  Every model
    keeps its own data order, callbacks (EarlyStopping, BackupAndRestore) and epoch-end host
    synchronisation; results match sequential ``fit`` calls up to the summation order of fp32
    atomics.  ``fit_kwargs`` as for :func:`fit`; per-model ``callbacks`` may be given as a list of lists.
    """
    import contextlib

    cbs = fit_kwargs.pop("callbacks", None)
    per_cbs = cbs if (cbs and isinstance(cbs[0], (list, tuple))) else [cbs] * len(models)
    dev = models[0].device if models else torch.device("cpu")
    x, y = _to_device(x, dev), _to_device(y, dev)  # one device copy shared by every member
    if batched is None:
        from ..ops import train_ops

        batched = len(models) > 1 and train_ops.ensemble_supported(models) and \
            fit_kwargs.get("grad_allreduce") is None
    if batched:
        return _fit_batched(models, x, y, per_cbs, **fit_kwargs)
    if streams is None:
        # 3 streams + the default one fit HIP's 4 hardware queues per process (GPU_MAX_HW_QUEUES);
        # more streams share queues and measured no faster (profiles/multistream_train_r1.json)
        streams = [torch.cuda.Stream(device=dev) for _ in range(min(3, len(models)))] if dev.type == "cuda" else [None]
    cur = torch.cuda.current_stream(dev) if dev.type == "cuda" else None
    for s in streams:
        if s is not None:
            s.wait_stream(cur)  # inputs produced on the current stream
    ctx = [(torch.cuda.stream(streams[i % len(streams)]) if streams[i % len(streams)] is not None
            else contextlib.nullcontext()) for i in range(len(models))]
    gens = []
    for i, m in enumerate(models):
        with ctx[i]:
            gens.append(fit_steps(m, x, y, callbacks=per_cbs[i], **fit_kwargs))
    hist: List[Optional[History]] = [None] * len(models)
    live = list(range(len(models)))
    while live:
        for i in list(live):
            with ctx[i]:
                try:
                    next(gens[i])
                except StopIteration as stop:
                    hist[i] = stop.value
                    live.remove(i)
    for s in streams:
        if s is not None and cur is not None:
            cur.wait_stream(s)
    return hist


# member groups per batch size, one batched graph + HIP stream each (profiles/x3_epilogue_ab_r3.md); 2 since
# the persistent dgrad / 8-wave wgrad (8 members x batch 1024: 4 groups 3.90 ms, 2 groups 3.73-3.80, 1 group
# 3.83, 8 groups 4.23; tools/probes/train_groups.sh, profiles/train_step_r5.md)
ENSEMBLE_GROUPS = 2


def _fit_batched(models: List, x, y, per_cbs, **fit_kwargs) -> List[History]:
    """fit_concurrent's member-batched mode: the members' fit_steps generators hand their batches out
    (``external_step``); each round the live members of one batch size are split into up to
    ``APNEAUQ_ENSEMBLE_GROUPS`` (default ENSEMBLE_GROUPS) groups, each run as one GraphedEnsembleStep replayed on its
    own HIP stream (the groups' latency-bound phases overlap: round 3, 8 members 1.67 M -> 1.80 M windows/s
    with 4 groups of 2; round 5, 2 groups of 4 2.17 M).  A group's steps, gathers and metric updates all run
    on its stream: no joins."""
    import os

    from ..ops import train_ops

    n_groups = max(1, int(os.environ.get("APNEAUQ_ENSEMBLE_GROUPS", str(ENSEMBLE_GROUPS))))
    dev = models[0].device
    gens = [fit_steps(m, x, y, callbacks=per_cbs[i], external_step=True, **fit_kwargs) for i, m in enumerate(models)]
    hist: List[Optional[History]] = [None] * len(models)
    req = {}
    for i, g in enumerate(gens):
        try:
            req[i] = next(g)
        except StopIteration as stop:
            hist[i] = stop.value
    steps = {}
    step_stream = {}  # step key -> the stream of its last replay
    streams: List = []
    # every member's step, its next batch's gather and its metric updates run on its group's stream, so
    # the groups are never joined between steps; a member whose group (stream) changes -- regrouping
    # after an early stop, the tail batch -- first waits for the stream that ran its previous step
    home = torch.cuda.current_stream(dev)
    last = {i: home for i in range(len(models))}
    while req:
        live = sorted(req)
        by_n = {}
        for i in live:
            by_n.setdefault(int(req[i][0].shape[0]), []).append(i)
        # keep only the graphs of the live set's groupings (any batch size: the tail batch's graphs are
        # replayed every epoch): when a member stops early the live members are regrouped, and a step of
        # the old grouping (a workspace per member + a graph pool) would never be replayed again
        want = set()
        for ids in [live] + list(by_n.values()):
            ng = min(n_groups, len(ids))
            want.update(tuple(ids[g::ng]) for g in range(ng))
        for key in [k for k in steps if k[0] not in want]:
            # its last replay may still run on a group stream home never waited on, and its workspace /
            # counters were allocated on home: join before the allocator may hand them out again
            if key in step_stream:
                home.wait_stream(step_stream.pop(key))
            del steps[key]
        for n, ids in by_n.items():
            ng = min(n_groups, len(ids))
            subs = [ids[g::ng] for g in range(ng)]
            while len(streams) < ng:
                streams.append(torch.cuda.Stream(device=dev))
            for sub, s_ in zip(subs, streams):
                ms = [models[i] for i in sub]
                key = (tuple(sub), n)
                st = steps.get(key)
                if st is None or not st.valid_for(ms):
                    if key in step_stream:
                        home.wait_stream(step_stream.pop(key))
                    st = steps[key] = train_ops.GraphedEnsembleStep(ms, n)
                    s_.wait_stream(home)  # built and initialised on home (zeros, counters)
                for prev in {id(last[i]): last[i] for i in sub if last[i] is not s_}.values():
                    s_.wait_stream(prev)
                for i in sub:
                    if last[i] is not s_:  # a batch allocated on another stream, read on this one
                        req[i][0].record_stream(s_)
                        req[i][1].record_stream(s_)
                step_stream[key] = s_
                with torch.cuda.stream(s_):
                    outs = st([req[i][0] for i in sub], [req[i][1] for i in sub])
                    for i, res in zip(sub, outs):
                        last[i] = s_
                        try:
                            req[i] = gens[i].send(res)
                        except StopIteration as stop:
                            hist[i] = stop.value
                            del req[i]
    for s_ in streams:
        home.wait_stream(s_)
    return hist


def fit_steps(model, x, y, batch_size: int = 32, epochs: int = 1, verbose: int = 1,
              callbacks: Optional[List[Callback]] = None, validation_split: float = 0.0, validation_data=None,
              shuffle: bool = True, seed: Optional[int] = None, initial_epoch: int = 0, grad_allreduce=None,
              external_step: bool = False):
    """Generator form of :func:`fit`: yields after every optimizer step, returns the History.

    ``external_step``: instead of calling ``model.train_step`` the generator yields ``(xb, yb)`` and
    expects ``(loss_sum, probs)`` of that step to be sent back (member-batched ensemble training)."""
    dev = model.device
    X = _to_device(x, dev)
    Y = _to_device(y, dev)
    if validation_data is not None:
        Xv, Yv = _to_device(validation_data[0], dev), _to_device(validation_data[1], dev)
        Xt, Yt = X, Y
    elif validation_split and 0.0 < validation_split < 1.0:
        split_at = int(X.shape[0] * (1.0 - validation_split))
        Xt, Yt, Xv, Yv = X[:split_at], Y[:split_at], X[split_at:], Y[split_at:]
    else:
        Xt, Yt, Xv, Yv = X, Y, None, None
    n = Xt.shape[0]
    history = History()
    cbs = [history] + list(callbacks or [])
    for cb in cbs:
        cb.set_model(model)
    model.stop_training = False
    gen = torch.Generator(device="cpu")
    gen.manual_seed(int(model.seed if seed is None else seed))
    steps = (n + batch_size - 1) // batch_size
    model._resume_epoch = 0
    for cb in cbs:
        cb.on_train_begin()
    if model._resume_epoch > initial_epoch:  # BackupAndRestore found a backup
        for _ in range(initial_epoch, model._resume_epoch):
            if shuffle:
                torch.randperm(n, generator=gen)  # keep the batch order of an uninterrupted run
        initial_epoch = model._resume_epoch
    if verbose:
        print(f"Train on {n} samples" + (f", validate on {Xv.shape[0]} samples" if Xv is not None else ""))
    for epoch in range(initial_epoch, epochs):
        for cb in cbs:
            cb.on_epoch_begin(epoch)
        t0 = time.time()
        perm = torch.randperm(n, generator=gen).to(dev) if shuffle else torch.arange(n, device=dev)
        loss_m, acc_m, auc_m = MeanMetric(), BinaryAccuracy(), AUC()
        loss_acc = torch.zeros((), dtype=torch.float64, device=dev)
        dp = getattr(model, "dp", None)
        n_seen = 0
        for s in range(steps):
            gidx = perm[s * batch_size: (s + 1) * batch_size]
            if dp is not None and dp.size > 1 and gidx.numel() < dp.size:
                continue  # a tail batch smaller than the DP group is dropped on every rank
            idx, off = split_batch(gidx, dp)
            xb, yb = Xt.index_select(0, idx), Yt.index_select(0, idx)
            if external_step:
                loss_sum, p = yield (xb, yb)
            else:
                loss_sum, p = model.train_step(xb, yb, return_probs=True, grad_allreduce=grad_allreduce,
                                               dp_step=(int(gidx.numel()), off))
            loss_acc += loss_sum
            n_seen += int(gidx.numel())
            acc_m.update_state(yb, p)
            auc_m.update_state(yb, p)
            if not external_step:
                yield
        if dp is not None and dp.size > 1:
            _sync_metrics(dp, loss_acc, acc_m, auc_m)
        loss_m.update(loss_acc.item(), n_seen)
        logs = {"loss": loss_m.result(), "accuracy": acc_m.result(), "auc": auc_m.result()}
        if Xv is not None and Xv.shape[0] > 0:
            vl, va, vauc = evaluate_arrays(model, Xv, Yv, batch_size)
            logs.update({"val_loss": vl, "val_accuracy": va, "val_auc": vauc})
        dt = time.time() - t0
        if verbose:
            line = " - ".join(f"{k}: {v:.4f}" for k, v in logs.items())
            print(f"Epoch {epoch + 1}/{epochs}\n{steps}/{steps} - {dt:.0f}s - {line}", flush=True)
        for cb in cbs:
            cb.on_epoch_end(epoch, logs)
        maybe_fail("fit.epoch_end", epoch=epoch)
        if model.stop_training:
            break
    for cb in cbs:
        cb.on_train_end()
    history.params = {"epochs": epochs, "steps": steps, "batch_size": batch_size}
    return history
