"""Deep Ensembles across GPUs: member-parallel training and inference.

Training replaces the reference's sequential member loop (``train_deep_ensemble_cnns.py:125-177``):

* **ensemble parallel** (default, ``world <= M``): member m trains on rank ``m % world`` with seed
  ``seed_base + m``; no communication at all;
* **ensemble x data parallel** (``world > M`` and ``world % M == 0``): member m trains on the
  ``world/M`` ranks of its group (``parallel/data_parallel.py``: SyncBN + one gradient bucket);
* **resume** at member granularity: a member whose checkpoint exists is skipped (the reference's
  skip-if-exists, ``:130-132``) — a killed job rerun retrains only the missing members; checkpoints
  are written atomically (tmp + rename) so a crash never leaves a half-written member;
* **concurrent members**: the members one rank owns (``world < M``) train at the same time
  (``training/trainer.py:fit_concurrent``; a batch-1024 step fills only part of the GPU): each round
  of optimizer steps is ONE member-batched HIP graph whose layer kernels cover all members
  (``ops/train_ops.py:GraphedEnsembleStep``, XCD-aware member placement), or, where that does not
  apply, the members' steps overlap on HIP streams; then they are saved in member order;
* **resume** at epoch granularity inside a member (``epoch_backup``): a per-member
  ``BackupAndRestore`` file holds weights + Adam state + epoch, so a member killed mid-training
  continues from its last finished epoch (fault sites for tests: ``utils/faults.py``).

Checkpoint names keep the reference's scheme ``{prefix}{name_offset + i}.keras``
(``AlCNN_smote_seed{21+i}``); :func:`load_ensemble` takes the loaders' offsets (``i+5`` in
``analyze_de_patient_level.py:45``, ``i`` in ``evaluate_de_global.py:29``).
"""
from __future__ import annotations

import os
from typing import List, Optional, Sequence

import numpy as np
import torch
import torch.distributed as dist

from ..utils.faults import maybe_fail
from ..models.cnn import AlarconCNN1D, load_model
from ..training.callbacks import BackupAndRestore, EarlyStopping
from ..training.trainer import fit_concurrent
from . import dist as pdist
from .data_parallel import DPContext

MODEL_PREFIX = "AlCNN_smote_seed"


def member_path(save_dir: str, i: int, prefix: str = MODEL_PREFIX, name_offset: int = 21) -> str:
    return os.path.join(save_dir, f"{prefix}{name_offset + i}.keras")


def plan(num_models: int, world: int) -> List[List[int]]:
    """Ranks assigned to each member."""
    if world > num_models and world % num_models == 0:
        per = world // num_models
        return [list(range(m * per, (m + 1) * per)) for m in range(num_models)]
    return [[m % world] for m in range(num_models)]


def train_ensemble(x_train, y_train, num_models: int = 5, seed_base: int = 2025, save_dir: str = "./models/ensemble_cnn_no_pool",
                   prefix: str = MODEL_PREFIX, name_offset: int = 21, epochs: int = 50, batch_size: int = 1024,
                   patience: int = 5, validation_split: float = 0.1, verbose: int = 2, resume: bool = True,
                   device=None, input_shape: Optional[Sequence[int]] = None, epoch_backup: bool = True,
                   extra_callbacks: Optional[Sequence] = None, concurrent: Optional[bool] = None) -> List[str]:
    """Train the members this rank owns; ``concurrent`` (default: on a GPU) trains them together
    (member-batched launches, or HIP streams)."""
    info = pdist.init()
    world, rank = info.world, info.rank
    groups = plan(num_models, world)
    pgroups = []
    if world > 1:
        for ranks in groups:  # every rank must create every group (collective)
            pgroups.append(dist.new_group(ranks) if len(ranks) > 1 else None)
    else:
        pgroups = [None] * num_models
    dev = device if device is not None else info.device
    os.makedirs(save_dir, exist_ok=True)
    shape = tuple(input_shape) if input_shape is not None else tuple(np.asarray(x_train).shape[1:])
    paths = []
    jobs = []  # (member, ranks, model, callbacks) this rank trains
    for m, ranks in enumerate(groups):
        path = member_path(save_dir, m, prefix, name_offset)
        paths.append(path)
        if rank not in ranks:
            continue
        if resume and os.path.exists(path):
            if verbose:
                print(f"\n--- Model {m + 1}/{num_models} (Seed: {seed_base + m}) already exists. Skipping training. ---")
            continue
        model = AlarconCNN1D(input_shape=shape, seed=seed_base + m, device=dev)
        if len(ranks) > 1:
            model.dp = DPContext(pgroups[m], len(ranks), ranks.index(rank))
        es = EarlyStopping(monitor="val_loss", patience=patience, restore_best_weights=True)
        cbs = [es] + list(extra_callbacks or [])
        if epoch_backup:  # a member killed mid-training resumes at its last finished epoch
            cbs.append(BackupAndRestore(os.path.join(save_dir, ".backup_" + os.path.splitext(os.path.basename(path))[0])))
        jobs.append((m, ranks, model, cbs))
    if concurrent is None:
        concurrent = torch.device(dev).type == "cuda"
    together = [j for j in jobs if len(j[1]) == 1] if concurrent else []
    if len(together) > 1:
        if verbose:
            print(f"\n--- Training Models {[j[0] + 1 for j in together]} concurrently on rank {rank} ---")
        hists = fit_concurrent([j[2] for j in together], x_train, y_train, callbacks=[j[3] for j in together],
                               epochs=epochs, batch_size=batch_size, validation_split=validation_split,
                               verbose=verbose)
        done = {j[0]: h for j, h in zip(together, hists)}
    else:
        done = {}
    for m, ranks, model, cbs in jobs:
        if m in done:
            hist = done[m]
        else:
            if verbose:
                print(f"\n--- Training Model {m + 1}/{num_models} (Seed: {seed_base + m}) on ranks {ranks} ---")
            hist = model.fit(x_train, y_train, epochs=epochs, batch_size=batch_size, validation_split=validation_split,
                             callbacks=cbs, verbose=verbose if ranks.index(rank) == 0 else 0)
        maybe_fail("ensemble.before_save", member=m)
        if ranks.index(rank) == 0:
            model.save(paths[m])
            if verbose:
                print(f"Model {m + 1} saved successfully (Trained for {len(hist.history.get('loss', []))} epochs).")
    pdist.barrier()
    return paths


def load_ensemble(model_dir: str, pattern: str = MODEL_PREFIX + "{}.keras", num_members: int = 5, offset: int = 5,
                  device=None) -> List[AlarconCNN1D]:
    """Load ``pattern.format(i + offset)`` for i < num_members (reference loader conventions)."""
    models = []
    for i in range(num_members):
        p = os.path.join(model_dir, pattern.format(i + offset))
        models.append(load_model(p, device=device))
    if len(models) != num_members:
        raise ValueError(f"Expected {num_members} models, but only loaded {len(models)}")
    return models


def load_ensemble_prefix(model_prefix: str, num_models: int, device=None) -> List[AlarconCNN1D]:
    """``evaluate_de_global.py`` convention: ``{prefix}{i}.keras`` for i < num_models."""
    return [load_model(f"{model_prefix}{i}.keras", device=device) for i in range(num_models)]
