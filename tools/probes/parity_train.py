"""bf16 HIP vs fp32 torch training trajectories on the noisy synthetic apnea set (diagnostic)."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from uncertaintyquantification_sleepapnea_1dcnn_amd.data.synthetic import synthetic_windows  # noqa: E402
from uncertaintyquantification_sleepapnea_1dcnn_amd.models.cnn import AlarconCNN1D  # noqa: E402

n, epochs, noise = int(sys.argv[1]), int(sys.argv[2]), float(sys.argv[3])
x, y, _ = synthetic_windows(n, seed=2025)
rs = np.random.RandomState(2025)
x = (x + rs.randn(*x.shape).astype(np.float32) * noise).astype(np.float32)
x = (x - x.mean(1, keepdims=True)) / (x.std(1, keepdims=True) + 1e-8)
for seed in (2025, 7):
    for backend in ("hip", "torch"):
        os.environ["APNEAUQ_TRAIN_BACKEND"] = backend
        m = AlarconCNN1D(seed=seed, device="cuda")
        h = m.fit(x, y.astype(np.float32), batch_size=1024, epochs=epochs, validation_split=0.1, verbose=0)
        print(json.dumps({"seed": seed, "backend": backend, "val_loss": [round(v, 4) for v in h.history["val_loss"]],
                          "val_auc": [round(v, 4) for v in h.history["val_auc"]],
                          "loss": [round(v, 4) for v in h.history["loss"]]}), flush=True)
