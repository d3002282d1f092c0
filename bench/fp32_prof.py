"""Short fp32-path loop for kernel traces: ``python -m bench.fp32_prof --mode de|mcd_batch|mcd_running|train``
(pooled CNN, 16384 windows; Deep Ensemble of 8 members or MC Dropout T=50, precision="fp32"; ``train``:
30 batch-1024 steps of the reference CNN at train_precision="fp32")."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", default="de")
    ap.add_argument("--reps", type=int, default=2)
    a = ap.parse_args()
    import torch

    from bench.fp32_micro import POOLED
    from uncertaintyquantification_sleepapnea_1dcnn_amd.models.cnn import AlarconCNN1D
    from uncertaintyquantification_sleepapnea_1dcnn_amd.uq import uq_techniques as U

    x = torch.randn(16384, 60, 4, generator=torch.Generator().manual_seed(0)).cuda()
    if a.mode == "train":
        y = (torch.rand(1024, generator=torch.Generator().manual_seed(1)) > 0.5).float().cuda()
        m = AlarconCNN1D(seed=3, device="cuda", train_precision="fp32")
        for _ in range(30):
            m.train_step(x[:1024], y)
        torch.cuda.synchronize()
        print("done", a.mode)
        return
    ms = [AlarconCNN1D(spec=POOLED, seed=10 + i, device="cuda", precision="fp32") for i in range(8)]
    for _ in range(a.reps):
        if a.mode == "de":
            U.deep_ensembles_predict(ms, x, as_numpy=False)
        else:
            U.mc_dropout_predict(ms[0], x, n_pred=50, bn_mode=a.mode.split("_")[1], seed=1, as_numpy=False)
    torch.cuda.synchronize()
    print("done", a.mode)


if __name__ == "__main__":
    main()
