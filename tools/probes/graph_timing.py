import time, torch, os, json
from uncertaintyquantification_sleepapnea_1dcnn_amd.models.cnn import AlarconCNN1D
from uncertaintyquantification_sleepapnea_1dcnn_amd.ops import train_ops
res = {}
for b in (128, 1024):
    m = AlarconCNN1D(seed=1, device="cuda")
    x = torch.randn(b, 60, 4, device="cuda"); y = (torch.rand(b, device="cuda") > 0.5).float()
    g = train_ops.GraphedTrainStep(m, b)
    for _ in range(3): g(x, y)
    torch.cuda.synchronize(); t = time.perf_counter()
    for _ in range(50): g.graph.replay()
    torch.cuda.synchronize(); res[f"replay_only_b{b}_ms"] = (time.perf_counter() - t) / 50 * 1e3
    os.environ["APNEAUQ_TRAIN_GRAPH"] = "0"
    for _ in range(3): m.train_step(x, y)
    torch.cuda.synchronize(); t = time.perf_counter()
    for _ in range(50): m.train_step(x, y)
    torch.cuda.synchronize(); res[f"eager_b{b}_ms"] = (time.perf_counter() - t) / 50 * 1e3
    os.environ["APNEAUQ_TRAIN_GRAPH"] = "1"
print(json.dumps(res))
