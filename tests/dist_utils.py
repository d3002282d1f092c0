"""Helpers to run a function on N CPU ranks with the gloo backend (127.0.0.1)."""
import os
import socket
import tempfile

import torch.multiprocessing as mp


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _entry(rank, world, port, fn, args, outdir, gpu=False):
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "RANK": str(rank),
                       "WORLD_SIZE": str(world), "LOCAL_RANK": "0" if gpu else str(rank)})
    if not gpu:
        os.environ["CUDA_VISIBLE_DEVICES"] = ""
    import torch

    torch.set_num_threads(2)
    from uncertaintyquantification_sleepapnea_1dcnn_amd.parallel import dist as pdist

    # gpu=True: every rank shares cuda:0 and talks gloo (RCCL needs one GPU per rank); exercises
    # the HIP paths of the sharded code on a 1-GPU box
    pdist.init(backend="gloo", device=None if gpu else "cpu")
    try:
        res = fn(rank, world, *args)
        torch.save(res, os.path.join(outdir, f"r{rank}.pt"))
    finally:
        pdist.shutdown()


def run_ranks(fn, world=2, args=(), gpu=False):
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_entry, args=(world, free_port(), fn, args, d, gpu), nprocs=world, join=True,
                           start_method="spawn")
        import torch

        return [torch.load(os.path.join(d, f"r{r}.pt"), weights_only=False) for r in range(world)]
