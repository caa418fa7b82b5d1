"""RCCL on one GPU of the box (not part of the tests): torch.distributed's nccl backend with one
rank, then the library's one-rank RCCL context (MIGMRES_FORCE_RCCL=1)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
which = sys.argv[1] if len(sys.argv) > 1 else "torch"
if which == "torch":
    import torch
    import torch.distributed as dist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29511")
    dist.init_process_group("nccl", rank=0, world_size=1)
    t = torch.ones(4, device="cuda:0")
    dist.all_reduce(t)
    torch.cuda.synchronize()
    print("torch nccl all_reduce ok", t.tolist(), flush=True)
    dist.destroy_process_group()
else:
    if which == "torch_then_lib":
        import torch
        torch.cuda.is_available()
    os.environ["MIGMRES_FORCE_RCCL"] = "1"
    import numpy as np
    import trilinos_amd as ta
    c = ta.Comm(device=0)
    print("migmres one-rank RCCL ok", c.sum_all(np.array([1.0, 2.0])).tolist(), flush=True)
# python tools/rccl_probe.py torch_then_lib: torch imported (and its HIP initialised) first
