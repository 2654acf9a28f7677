"""Probe: can two ranks on ONE GPU form a direct RCCL communicator (rehearsal of the
multi-rank RcclGradAllReduce path on a 1-GPU box)?  gloo is the control plane."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
dist.init_process_group("gloo", rank=rank, world_size=world)
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
from apex_amd.parallel.rccl import RcclComm, RcclGradAllReduce  # noqa: E402

try:
    ar = RcclGradAllReduce(dev)
except Exception as e:  # noqa: BLE001
    print(f"rank {rank}: comm init failed: {e}", flush=True)
    sys.exit(3)
t = torch.full((1 << 20,), float(rank + 1), device=dev)
w = ar.start(t)
ar.wait(w)
torch.cuda.synchronize()
print(f"rank {rank}: all_reduce ok, value {t[0].item()} (expect {world * (world + 1) / 2})", flush=True)
dist.destroy_process_group()
