"""Probe: can two ranks share one GPU in an RCCL communicator on this box?"""
import os, torch, torch.distributed as dist
dist.init_process_group("nccl")
r = dist.get_rank()
torch.cuda.set_device(0)
t = torch.full((1 << 20,), float(r + 1), device="cuda:0", dtype=torch.float64)
dist.all_reduce(t)
torch.cuda.synchronize()
print("rank", r, "allreduce ok", float(t[0]), flush=True)
dist.destroy_process_group()
