"""Probe: can two RCCL ranks share one GPU on this box?  (tiny all_reduce, prints the outcome)"""
import os
import torch
import torch.distributed as dist

dist.init_process_group("nccl", init_method="env://", device_id=torch.device("cuda", 0))
r = dist.get_rank()
x = torch.full((1 << 20,), float(r + 1), device="cuda:0")
dist.all_reduce(x)
torch.cuda.synchronize()
print(f"rank {r}: all_reduce ok, value {x[0].item()}", flush=True)
dist.destroy_process_group()
