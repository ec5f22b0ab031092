"""Probe: can two ranks share the box's one GPU over RCCL (backend "nccl")?  Each rank all-gathers a small tensor
holding its rank; rank 0 prints the result.  (NCCL refuses duplicate devices; this checks RCCL's behaviour here.)"""
import os
import sys

import torch
import torch.distributed as dist


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", 0))
    x = torch.full((4,), float(rank), device="cuda")
    out = torch.empty(world * 4, device="cuda")
    dist.all_gather_into_tensor(out, x)
    torch.cuda.synchronize()
    ok = torch.equal(out.cpu(), torch.arange(world).repeat_interleave(4).float())
    print(f"rank {rank}: all_gather {'ok' if ok else 'WRONG'} {out.tolist()}", flush=True)
    dist.destroy_process_group()
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
