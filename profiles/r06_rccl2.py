#!/usr/bin/env python3
"""Round 6: can two ranks share the one card of a 1-GPU box over RCCL (backend "nccl")?
Launched as  torchrun --nproc-per-node 2 --master-addr 127.0.0.1 profiles/r06_rccl2.py OUT.json
Each rank binds cuda:0, initialises the nccl process group and runs the detector's one
collective -- a SUM all_reduce of an int64 count tensor -- then rank 0 writes what happened."""
import json
import os
import sys
import time

import torch
import torch.distributed as dist


def main():
    out = sys.argv[1]
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    rec = {"rank": rank, "world": world, "device": torch.cuda.get_device_name(0)}
    t0 = time.time()
    try:
        dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
        x = torch.tensor([[rank + 1, 10 * (rank + 1)]], dtype=torch.int64, device="cuda:0")
        dist.all_reduce(x)
        torch.cuda.synchronize()
        rec["all_reduce"] = x.cpu().tolist()
        rec["expected"] = [[sum(r + 1 for r in range(world)), sum(10 * (r + 1) for r in range(world))]]
        rec["ok"] = rec["all_reduce"] == rec["expected"]
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001 -- the record says what RCCL refused
        rec["ok"] = False
        rec["error"] = f"{type(e).__name__}: {e}"[:2000]
    rec["seconds"] = time.time() - t0
    with open(f"{out}.rank{rank}", "w") as f:
        json.dump(rec, f)
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
