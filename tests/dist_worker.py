"""Worker of tests/test_gpu_distributed.py (run as its own process, one per rank).

  python tests/dist_worker.py nccl1 OUT.json     # world 1 over RCCL (init_method tcp)
  torchrun --nproc-per-node 2 tests/dist_worker.py gloo2 OUT.json   # 2 ranks, one GPU

Each runs the product's run_experiment on the GPU engine under a process group
(trial sharding + the one count all_reduce) and rank 0 writes the DataFrame rows."""
import json
import os
import socket
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from __graft_entry__ import load_package  # noqa: E402

CASE = dict(k=1, n=2, m=2, num_iter=3001, p_vec=[0.03, 0.1], learn_len=None, learn_burn=200, laplace=1.0,
            seed=7, N_list=[300, 1000])


def run(pkg):
    cc = pkg.CONFIG_CODES["m2"]
    df = pkg.run_experiment(CASE["k"], CASE["n"], CASE["m"], cc["gen1"], cc["gen2"], CASE["num_iter"],
                            CASE["p_vec"], CASE["learn_len"], CASE["learn_burn"], CASE["laplace"], CASE["seed"],
                            N_list=CASE["N_list"], device=0)
    return df.to_dict(orient="records")


def main():
    mode, out = sys.argv[1], sys.argv[2]
    pkg = load_package()
    if mode == "nccl1":
        torch.cuda.set_device(0)
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
        single = run(pkg)                       # no process group: no collective
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                                device_id=torch.device("cuda", 0))
        assert dist.get_backend() == "nccl"
        rows = run(pkg)                         # run_sharded all_reduces over RCCL at world 1
        t = torch.arange(6, dtype=torch.int64, device="cuda")
        dist.all_reduce(t)
        dist.destroy_process_group()
        json.dump({"single": single, "rccl": rows, "allreduce": t.cpu().tolist()}, open(out, "w"))
    elif mode == "gloo2":
        dist.init_process_group("gloo")
        rows = run(pkg)
        if dist.get_rank() == 0:
            json.dump({"rows": rows, "world": dist.get_world_size()}, open(out, "w"))
        dist.destroy_process_group()
    else:
        raise SystemExit(f"unknown mode {mode}")


if __name__ == "__main__":
    main()
