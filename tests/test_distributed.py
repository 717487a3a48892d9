"""Multi-process (world_size 2, gloo, CPU) test of the trial sharding and the
single count reduction used on GPUs (RCCL).  The per-rank engine here is the C
oracle (CPU); the sharding/reduction code is the product's
(distributed.run_sharded), the same function run_experiment uses on GPUs."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, out_path):
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from __graft_entry__ import load_package
    from oracle import c_oracle as C
    pkg = load_package()
    from dccvm_amd.distributed import run_sharded, run_sharded_grid, pd_rows  # noqa: F401
    cc = pkg.CONFIG_CODES["m2"]
    c1, c2 = C.Code(cc["gen1"], 2, 1, 2), C.Code(cc["gen2"], 2, 1, 2)
    models = {}

    def count_fn(iN, N, ip, p, lo, hi, out):
        if p not in models:
            models[p] = C.Model(c1, p, None, 200, 1.0, 7)
        cnt, _ = models[p].run_trials(c1, c2, N, p, 7, lo, hi, nthreads=1)
        out += torch.from_numpy(cnt)

    counts = run_sharded(count_fn, [60, 120], [0.02, 0.1], 101, torch.device("cpu"))

    def grid_fn(lo, hi, out):     # the grid form run_experiment uses (one call per rank)
        for iN, N in enumerate([60, 120]):
            for ip, p in enumerate([0.02, 0.1]):
                count_fn(iN, N, ip, p, lo, hi, out[iN, ip])

    grid = run_sharded_grid(grid_fn, [60, 120], [0.02, 0.1], 101, torch.device("cpu"))
    if rank == 0:
        np.save(out_path, np.stack([counts.numpy(), grid.numpy()]))
    dist.destroy_process_group()


def test_shard_covers_range(pkg):
    from dccvm_amd.distributed import shard
    for T in (0, 1, 7, 101, 1000):
        for W in (1, 2, 3, 8):
            blocks = [shard(T, r, W) for r in range(W)]
            assert blocks[0][0] == 0 and blocks[-1][1] == T
            assert all(blocks[i][1] == blocks[i + 1][0] for i in range(W - 1))


@pytest.mark.parametrize("world", [2])
def test_sharded_counts_equal_single_process(pkg, tmp_path, world):
    from oracle import c_oracle as C
    out = str(tmp_path / "counts.npy")
    mp.start_processes(_worker, args=(world, _free_port(), out), nprocs=world, join=True,
                       start_method="spawn")
    both = np.load(out)
    assert np.array_equal(both[0], both[1])          # run_sharded == run_sharded_grid
    got = both[0]
    cc = pkg.CONFIG_CODES["m2"]
    c1, c2 = C.Code(cc["gen1"], 2, 1, 2), C.Code(cc["gen2"], 2, 1, 2)
    for iN, N in enumerate([60, 120]):
        for ip, p in enumerate([0.02, 0.1]):
            mod = C.Model(c1, p, None, 200, 1.0, 7)
            cnt, _ = mod.run_trials(c1, c2, N, p, 7, 0, 101, nthreads=2)
            assert got[iN, ip].tolist() == cnt.tolist()


def _reduce_worker(rank, world, port, out_path):
    """bench.reduce_record on gloo ranks: the true reduce passes, a corrupted one raises."""
    import json
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    shard = torch.tensor([[rank + 1, 10 * rank], [7, rank]], dtype=torch.int64)
    red = shard.clone()
    dist.all_reduce(red)
    rec = bench.reduce_record(dist, shard, red, world, rank, "test")
    bad = red.clone()
    bad[0, 0] += 1                      # a reduce that lost or doubled a shard
    try:
        bench.reduce_record(dist, shard, bad, world, rank, "test")
        raised = False
    except RuntimeError:
        raised = True
    if rank == 0:
        with open(out_path, "w") as f:
            json.dump({"rec": rec, "raised": raised, "red": red.tolist()}, f)
    dist.destroy_process_group()


def test_bench_reduce_record_checks_the_reduce(tmp_path):
    import json
    out = str(tmp_path / "rec.json")
    mp.start_processes(_reduce_worker, args=(2, _free_port(), out), nprocs=2, join=True, start_method="spawn")
    got = json.load(open(out))
    rec = got["rec"]
    assert rec["world_size"] == 2 and rec["backend"] == "gloo" and rec["shards_sum_equals_reduced"]
    assert rec["rank_shards"] == [[[1, 0], [7, 0]], [[2, 10], [7, 1]]]
    assert got["red"] == [[3, 10], [14, 1]]
    assert got["raised"]
