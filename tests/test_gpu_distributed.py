"""Multi-GPU path on the one-GPU box: RCCL itself (the C-ABI's collective at world 1
and a torch.distributed "nccl" group at world 1), the trial sharding of the GPU
engine under 2 ranks (gloo, both ranks on the one device), and bench.py's own
rank launcher (--gpus 2)."""
import ctypes
import json
import os
import socket
import subprocess
import sys

import pytest
import torch

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_rccl_allreduce_counts_one_device(pkg):
    """cvd_allreduce_counts (ncclCommInitAll + grouped ncclAllReduce) at ndev = 1."""
    from dccvm_amd.distributed import allreduce_counts
    t = torch.tensor([[3, 5], [7, 11], [0, 1 << 40]], dtype=torch.int64, device="cuda:0")
    want = t.clone()
    allreduce_counts([t])
    assert torch.equal(t, want)
    allreduce_counts([t.view(-1)])          # second call: cached communicator
    assert torch.equal(t, want)


def test_rccl_comm_world_one(pkg):
    """cvd_comm_unique_id -> cvd_comm_init (1 rank) -> cvd_comm_allreduce_counts."""
    L = pkg.lib()
    uid = ctypes.create_string_buffer(128)
    pkg._lib.check(L.cvd_comm_unique_id(uid))
    comm = ctypes.c_void_p()
    pkg._lib.check(L.cvd_comm_init(uid, 1, 0, 0, ctypes.byref(comm)))
    try:
        t = torch.tensor([1, 2, 3, 4], dtype=torch.int64, device="cuda:0")
        s = torch.cuda.current_stream()
        pkg._lib.check(L.cvd_comm_allreduce_counts(comm, ctypes.c_void_p(t.data_ptr()), 4,
                                                   ctypes.c_void_p(s.cuda_stream)))
        torch.cuda.synchronize()
        assert t.cpu().tolist() == [1, 2, 3, 4]
    finally:
        L.cvd_comm_destroy(comm)


def test_nccl_group_world_one_run_experiment(tmp_path):
    """run_experiment under a torch.distributed "nccl" (RCCL) group of one rank: the
    count all_reduce runs over RCCL and the table equals the no-group run."""
    out = tmp_path / "nccl1.json"
    subprocess.run([sys.executable, os.path.join(ROOT, "tests", "dist_worker.py"), "nccl1", str(out)],
                   check=True, timeout=300)
    r = json.load(open(out))
    assert r["rccl"] == r["single"]
    assert r["allreduce"] == list(range(6))
    assert any(0.0 < row["Pd"] < 1.0 for row in r["single"])


def test_gloo_two_ranks_gpu_engine(pkg, tmp_path):
    """Two ranks (gloo) share the one GPU; each runs run_experiment on its trial shard of
    the GPU engine; the all-reduced table equals the single-process table."""
    out = tmp_path / "gloo2.json"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
           os.path.join(ROOT, "tests", "dist_worker.py"), "gloo2", str(out)]
    subprocess.run(cmd, check=True, timeout=300)
    r = json.load(open(out))
    assert r["world"] == 2
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import dist_worker
    assert r["rows"] == dist_worker.run(pkg)


def test_bench_launches_its_own_ranks(tmp_path):
    """`bench.py --gpus 2` without a launcher starts two ranks itself (gloo, both on the
    one GPU): n_gpus = 2, and the counts equal one rank running twice the steps (the same
    global trial ids at one p)."""
    env = dict(os.environ, CVD_BENCH_ONE_DEVICE="1")
    env.pop("WORLD_SIZE", None)
    common = ["--config", "m2", "--N", "1000", "--batch", "65536", "--warmup", "0", "--p", "0.092",
              "--cpu-baseline", "0"]
    two = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dist-backend", "gloo",
                          "--steps", "2", *common], timeout=300, capture_output=True, text=True, env=env)
    assert two.returncode == 0, two.stderr[-4000:]
    one = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--steps", "4", *common],
                         timeout=300, capture_output=True, text=True, env=env)
    assert one.returncode == 0, one.stderr[-4000:]
    j2 = json.loads([ln for ln in two.stdout.splitlines() if ln.startswith("{")][-1])
    j1 = json.loads([ln for ln in one.stdout.splitlines() if ln.startswith("{")][-1])
    assert j2["n_gpus"] == 2 and j1["n_gpus"] == 1
    assert j2["diagnostic"]["per_p"] == j1["diagnostic"]["per_p"]
    bad = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", *common],
                         timeout=120, capture_output=True, text=True, env=dict(env, WORLD_SIZE="1"))
    assert bad.returncode != 0


def test_bench_c4_counts_rank_invariant():
    """`bench.py --config c4` (BASELINE configs[4]: the m6 pair over an N grid x the p grid,
    a fixed total of trials split evenly over the grid points, every step of every trial,
    one count all_reduce): two ranks (gloo, both on the one GPU) give exactly the counts of
    one rank, since the streams are keyed by the global trial id."""
    env = dict(os.environ, CVD_BENCH_ONE_DEVICE="1")
    env.pop("WORLD_SIZE", None)
    common = ["--config", "c4", "--c4-trials", "4800", "--c4-N", "1000,10000", "--learn-len", "100000",
              "--cpu-baseline", "0"]
    two = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dist-backend", "gloo",
                          *common], timeout=300, capture_output=True, text=True, env=env)
    assert two.returncode == 0, two.stderr[-4000:]
    one = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *common],
                         timeout=300, capture_output=True, text=True, env=env)
    assert one.returncode == 0, one.stderr[-4000:]
    j2 = json.loads([ln for ln in two.stdout.splitlines() if ln.startswith("{")][-1])
    j1 = json.loads([ln for ln in one.stdout.splitlines() if ln.startswith("{")][-1])
    assert j2["n_gpus"] == 2 and j1["n_gpus"] == 1 and j1["scaling"] == "strong"
    assert j1["config"]["total_trials"] == 4800 and set(j1["per_N"]) == {"1000", "10000"}
    assert j2["counts"] == j1["counts"]
    assert sum(c[0] + c[1] for row in j1["counts"] for c in row) > 0
