"""Trial sharding over ranks and the one count reduction.

One process per GPU.  Every (N, p) grid point's global trial range
[0, num_iter) is split into contiguous per-rank blocks; because the trial
streams are keyed by the global trial id (Philox counter, see include/cvd.h),
the per-rank success counts add up to exactly the single-GPU counts for any
world size.  The only collective is one SUM all_reduce of the
[n_N, n_p, 2] int64 count tensor (RCCL over xGMI for CUDA/HIP tensors, gloo on
CPU), issued once after all grid points.
"""
import torch


def shard(num_trials, rank, world):
    """Contiguous block of global trial ids for `rank` (covers [0, num_trials) exactly)."""
    if world < 1 or not (0 <= rank < world):
        raise ValueError("bad rank/world")
    return num_trials * rank // world, num_trials * (rank + 1) // world


def dist_info():
    import torch.distributed as tdist
    if tdist.is_available() and tdist.is_initialized():
        return tdist.get_rank(), tdist.get_world_size()
    return 0, 1


def run_sharded(count_fn, N_list, p_vec, num_iter, device, rank=None, world=None):
    """counts[iN, ip, :] += count_fn(iN, N, ip, p, lo, hi, out) for this rank's
    trial block, then one all_reduce over the default process group (whenever one
    is initialised, world 1 included).  `count_fn` accumulates (s1, s2) into the
    2-element tensor `out` (device-side for the GPU engine)."""
    import torch.distributed as tdist
    r0, w0 = dist_info()
    rank = r0 if rank is None else rank
    world = w0 if world is None else world
    counts = torch.zeros((len(N_list), len(p_vec), 2), dtype=torch.int64, device=device)
    lo, hi = shard(num_iter, rank, world)
    for iN, N in enumerate(N_list):
        for ip, p in enumerate(p_vec):
            count_fn(iN, N, ip, p, lo, hi, counts[iN, ip])
    if tdist.is_available() and tdist.is_initialized():
        tdist.all_reduce(counts, op=tdist.ReduceOp.SUM)
    return counts


def run_sharded_grid(grid_fn, N_list, p_vec, num_iter, device, rank=None, world=None):
    """The same with the whole grid in one call: grid_fn(lo, hi, counts) accumulates this
    rank's trial block [lo, hi) of EVERY (N, p) point into counts[nN, np, 2] (e.g.
    Detector.run_grid, cvd_mc_run_grid), then one all_reduce."""
    import torch.distributed as tdist
    r0, w0 = dist_info()
    rank = r0 if rank is None else rank
    world = w0 if world is None else world
    counts = torch.zeros((len(N_list), len(p_vec), 2), dtype=torch.int64, device=device)
    lo, hi = shard(num_iter, rank, world)
    grid_fn(lo, hi, counts)
    if tdist.is_available() and tdist.is_initialized():
        tdist.all_reduce(counts, op=tdist.ReduceOp.SUM)
    return counts


def allreduce_counts(tensors, streams=None):
    """SUM-reduce int64 count tensors, one per device of this process, in place
    through the C-ABI's RCCL entry (cvd_allreduce_counts: ncclCommInitAll + one
    grouped ncclAllReduce) -- the multi-GPU route for callers without
    torch.distributed.  Synchronises the devices' streams before returning."""
    import ctypes
    from . import _lib
    n = len(tensors)
    if n == 0:
        return tensors
    length = tensors[0].numel()
    for t in tensors:
        if t.dtype != torch.int64 or not t.is_cuda or not t.is_contiguous() or t.numel() != length:
            raise ValueError("allreduce_counts: contiguous int64 device tensors of one length")
    ptrs = (ctypes.c_void_p * n)(*[t.data_ptr() for t in tensors])
    devs = (ctypes.c_int32 * n)(*[t.device.index for t in tensors])
    strm = (ctypes.c_void_p * n)(*[(s or torch.cuda.current_stream(t.device)).cuda_stream
                                   for s, t in zip(streams or [None] * n, tensors)])
    _lib.check(_lib.lib().cvd_allreduce_counts(ptrs, length, n, devs, strm))
    for t in tensors:
        torch.cuda.synchronize(t.device)
    return tensors


def pd_rows(counts, N_list, p_vec, num_iter):
    """Rows {N, p, Pd, Pc} exactly as Pd_plotter.py:225-233."""
    c = counts.cpu().numpy()
    rows = []
    for iN, N in enumerate(N_list):
        for ip, p in enumerate(p_vec):
            s1, s2 = int(c[iN, ip, 0]), int(c[iN, ip, 1])
            rows.append({"N": N, "p": p, "Pd": s1 / num_iter, "Pc": (s1 + s2) / (2 * num_iter)})
    return rows
