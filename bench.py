#!/usr/bin/env python3
"""Benchmark: Monte-Carlo trials/s of the relative-Viterbi-metric detector.

BASELINE.json metric: "MC trials/sec at N=1e5, rate-1/2 m=6 pair, 1/2/4/8 GPUs;
Pd match vs CPU".  Workload (configs[2]): the m = 6 pair (133,171) vs (171,133),
N = 1e5, p swept over {0.01, 0.02, 0.05, 0.10, 0.15, 0.20}.

One trial = one H1 plus one H2 sequence of length N (one iteration of
Pd_plotter.py:210-223).  One step = one pass over the config's p grid with
`--batch` trials per GPU at EVERY p (Pd_plotter.py:199-233 runs num_iter trials
at every p, so the sweep's p weigh equally whatever --steps is): per p the
generator kernel writes the batch's BSC-noised received streams to HBM (encoder
+ Philox noise, two launches: H1 with G1, H2 with G2), then the detector kernels
read them (Eq. 4-5 recursion, T_ref count, hashed P̂1 row lookup, fp64
log-likelihood sums, decisions, counts), the step's detector launches spread
over `--streams` device queues.  Both kernels are inside the timed region;
learning P̂1 (host setup, once per p) is not.

Multi-GPU: one process per GPU, rank r takes its own global trial ids every
step (weak scaling); the success counts are reduced with one RCCL all_reduce
at the end of the timed region.  `--gpus N` without a torch.distributed
launcher (no WORLD_SIZE in the environment) starts the N ranks itself, before
any GPU call, and exits with their status; under a launcher WORLD_SIZE must
equal --gpus.

After the timed region (rank 0, one GPU): the CPU baseline (the C oracle on
this host's cores), the "Pd match vs CPU" check at the config's informative
grid point (where Pd is neither 0 nor 1: exact counts on shared trial ids plus
a 3-sigma binomial test against a large independent GPU sample), and the C0
demo preset run in full on both sides.

Prints ONE JSON line on rank 0.
"""
import argparse
import json
import math
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "MC trials/sec at N=1e5, rate-1/2 m=6 pair, 1/2/4/8 GPUs; Pd match vs CPU"
P_GRID = [0.01, 0.02, 0.05, 0.10, 0.15, 0.20]
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
# VALU issue peak: 1024 SIMDs x 2.4 GHz, one wave64 instruction per 2 cycles per SIMD
# (MI355X_MICROARCH.md: "issues each VALU instruction over 2 cycles")
SHADER_GHZ = 2.4
VALU_PEAK_WINST = 1024 * SHADER_GHZ * 1e9 / 2

# Informative grid points (Pd neither 0 nor 1) at each config's own N, found with the
# C oracle (profiles/pd_points.jsonl): the headline sweep's Pd is 0 for m = 6 (the
# reference estimator's S*laplace denominator), so the Pd match runs here.
PD_POINTS = {
    "m6": {"N": 100_000, "p": 0.0033, "learn_len": 10_000_000},     # Pd ~ 0.27
    "m2": {"N": 10_000, "p": 0.092, "learn_len": None},             # Pd ~ 0.57
    "r23_m4": {"N": 100_000, "p": 0.0135, "learn_len": None},       # Pd ~ 0.33
}
# The points were chosen on the first trial ids (0..2000) of seed 12345, so the check runs
# on fresh ids: the CPU sample (and the GPU's exact repeat of it) starts at trial 10^6, the
# large GPU sample at 2^40 (selection and confirmation data kept apart; round 1's streams
# showed a 3-4 sigma low run in the first ~800 trials at the m6 point, profiles/diag/).
PD_SAMPLE_START = 1_000_000
# C0: demo_script.py preset 1 as BASELINE.json configs[0] states it -- (7,5) vs (5,7),
# m = 2, N = 1e3, 1e3 trials, the demo's p grid and seed (demo_script.py:114-131)
C0 = {"gen1": [[[1, 1, 1]], [[1, 0, 1]]], "gen2": [[[1, 0, 1]], [[1, 1, 1]]], "N": 1000, "trials": 1000,
      "p_vec": [0.01, 0.05, 0.1, 0.2, 0.3], "seed": 123}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl (= RCCL, one GPU per rank); gloo only to rehearse the multi-rank path")
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="m6", choices=["m6", "m2", "r23_m4", "c4"],
                    help="m6 (headline, BASELINE configs[2]), m2 (configs[1]), r23_m4 (configs[3]), c4 "
                         "(configs[4]: the m6 pair over the N-sweep x p-grid, a fixed total of trials sharded "
                         "over the ranks, every step of every trial, one count all_reduce)")
    ap.add_argument("--c4-trials", type=float, default=1e8,
                    help="c4: total trials over all ranks and grid points (BASELINE configs[4]: 1e8), split "
                         "evenly over the (N, p) grid points like the reference's num_iter per point")
    ap.add_argument("--c4-N", default="1000,10000,100000,1000000", help="c4: the N grid (Pd_plotter.py:196)")
    ap.add_argument("--N", type=int, default=None)
    ap.add_argument("--batch", type=int, default=None,
                    help="trials per GPU per p per step (a step runs every p of the config's grid)")
    ap.add_argument("--sweep", default="per-p", choices=["per-p", "all"],
                    help="per-p: a step is one batch at one p (step s at p_grid[s %% #p]) and value weighs "
                         "every p equally from the per-p mean step times; all: a step is one batch at every p "
                         "(multi-model launches), value = trials / elapsed")
    ap.add_argument("--group-streams", type=int, default=1,
                    help="device queues the step's detector launch groups are spread over (2: the LDS-filter "
                         "model's launch beside the multi-model launch, so its last round is not a tail)")
    ap.add_argument("--multi", type=int, default=1,
                    help="detect a step's grid points in multi-model launches (cvd_detect_multi: the models "
                         "that share the specialised kernel variant in ONE launch, so the step pays one "
                         "last-round tail instead of one per p); 0: one launch per p")
    ap.add_argument("--learn-len", type=int, default=1_000_000,
                    help="P̂1 learning chain length for non-enumerable codes")
    ap.add_argument("--seed", type=int, default=12345)
    ap.add_argument("--p", type=float, default=None, help="diagnostic: run one p instead of the sweep")
    ap.add_argument("--detector", default="markov", choices=["markov", "parity"],
                    help="markov: the relative-Viterbi-metric detector (headline); parity: the "
                         "parity-template baseline of comp_parity.py on the same streams")
    ap.add_argument("--gamma", type=float, default=0.6, help="parity baseline threshold (comp_parity.py:151)")
    ap.add_argument("--overlap", type=int, default=-1,
                    help="generate the next batch on a second stream while the detector runs "
                         "(-1: auto = on for the table automaton, where it measured faster)")
    ap.add_argument("--fused", type=int, default=-1,
                    help="dense (table-automaton) configs: generator and detector in ONE kernel per step "
                         "(cvd_mc_fused: each lane generates its own words and feeds the LDS-resident "
                         "automaton, no streams in HBM); -1: auto = where the library prefers it "
                         "(cvd_model_info.mc_fused: small tables, e.g. m2)")
    ap.add_argument("--cpu-baseline", type=int, default=1,
                    help="time the C oracle port on this host (rank 0, one GPU), check Pd against it at "
                         "the config's informative point, and run the C0 demo preset on both sides")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU work per timed CPU sample")
    ap.add_argument("--cpu-threads", type=int, default=None,
                    help="C oracle threads (default: the host CPUs this process may run on, capped by "
                         "OMP_NUM_THREADS when set -- the GPU box's CPU share)")
    ap.add_argument("--early-decision", type=int, default=1,
                    help="also time the same steps with early decision (counts only; a trial stops once "
                         "its decision is certain) and check its counts equal the full run's -- reported "
                         "beside the headline, which always runs every step of every trial")
    ap.add_argument("--pmc-traffic", default=None,
                    help="per-launch detector counter summary of rocprofv3 --pmc passes "
                         "(profiles/collect.sh + summarize.py; default profiles/pmc_<detector>_<config>.json); "
                         "used only when its config/batch/N match this run")
    return ap.parse_args()


def sweep_value(step_ms, npg, B, world, sweep_all=False):
    """Trials/s of a p sweep from the timed steps' durations (ms, max over ranks).
    Per-p steps (step s at p_grid[s % npg], B trials per rank): B x ranks / (the mean over
    the p of the mean step time at p), so every p weighs the same however many steps each
    p got (Pd_plotter.py:199-233 runs num_iter trials at every p).  Sweep steps (every p
    in every step): trials / total time.  Returns (value, indices of the p covered)."""
    import numpy as np
    if not step_ms:
        raise ValueError("no timed steps")
    if sweep_all:
        return world * npg * B / (float(np.mean(step_ms)) * 1e-3), list(range(npg))
    by = {}
    for s, t in enumerate(step_ms):
        by.setdefault(s % npg, []).append(t)
    return world * B / (float(np.mean([np.mean(v) for v in by.values()])) * 1e-3), sorted(by)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(a):
    """`--gpus N` without a launcher: start N ranks (torch.distributed.run, one
    process per GPU) as children before this process touches the GPU, and
    return their exit status.  Under a launcher, check WORLD_SIZE == --gpus."""
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is not None:
        if int(world_env) != a.gpus:
            print(json.dumps({"error": f"WORLD_SIZE={world_env} but --gpus {a.gpus}"}), flush=True)
            sys.exit(2)
        return None
    if a.gpus <= 1:
        return None
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def _smi(args, timeout=20):
    """rocm-smi's JSON for `args` (a child process; {} when the tool or the query fails)."""
    try:
        out = subprocess.run(["rocm-smi"] + args + ["--json"], capture_output=True, text=True, timeout=timeout)
        txt = out.stdout
        return json.loads(txt[txt.index("{"):]) if "{" in txt else {}
    except (OSError, ValueError, subprocess.SubprocessError):
        return {}


def _visible_cards(d):
    """the rocm-smi card entries of the GPU(s) this process may use (HIP/ROCR visibility lists
    index the host's cards in rocm-smi's order; without one, every card)."""
    cards = sorted((k for k in d if k.startswith("card")), key=lambda k: int(k[4:]) if k[4:].isdigit() else 0)
    vis = os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("ROCR_VISIBLE_DEVICES") or \
        os.environ.get("CUDA_VISIBLE_DEVICES")
    if vis:
        try:
            idx = [int(x) for x in vis.split(",") if x.strip() != ""]
            sel = [cards[i] for i in idx if 0 <= i < len(cards)]
            if sel:
                return sel
        except ValueError:
            pass
    return cards


def box_identity():
    """The box and its GPU before this process touches the GPU (rocm-smi in a child process):
    product, serial / unique id, power cap, the clock levels, and the idle clocks.  Boxes differ
    by a few per cent on the same tree; the record makes that attributable."""
    ident = _smi(["--showproductname", "--showserial", "--showuniqueid", "--showmaxpower", "--showdriverversion"])
    clk = _smi(["--showclocks", "--showtemp", "--showpower"])
    cards = _visible_cards(ident) or _visible_cards(clk)
    keep = ("Card Series", "Card SKU", "Card model", "GFX Version", "Serial Number", "Unique ID",
            "Max Graphics Package Power (W)", "Driver version")
    out = {"hostname": socket.gethostname(), "cards": {}}
    for c in cards:
        e = {k: v for k, v in ident.get(c, {}).items() if any(s in k for s in keep)}
        e["idle"] = {k: v for k, v in clk.get(c, {}).items() if "clk" in k.lower() or "Temperature" in k
                     or "Power" in k}
        out["cards"][c] = e
    drv = ident.get("system", {}).get("Driver version")
    if drv:
        out["driver"] = drv
    if not cards:
        out["note"] = "rocm-smi gave no card records"
    return out


class ClockSampler:
    """rocm-smi's current clocks, power and temperature of the visible card(s), sampled from a
    host thread every `period` s while the timed region runs (child processes; no GPU call from
    this process).  summary() gives each field's median over the samples."""

    def __init__(self, period=4.0):
        import threading
        self.period, self.samples, self._stop = period, [], threading.Event()
        self._t = threading.Thread(target=self._run, daemon=True)

    def _run(self):
        while not self._stop.is_set():
            d = _smi(["--showclocks", "--showpower", "--showtemp"], timeout=15)
            cards = _visible_cards(d)
            if cards:
                self.samples.append({c: d[c] for c in cards})
            self._stop.wait(self.period)

    def start(self):
        self._t.start()
        return self

    def stop(self):
        self._stop.set()
        self._t.join(timeout=30)

    def summary(self):
        import re
        vals = {}
        for s in self.samples:
            for c, e in s.items():
                for k, v in e.items():
                    m = re.search(r"(-?\d+(?:\.\d+)?)\s*(Mhz|MHz|W)?\)?\s*$", str(v))
                    if m and ("clk" in k.lower() or "Power" in k or "Temperature" in k):
                        vals.setdefault(c, {}).setdefault(k, []).append(float(m.group(1)))
        med = {c: {k: sorted(v)[len(v) // 2] for k, v in e.items()} for c, e in vals.items()}
        return {"samples": len(self.samples), "period_s": self.period, "median_under_load": med}


def main():
    a = parse()
    rc = launch_ranks(a)
    if rc is not None:
        sys.exit(rc)
    # (before any GPU call: rocm-smi in child processes; not under a profiler, whose preloaded
    # library would initialise the GPU in those children before their interpreter's exec)
    profiled = any(k.startswith("ROCPROF") for k in os.environ) or "rocprof" in os.environ.get("LD_PRELOAD", "")
    box = box_identity() if (int(os.environ.get("RANK", "0")) == 0 and os.environ.get("CVD_BENCH_SMI", "1") != "0"
                             and not profiled) else None
    import numpy as np
    import torch
    from __graft_entry__ import load_package
    pkg = load_package()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if a.dist_backend == "gloo" and os.environ.get("CVD_BENCH_ONE_DEVICE") == "1":
        local = 0   # rehearsal of the multi-rank path on a one-GPU box (RCCL needs one GPU per rank)
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if a.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")

    if a.config == "c4":
        return run_c4(a, pkg, world, rank, local, dist)
    cc = pkg.CONFIG_CODES[a.config]
    k, n, m = cc["k"], cc["n"], cc["m"]
    N = a.N if a.N is not None else {"m6": 100_000, "m2": 10_000, "r23_m4": 100_000}[a.config]
    p_grid = P_GRID if a.config != "m2" else [0.05]
    if a.p is not None:
        p_grid = [a.p]   # diagnostic: one grid point only (not the headline sweep)
    det = pkg.Detector(k, n, m, cc["gen1"], device=local)
    g1 = pkg.Code(cc["gen1"], m, k, n)
    g2 = pkg.Code(cc["gen2"], m, k, n)
    parity = a.detector == "parity"
    t_setup = time.perf_counter()
    if parity:
        # parity-template baseline (comp_parity.py): template of G1, no learned model
        tpl = pkg.default_template(cc["gen1"], m)
        models, info = {}, {"kind": 0, "explicit_kernel": 0, "learn_len_eff": 0, "n_rows": 0}
    else:
        models = dict(zip(p_grid, det.prepare_models(p_grid, a.learn_len if m == 6 else None, 200, 1.0, a.seed)))
        info = models[p_grid[0]].info()
    t_setup = time.perf_counter() - t_setup
    # Steps and the weighting of the p grid (Pd_plotter.py:199-233 runs num_iter trials at
    # EVERY p, so a sweep's throughput is (trials per p x #p) / sum over p of its time: the
    # p weigh equally).
    #  --sweep per-p (default): step s is one batch of B trials per GPU at p_grid[s % #p] --
    #    C2's 1e7 trials per p run as launches of B = 2,621,440 trials (20 residency rounds
    #    of 131,072 trials: 4 waves/SIMD x 1024 SIMDs x 64 lanes = 262,144 sequences; the
    #    last round's uneven wave finish is < 1% of such a launch).  `value` = B x ranks /
    #    (the mean over p of the mean step time at p), so every p weighs the same whatever
    #    --steps is; `value_wall` = trials / elapsed of the same steps.
    #  --sweep all: step s runs B trials at every p (the models that share the specialised
    #    kernel variant in one launch, cvd_detect_multi); `value` = trials / elapsed.  The
    #    smaller per-p batches cost ~2-3% against the per-p launches (profiles/r04c/).
    sweep_all = a.sweep == "all"
    npg = len(p_grid)
    B = a.batch or ({"m6": 655_360, "m2": 4_194_304, "r23_m4": 131_072} if sweep_all
                    else {"m6": 2_621_440, "m2": 4_194_304, "r23_m4": 131_072})[a.config]
    if a.fused < 0:
        a.fused = int(not parity and bool(info["mc_fused"]))   # where it measured faster (cvd_model_info)
    if a.fused:
        a.overlap = 0
    overlap_rec = {"requested": a.overlap}
    if a.overlap < 0:
        # the next batch's generator on its own queue, beside the detector: for the dense table
        # kernel (kind 0), and for persistent detector launches (k1s), whose retiring waves the
        # generator's blocks follow -- +1.1% at m6 (profiles/r05bd2); the m = 6 butterfly
        # kernel's block launches lost ~2% to it (profiles/r04y).  --sweep all keeps its
        # multi-model launches unless --overlap 1 is passed
        persistent = any(mm.info().get("persist_seqs", 0) > 0 for mm in models.values())
        a.overlap = int((not info["kind"] or persistent) and not (sweep_all and a.multi and not parity))
        overlap_rec["auto"] = {"dense_table": not info["kind"], "persistent_detector": persistent,
                               "sweep_all_multi_kept": bool(sweep_all and a.multi and not parity)}
    buf_bytes = det.words_per_seq(N) * 4 * 2 * B
    if a.overlap:
        # two stream buffers must fit the free HBM with 16 GiB to spare (the m6 headline's two
        # are 2 x 131 GB; CVD_BENCH_OVERLAP_CAP_GB sets the limit instead)
        cap = os.environ.get("CVD_BENCH_OVERLAP_CAP_GB")
        free_b = torch.cuda.mem_get_info(det.device)[0] if torch.cuda.is_available() else 0
        limit = (int(cap) << 30) if cap else free_b - (16 << 30)
        overlap_rec.update({"free_bytes": free_b, "two_buffers_bytes": 2 * buf_bytes, "limit_bytes": limit,
                            "limit_source": "CVD_BENCH_OVERLAP_CAP_GB" if cap else "free HBM - 16 GiB"})
        if 2 * buf_bytes > limit:
            a.overlap = 0
            overlap_rec["turned_off"] = "two stream buffers exceed the limit"
    overlap_rec["on"] = bool(a.overlap)
    per_step = npg if sweep_all else 1        # grid points (launch units) per step

    def units(s):
        """the step's (grid point, first global trial id of this rank's batch)"""
        tb = (s * world + rank) * B
        return [(i, tb) for i in range(npg)] if sweep_all else [(s % npg, tb)]

    # Overlap (table automaton): double-buffered generator on its own stream, units in
    # sequence; otherwise one buffer per unit of a step, the step's generator launches
    # first, then its detector launches -- with --sweep all and --multi, the grid points
    # whose models share the specialised kernel variant in one launch each (m6: p = 0.01
    # with its LDS filter, then the other five).  (Concurrent per-p launches on 2, 3 or 6
    # device queues measured 0.3%, 12% and 8% slower than one queue: the models' tables
    # compete for the caches, profiles/r04a/.)
    nbuf = 0 if a.fused else (2 if a.overlap else per_step)
    bufs = [det.stream_buffer(N, 2 * B) for _ in range(nbuf)]
    counts = torch.zeros((npg, 2), dtype=torch.int64, device=det.device)
    main = torch.cuda.current_stream()
    gstream = torch.cuda.Stream(device=det.device) if a.overlap else main
    use_multi = sweep_all and bool(a.multi) and not (a.overlap or a.fused or parity)
    groups = (det.multi_groups([models[p] for p in p_grid], [2 * B] * len(p_grid)) if use_multi
              else [[j] for j in range(per_step)])      # positions within a step's units
    nq = 1 if (a.overlap or not sweep_all) else max(1, min(a.group_streams, len(groups)))
    queues = [main] + [torch.cuda.Stream(device=det.device) for _ in range(nq - 1)]

    def gen(unit, buf, ev=None):
        if a.fused:
            return   # the fused kernel generates its own words (detect below)
        i, tb = unit
        p = p_grid[i]
        tag = pkg.grid_tag(N, p)
        if ev is not None:
            ev[0].record(gstream)
        det.generate(g1, N, p, a.seed, tag, 2 * tb, 2, B, out=buf, q0=0, pitch=2 * B, stream=gstream)
        det.generate(g2, N, p, a.seed, tag, 2 * tb + 1, 2, B, out=buf, q0=B, pitch=2 * B, stream=gstream)
        if ev is not None:
            ev[1].record(gstream)

    early = [False]

    def detect(us, bs, st, ev=None):
        """units us (with their stream buffers bs) in one call"""
        if ev is not None:
            ev[0].record(st)
        if len(us) > 1:
            det.detect_multi([models[p_grid[i]] for i, _ in us], bs, N, [2 * B] * len(us), [B] * len(us),
                             [counts[i] for i, _ in us], stream=st, early_decision=early[0])
        else:
            (i, tb), = us
            p = p_grid[i]
            if parity:
                pkg.parity_detect(bs[0], n, N, 2 * B, B, tpl, a.gamma, counts=counts[i], stream=st)
            elif a.fused:
                det.run_trials(models[p], cc["gen1"], cc["gen2"], N, p, a.seed, tb, tb + B,
                               counts=counts[i], stream=st, early_decision=early[0], fused=True)
            else:
                det.detect(models[p], bs[0], N, 2 * B, B, counts=counts[i], stream=st, early_decision=early[0])
        if ev is not None:
            ev[1].record(st)

    def run(steps, base, ev=None):
        """steps from step `base`; ev: {"gen": per unit, "det": [step][group], "end": per step
        (main stream, after the step's detector launches), "t0": start}"""
        if steps <= 0:
            return
        if ev is not None:
            ev["t0"].record(main)
        if not a.overlap:
            for s in range(steps):
                us = units(base + s)
                for j, u in enumerate(us):
                    gen(u, bufs[j] if nbuf else None, ev["gen"][s * per_step + j] if ev else None)
                if nq > 1:
                    ready = torch.cuda.Event()
                    ready.record(main)
                    for q in queues[1:]:
                        q.wait_event(ready)
                # (nq > 1: the largest group goes last on the main queue, the others first on
                # their own queues, so their last rounds overlap the large launch)
                order = sorted(range(len(groups)), key=lambda g: len(groups[g])) if nq > 1 else range(len(groups))
                for k, g in enumerate(order):
                    q = queues[(len(groups) - 1 - k) % nq] if nq > 1 else main
                    detect([us[j] for j in groups[g]], [bufs[j] for j in groups[g]] if nbuf else [None],
                           q, ev["det"][s][g] if ev else None)
                for q in queues[1:]:
                    main.wait_stream(q)
                if ev is not None:
                    ev["end"][s].record(main)
            return
        flat = [(s, j, u) for s in range(steps) for j, u in enumerate(units(base + s))]
        nu = len(flat)
        done = [torch.cuda.Event() for _ in range(nu)]
        ready = [torch.cuda.Event() for _ in range(nu)]
        gen(flat[0][2], bufs[0], ev["gen"][0] if ev else None)
        ready[0].record(gstream)
        for x in range(nu):
            s, j, u = flat[x]
            main.wait_event(ready[x])
            detect([u], [bufs[x % 2]], main, ev["det"][s][j] if ev else None)
            done[x].record(main)
            if ev is not None and j == per_step - 1:
                ev["end"][s].record(main)
            if x + 1 < nu:
                if x >= 1:
                    gstream.wait_event(done[x - 1])   # buffer (x+1)%2 was read by detect(x-1)
                gen(flat[x + 1][2], bufs[(x + 1) % 2], ev["gen"][x + 1] if ev else None)
                ready[x + 1].record(gstream)
        main.wait_stream(gstream)

    def make_events(steps):
        E = lambda: torch.cuda.Event(enable_timing=True)   # noqa: E731
        return {"t0": E(), "gen": [[E(), E()] for _ in range(steps * per_step)],
                "det": [[[E(), E()] for _ in groups] for _ in range(steps)], "end": [E() for _ in range(steps)]}

    def step_times(ev, steps):
        """ms of each step on the main stream (from the previous step's end)"""
        out, prev = [], ev["t0"]
        for s in range(steps):
            out.append(prev.elapsed_time(ev["end"][s]))
            prev = ev["end"][s]
        return out

    def weighted_value(st_ms, steps):
        return sweep_value(st_ms[:steps], npg, B, world, sweep_all)

    # warmup steps use trial ids far from the timed ones (base 10,000 steps)
    run(a.warmup, 10_000)
    counts.zero_()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    ev = make_events(a.steps)
    sampler = ClockSampler().start() if box is not None else None
    t0 = time.perf_counter()
    run(a.steps, 0, ev)
    shard = counts.clone() if dist else None   # this rank's own counts (reduce_record checks the reduce)
    if dist:
        dist.all_reduce(counts)                # the one collective: success counts over RCCL
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if sampler is not None:
        sampler.stop()
        box["under_load"] = sampler.summary()

    def max_over_ranks(x):
        # RCCL reduces device tensors only; gloo host tensors
        t = torch.tensor(x if isinstance(x, list) else [x], device=det.device if a.dist_backend == "nccl" else "cpu",
                         dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return [float(v) for v in t.tolist()] if isinstance(x, list) else float(t[0])

    st_ms = step_times(ev, a.steps)
    if dist:
        elapsed = max_over_ranks(elapsed)
        st_ms = max_over_ranks(st_ms)          # each step's time: the slowest rank's
    for mdl in models.values():
        mdl.device_error()                     # raises if a detector launch flagged an error
    gen_ms = 0.0 if a.fused else float(np.mean([e[0].elapsed_time(e[1]) for e in ev["gen"]])) * per_step
    # detector launches: per launch group, mean over the steps (ms)
    grp_all = [[ev["det"][s][g][0].elapsed_time(ev["det"][s][g][1]) for s in range(a.steps)]
               for g in range(len(groups))]
    grp_ms = [float(np.mean(x)) for x in grp_all]
    phase_ms = float(np.sum(grp_ms)) if nq == 1 else float(np.mean(
        [max(ev["gen"][(s + 1) * per_step - 1][1].elapsed_time(ev["det"][s][g][1]) for g in range(len(groups)))
         for s in range(a.steps)]))
    # the dominant launch (the roofline's kernel): the group with the most grid points
    gdom = max(range(len(groups)), key=lambda g: (len(groups[g]), grp_ms[g]))
    det_ms = grp_ms[gdom]
    if sweep_all:
        det_by = [{"p": [p_grid[i] for i in groups[g]], "ms": grp_ms[g]} for g in range(len(groups))]
    else:
        det_by = [{"p": [p_grid[i]], "ms": float(np.mean(grp_all[0][i::npg])), "launches": len(grp_all[0][i::npg])}
                  for i in range(min(npg, a.steps))]
        # one launch per step: the detector's launch time weighted like `value` (mean over p)
        det_ms = phase_ms = float(np.mean([x["ms"] for x in det_by]))
    steps_at = [len(range(i, a.steps, npg)) if not sweep_all else a.steps for i in range(npg)]
    value, p_covered = weighted_value(st_ms, a.steps)

    # the same steps (same trial ids) with early decision: counts must be identical
    early_out = None
    if a.early_decision and not parity:
        full_counts = counts.clone()
        counts.zero_()
        early[0] = True
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        ev2 = make_events(a.steps)
        t1 = time.perf_counter()
        run(a.steps, 0, ev2)
        if dist:
            dist.all_reduce(counts)
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        torch.cuda.synchronize()
        el2 = time.perf_counter() - t1
        st2 = step_times(ev2, a.steps)
        if dist:
            el2 = max_over_ranks(el2)
            st2 = max_over_ranks(st2)
        early[0] = False
        early_out = {"value": weighted_value(st2, a.steps)[0], "value_wall": a.steps * per_step * B * world / el2,
                     "unit": "trials/s", "ms_per_step": el2 / a.steps * 1e3,
                     "counts_equal_full_run": bool(torch.equal(counts, full_counts)),
                     "note": "counts only: each trial stops once its decision is certain (rigorous IEEE "
                             "bounds on the remaining increments, CVD_DETECT_EARLY_DECISION); the "
                             "headline value above runs every step of every trial"}
        counts.copy_(full_counts)

    dist_rec = reduce_record(dist, shard, counts, world, rank,
                             f"rank r takes global trial ids [(s W + r) B, (s W + r + 1) B) of step s, B = {B}")
    # per-rank setup (model learning on the GPU + the JIT compile of the specialised kernel,
    # every rank at once): the multi-rank rehearsal's evidence, one entry per rank
    setup_by_rank = [{"rank": rank, "setup_s": t_setup, "host": socket.gethostname(), "device": local}]
    if dist:
        lst = [None] * world
        dist.all_gather_object(lst, setup_by_rank[0])
        setup_by_rank = lst
    if rank != 0:
        if dist:
            dist.destroy_process_group()
        return
    trials = a.steps * per_step * B * world
    value_wall = trials / elapsed
    # roofline of the dominant kernel (detector): algorithmic bytes = the packed received
    # streams read once, 2 * ceil(N * n / 8) bytes per trial, per launch of
    # the dominant launch group (m6: the multi-model launch of five grid points), over that
    # launch's average duration (HIP events on its stream, the figure rocprofv3 reports)
    alg_bytes = B * 2 * ((N * n + 7) // 8)               # one grid point's batch
    alg_launch = len(groups[gdom]) * alg_bytes
    achieved = alg_launch / (det_ms * 1e-3) / 1e9
    # Dense-table kernels (C1 fused, C3 table16): bound by the LDS array, measured --
    # SQ_LDS_IDX_ACTIVE over the launch's CU-cycles, and the share of it that is bank-
    # conflict cycles (profiles/lds_bound.py over the r04_lds_pmc.sh passes).  The roofline
    # keeps SURVEY §8(d)'s stream bytes (which the fused kernel never writes to HBM: it is
    # the figure the §8(d) fraction is defined on) and carries the LDS counters beside it.
    lds_diag = None
    lds_path = os.path.join(ROOT, "profiles", f"pmc_lds_{a.config}.json")
    if not parity and info["kind"] == 0 and os.path.exists(lds_path):
        with open(lds_path) as f:
            ld = json.load(f)
        lds_diag = {k: ld[k] for k in ("kernel", "lds_busy", "lds_conflict_frac", "lds_array_cycles_per_lds_inst",
                                        "valu_issue_2cyc", "source")}
        lds_diag["meaning"] = ("lds_busy = SQ_LDS_IDX_ACTIVE / (256 CUs x kernel cycles); lds_conflict_frac = "
                               "SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE; valu_issue_2cyc = SQ_INSTS_VALU x 2 / "
                               "(1024 SIMDs x kernel cycles)")
    traffic, traffic_src, pmc = None, None, None
    if a.pmc_traffic is None:
        a.pmc_traffic = os.path.join(ROOT, "profiles", f"pmc_{a.detector}_{a.config}.json")
    if a.pmc_traffic and os.path.exists(a.pmc_traffic):
        with open(a.pmc_traffic) as f:
            pmc = json.load(f)
        if (pmc.get("config"), pmc.get("N"), pmc.get("detector", "markov"),
                bool(pmc.get("fused", False))) != (a.config, N, a.detector, bool(a.fused)) or \
                sorted(pmc.get("per_p", {})) != sorted(str(p) for p in p_grid):
            pmc = None   # counters of another workload (or of a single-p diagnostic run)
    valu = None
    traffic_by_p, gen_pmc = None, None
    if pmc is not None:
        # launch-weighted mean over the sweep, per trial of the PMC run's launches (whole
        # residency rounds like this run's) times this run's trials per launch
        pmc_scale = B / float(pmc.get("batch") or B)
        # per launch: --sweep per-p, the launch-weighted mean over the sweep (each p one launch,
        # like `value`'s weighting); --sweep all, the FETCH of the dominant launch's grid points
        try:
            traffic = (sum(pmc["per_p"][str(p_grid[i])]["fetch_bytes"] for i in groups[gdom]) if sweep_all
                       else pmc["detector_fetch_bytes_per_launch"]) * pmc_scale
        except (KeyError, TypeError):
            traffic = None
        traffic_by_p = {p: {"fetch_bytes": e["fetch_bytes"] * pmc_scale, "fetch_x_algorithmic": e["fetch_x_algorithmic"],
                            "fetch_raw_x_algorithmic": e["fetch_raw_x_algorithmic"],
                            "valu_insts_per_wave_step": e["VALU_insts_per_wave_step"],
                            "vmem_rd_insts_per_wave_step": e["VMEM_RD_insts_per_wave_step"]}
                        for p, e in pmc["per_p"].items()}
        g = pmc.get("generator") or {}
        if g.get("counters_per_launch"):
            gen_pmc = {k: g[k] for k in ("kernel", "fetch_bytes_raw", "VALU_insts_per_wave", "VALU_insts_per_stream_word",
                                         "SALU_insts_per_stream_word", "busy_frac_of_wave_cycles",
                                         "wait_any_frac_of_wave_cycles") if k in g}
        traffic_src = (os.path.relpath(a.pmc_traffic, ROOT) + " (" + pmc.get("traffic_basis", "rocprofv3 FETCH_SIZE")
                       + (f"; counted on {pmc.get('batch')}-trial launches, scaled to {B}" if pmc_scale != 1.0 else "")
                       + ")")
        ipws = pmc.get("VALU_insts_per_wave_step")
        if ipws:
            # VALU roofline of the detector (its binding resource): wave-instructions
            # per launch from the counter pass, over this run's live launch time
            winst = ipws * (2 * B * len(groups[gdom]) / 64) * N    # the dominant launch
            ach = winst / (det_ms * 1e-3)
            # (counted instructions at the 2-cycle wave64 issue rate; round 5's modelled issue-cycle
            # fraction -- a static instruction mix priced per opcode -- read above 1 at p = 0.02 and
            # is no longer reported)
            valu = {"insts_per_wave_step": ipws, "achieved": ach, "peak": VALU_PEAK_WINST,
                    "unit": "wave-instructions/s", "frac": ach / VALU_PEAK_WINST,
                    "source": os.path.relpath(a.pmc_traffic, ROOT) + " (SQ_INSTS_VALU) + live HIP-event time "
                              "of the launch"}
            # where the detector's wave-cycles go (SQ_WAVE_CYCLES = ACTIVE_INST_ANY + WAIT_ANY +
            # WAIT_INST_ANY, MI355X_MICROARCH.md), launch-weighted over the sweep
            cpl = pmc.get("counters_per_launch") or {}
            wc = cpl.get("SQ_WAVE_CYCLES")
            if wc:
                valu["wave_cycles_split"] = {k: cpl.get(c, 0.0) / wc for k, c in (
                    ("issuing", "SQ_ACTIVE_INST_ANY"), ("waiting_on_memory_or_barrier", "SQ_WAIT_ANY"),
                    ("issue_stalled", "SQ_WAIT_INST_ANY"))}
    # What bounds the m = 6 detector (k1s): VALU issue -- not HBM bandwidth, not lookup bytes and
    # not lookup latency.  The ablations it rests on (same-box A/Bs): extra VALU per
    # step (CVD_K1S_PADV, timing only) lengthens p = 0.05 by +3.4 / +6.5 / +15% for 8 / 16 / 32
    # independent v_bitop3 -- each added instruction costs ~2.3 SIMD-cycles, its full issue cost --
    # and p = 0.2 by about half that (profiles/r06w); doubling every lookup load's latency budget
    # (the two-step lookup pipeline, CVD_K1S_DEEP) changes nothing (profiles/r06u); a third fewer
    # lookup bytes changes nothing (three-line slots, profiles/r06j); the VALU issues one wave64
    # instruction per 3.65 SIMD-cycles at p = 0.05 (profiles/r06v) against measured issue costs of
    # 2.4-4.6 cycles per instruction form (profiles/r05an).
    valu_bound = (not parity and not lds_diag and info.get("kind") == 1 and info.get("explicit_kernel") == 5)
    bound_basis = None
    if valu_bound:
        bound_basis = ("VALU issue at p >= 0.05 (partly at p = 0.2): +8/+16/+32 independent VALU per step (timing only) "
                       "-> p = 0.05 +3.4/+6.5/+15%, p = 0.2 +1.6/+3.6/+9%, ~2.3 SIMD-cycles per added v_bitop3 at "
                       "p = 0.05 = its issue cost (profiles/r06w); one VALU instruction per 3.65 SIMD-cycles against "
                       "2.4-4.6-cycle issue costs per form (profiles/r06v, r05an); not lookup latency (twice the "
                       "latency budget for every lookup load: +-0.5%, profiles/r06u); not lookup bytes (three-line "
                       "slots: FETCH -18-25%, time +1%, profiles/r06j); not HBM (0.009 of peak)")
    elif lds_diag:
        bound_basis = "LDS array busy (roofline.lds, profiles/pmc_lds_<config>.json)"
    c = counts.cpu().numpy()
    per_p = {str(p): {"Pd": float(c[i, 0]) / max(1, steps_at[i] * B * world),
                      "Pc": float(c[i, 0] + c[i, 1]) / max(1, 2 * steps_at[i] * B * world),
                      "trials": steps_at[i] * B * world,
                      "h1_successes": int(c[i, 0]), "h2_successes": int(c[i, 1])}
             for i, p in enumerate(p_grid)}
    out = {
        "metric": (METRIC if a.config == "m6" and not parity
                   else f"MC trials/sec ({a.config}, N={N}{', parity-template baseline' if parity else ''})"),
        "value": value,
        "value_wall": value_wall,
        "unit": "trials/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": elapsed / a.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": ("u32 bit-planes (metrics, four planes of the 64 states) + f64 (log-likelihood sums)"
                  if info.get("explicit_kernel") == 5 else "u16x2 (metrics) + f64 (log-likelihood sums)"),
        "data": "synthetic: Philox4x32-10 encoder inputs and BSC(p) flips (build spec), learned P̂1",
        "config": {"name": a.config, "detector": a.detector,
                   "workload": (f"{a.config} pair {cc['gen1']} vs {cc['gen2']}, N={N}, p-sweep {p_grid}, "
                                + (f"every p in every step ({B} trials per p per GPU)" if sweep_all else
                                   f"one p per step ({B} trials per GPU, step s at p_grid[s % {npg}])")),
                   "N": N, "p_grid": p_grid, "sweep": a.sweep,
                   "p_weighting": ("equal: each step runs the same trials per GPU at every p of the grid; value = "
                                   "trials / elapsed" if sweep_all else
                                   "equal: value = B x GPUs / (mean over p of the mean step time at p), the sweep's "
                                   "throughput at the same trials per p (Pd_plotter.py:199-233 runs num_iter trials "
                                   "per p) whatever --steps is; value_wall = trials / elapsed weighs p by its step count"),
                   "p_covered": [p_grid[i] for i in p_covered],
                   "trials_per_p_per_step_per_gpu": B, "trials_per_step_per_gpu": B * per_step,
                   "k": k, "n": n, "m": m,
                   "model": info["kind"] and "sparse(learned)" or "dense",
                   "learn_len": info["learn_len_eff"], "model_rows_p0": info["n_rows"],
                   "parallelism": f"dp{world} (trial sharding, one RCCL all_reduce of counts)"},
        "distributed": dist_rec,
        "roofline": {"bound": "lds" if lds_diag else ("valu" if valu_bound else "hbm"), "achieved": achieved,
                     "bound_basis": bound_basis,
                     "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                     "lds": lds_diag,
                     "traffic": traffic,
                     "kernel": ("parity_kernel (parity-template baseline, cvd_parity.hip)" if parity
                                else "mc_table16_kernel (generator + LDS table automaton fused, cvd_mc_fused; "
                                     "achieved = SURVEY 8(d) stream bytes, which stay on chip)" if a.fused
                                else pkg.KERNEL_NAMES[info["explicit_kernel"]] if info["kind"]
                                else "detect_table_kernel (enumerated state automaton)"),
                     "traffic_source": traffic_src,
                     "traffic_x_algorithmic": (traffic / alg_launch) if traffic else None,
                     "traffic_by_p": traffic_by_p,
                     "algorithmic_bytes_per_launch": alg_launch, "avg_launch_ms": det_ms,
                     "launch_grid_points": [p_grid[i] for i in groups[gdom]],
                     "detector_launches_per_step": len(groups), "detector_ms_per_step": phase_ms,
                     "valu": valu},
        "diagnostic": {"generator_ms_per_step": gen_ms, "detector_ms_per_step": phase_ms,
                       "overlap": bool(a.overlap), "overlap_decision": overlap_rec, "fused": bool(a.fused),
                       "model_setup_s": t_setup,
                       "setup_by_rank": setup_by_rank,
                       "multi_model_launches": use_multi,
                       "seq_steps_per_s_detector": 2 * B * per_step * N / (phase_ms * 1e-3),
                       "step_ms": st_ms,
                       "detector_ms_by_launch": det_by,
                       "generator_pmc": gen_pmc,
                       # walk mode of the m = 6 kernel per grid point (cvd_model_info.walk)
                       "walk_by_p": {str(p): int(models[p].info().get("walk", 0)) for p in p_grid} if models else None,
                       "lds_filter_by_p": ({str(p): int(models[p].info().get("lds_filter", 0)) for p in p_grid}
                                           if models else None),
                       "per_p": per_p},
    }
    if early_out is not None:
        out["early_decision"] = early_out
    out["box"] = box
    bufs.clear()                               # the stream buffers (up to 2 x 131 GB) before the legs below
    torch.cuda.empty_cache()
    if a.cpu_baseline and world == 1 and not parity:
        host = host_info(a.cpu_threads)
        out["cpu_baseline"], _ = cpu_baseline(cc, k, n, m, N, a.seed, a.learn_len, a.cpu_seconds, host)
        out["pd_match_vs_cpu"] = pd_match(pkg, det, cc, a.config, k, n, m, a.seed, a.cpu_seconds, host)
        out["c0_demo"] = c0_demo(pkg, host)
        if a.config == "m6":
            out["reference_call"] = reference_call(pkg, cc, k, n, m, N, p_grid, a.learn_len, a.seed)
    print(json.dumps(out, default=_json_default), flush=True)
    if dist:
        dist.destroy_process_group()


def run_c4(a, pkg, world, rank, local, dist):
    """BASELINE.json configs[4]: the m = 6 pair over N in {1e3, 1e4, 1e5, 1e6} x the
    p grid, `--c4-trials` trials in total (1e8), the same number at every (N, p) grid
    point (the reference's num_iter per point, Pd_plotter.py:196-233: N outer, p
    inner).  Rank r of W takes the contiguous global trial ids [r T/W, (r+1) T/W) of
    every point; every step of every trial runs (cvd_mc_run: generator + detector,
    no early decision); ONE all_reduce of the [nN, np, 2] count tensor at the end.
    The counts depend on the global trial ids only, so they are the same for any W."""
    import numpy as np
    import torch
    cc = pkg.CONFIG_CODES["m6"]
    k, n, m = cc["k"], cc["n"], cc["m"]
    Ns = [int(float(x)) for x in a.c4_N.split(",") if x]
    p_grid = P_GRID if a.p is None else [a.p]
    npt = len(Ns) * len(p_grid)
    T = max(world, int(a.c4_trials) // npt)        # trials per grid point (all ranks)
    lo, hi = rank * T // world, (rank + 1) * T // world
    det = pkg.Detector(k, n, m, cc["gen1"], device=local)
    t_setup = time.perf_counter()
    models = dict(zip(p_grid, det.prepare_models(p_grid, a.learn_len, 200, 1.0, a.seed)))
    t_setup = time.perf_counter() - t_setup
    free, _ = torch.cuda.mem_get_info(det.device)
    # one batch's streams: up to 200 GB of the 288 GB, so N = 1e6 launches hold three
    # residency rounds (393,216 trials, 197 GB) instead of two
    budget = min(int(free * 0.75), 200 << 30)

    def batch_of(N, slots=1):
        # slots: stream slots the call holds at once (a p row in one cvd_mc_run_grid call: one
        # per p), so that the call's whole workspace, not one slot, fits the budget
        b = det.default_batch(N, hi - lo, budget // slots)
        return max(1, b)

    def row_call(N):
        return N < 100_000       # the whole p row of this N in one grid call (below)

    counts = torch.zeros((len(Ns), len(p_grid), 2), dtype=torch.int64, device=det.device)
    # the largest stream workspace, allocated once before the timed region and left in
    # torch's caching allocator, so no grid call inside it pays a fresh ~200 GB hipMalloc
    # (N = 1e5's first point took 7.4 s instead of 3.4 s that way, profiles/r04j/)
    g1c = pkg.Code(cc["gen1"], m, k, n)
    from dccvm_amd.detector import grid_workspace_bytes
    mlist = [models[p] for p in p_grid]
    ws = max(grid_workspace_bytes(mlist, g1c, [N], batch_of(N, len(p_grid)), 0) if row_call(N)
             else pkg.lib().cvd_mc_workspace_bytes(g1c.c, N, batch_of(N)) for N in Ns)
    del_me = torch.empty(max(ws, 4) // 4, dtype=torch.int32, device=det.device)
    del del_me
    # warmup: one small launch per p (smallest N) at trial ids far from the timed ones
    for p in p_grid:
        det.run_trials(models[p], cc["gen1"], cc["gen2"], min(Ns), p, a.seed, 1 << 44, (1 << 44) + 1024,
                       batch=1024, counts=torch.zeros(2, dtype=torch.int64, device=det.device))
    torch.cuda.synchronize()
    per_n_s = []
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for iN, N in enumerate(Ns):
        tn = time.perf_counter()
        B = batch_of(N, len(p_grid)) if row_call(N) else batch_of(N)
        if not row_call(N):
            # a progress line per long grid point (the launches are queued): one grid call per p
            for ip, p in enumerate(p_grid):
                det.run_grid([models[p]], cc["gen1"], cc["gen2"], [p], [N], a.seed, lo, hi, batch=B,
                             counts=counts[iN, ip].view(1, 1, 2), budget=budget)
                torch.cuda.synchronize()
                print(json.dumps({"c4_point": {"rank": rank, "N": N, "p": p, "seconds": time.perf_counter() - tn}}),
                      file=sys.stderr, flush=True)
        else:
            # the whole p row of this N in ONE library call (cvd_mc_run_grid)
            det.run_grid(mlist, cc["gen1"], cc["gen2"], p_grid, [N], a.seed, lo, hi, batch=B,
                         counts=counts[iN].view(1, len(p_grid), 2), budget=budget)
        torch.cuda.synchronize()
        per_n_s.append(time.perf_counter() - tn)
        print(json.dumps({"c4_progress": {"rank": rank, "N": N, "seconds": per_n_s[-1]}}), file=sys.stderr,
              flush=True)
    shard = counts.clone() if dist else None
    if dist:
        dist.all_reduce(counts)                  # the one collective: success counts over RCCL
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    dist_rec = reduce_record(dist, shard, counts, world, rank,
                             f"rank r takes global trial ids [r T / W, (r + 1) T / W) of every grid point, T = {T}")
    if dist:
        dev = det.device if a.dist_backend == "nccl" else "cpu"
        t = torch.tensor([elapsed] + per_n_s, device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, per_n_s = float(t[0]), [float(x) for x in t[1:].tolist()]
    if rank != 0:
        if dist:
            dist.destroy_process_group()
        return
    c = counts.cpu().numpy()
    total = T * npt
    def roof_N(i, N):
        # the packed streams read once, 2 ceil(N n / 8) bytes per trial, over
        # the N's whole pipeline time (generator + detector, max over ranks)
        ab = T * len(p_grid) * 2 * ((N * n + 7) // 8)
        ach = ab / per_n_s[i] / 1e9
        b = batch_of(N, len(p_grid)) if row_call(N) else batch_of(N)
        lpp = -(-(hi - lo) // b)                          # launches per grid point on a rank
        return {"algorithmic_bytes": ab, "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": ach / HBM_PEAK_GBS, "basis": "whole pipeline time of this N (generator + detector)",
                "launches_per_point_per_rank": lpp,
                "residency_rounds_per_launch": b / pkg.Detector.FULL_ROUND_TRIALS,
                "last_launch_rounds": ((hi - lo) - (lpp - 1) * b) / pkg.Detector.FULL_ROUND_TRIALS}

    per_N = {str(N): {"trials": T * len(p_grid), "seconds": per_n_s[i], "trials_per_s": T * len(p_grid) / per_n_s[i],
                      "seq_steps_per_s": 2 * T * len(p_grid) * N / per_n_s[i],
                      "batch_per_rank": batch_of(N, len(p_grid)) if row_call(N) else batch_of(N),
                      "roofline": roof_N(i, N),
                      "per_p": {str(p): {"h1_successes": int(c[i, j, 0]), "h2_successes": int(c[i, j, 1]),
                                         "Pd": float(c[i, j, 0]) / T, "Pc": float(c[i, j, 0] + c[i, j, 1]) / (2 * T)}
                                for j, p in enumerate(p_grid)}}
             for i, N in enumerate(Ns)}
    out = {
        "metric": "MC trials/sec (C4: m=6 pair, N-sweep x p-grid, fixed total trials, sharded over GPUs)",
        "value": total / elapsed,
        "unit": "trials/s",
        "n_gpus": world,
        "steps": npt,
        "warmup": 1,
        "ms_per_step": elapsed / npt * 1e3,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": ("u32 bit-planes (metrics, four planes of the 64 states) + f64 (log-likelihood sums)"
                  if models[p_grid[0]].info().get("explicit_kernel") == 5
                  else "u16x2 (metrics) + f64 (log-likelihood sums)"),
        "data": "synthetic: Philox4x32-10 encoder inputs and BSC(p) flips (build spec), learned P̂1",
        "config": {"name": "c4", "workload": f"m6 pair {cc['gen1']} vs {cc['gen2']}, N in {Ns} x p {p_grid}, "
                                             f"{T} trials per grid point ({total} total), one step = one grid point",
                   "N_grid": Ns, "p_grid": p_grid, "trials_per_point": T, "total_trials": total,
                   "learn_len": a.learn_len, "early_decision": False,
                   "parallelism": f"dp{world} (trial sharding, one RCCL all_reduce of counts)"},
        "per_N": per_N,
        "roofline": {"bound": "valu", "achieved": sum(per_N[str(N)]["roofline"]["algorithmic_bytes"] for N in Ns)
                     / elapsed / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": sum(per_N[str(N)]["roofline"]["algorithmic_bytes"] for N in Ns) / elapsed / 1e9 / HBM_PEAK_GBS,
                     "traffic": None,
                     "basis": "algorithmic stream bytes of every grid point (SURVEY §8(d)) over the whole timed "
                              "region (generator + detector); per N in per_N[N].roofline"},
        "counts": c.tolist(),
        "distributed": dist_rec,
        "diagnostic": {"model_setup_s": t_setup, "elapsed_s": elapsed},
    }
    if a.cpu_baseline and world == 1:
        host = host_info(a.cpu_threads)
        out["cpu_baseline"], _ = cpu_baseline(cc, k, n, m, 100_000, a.seed, a.learn_len, a.cpu_seconds, host)
    print(json.dumps(out, default=_json_default), flush=True)
    if dist:
        dist.destroy_process_group()


def reduce_record(dist, shard, reduced, world, rank, sharding):
    """The multi-GPU run checks itself: the communicator holds `world` ranks, and the
    reduced success counts equal the sum of every rank's own counts (gathered to the host
    after the timed region).  A wrong-rank, partial or double reduce raises instead of
    printing a line; the record (communicator size, backend, each rank's shard) goes into
    the bench line."""
    import numpy as np
    if not dist:
        return {"backend": None, "world_size": 1, "shards_sum_equals_reduced": True, "sharding": sharding}
    size = dist.get_world_size()
    mine = {"rank": rank, "counts": shard.cpu().tolist()}
    lst = [None] * size
    dist.all_gather_object(lst, mine)
    total = None
    for e in lst:
        v = np.asarray(e["counts"], dtype=np.int64)
        total = v if total is None else total + v
    red = reduced.cpu().numpy()
    ok = size == world and sorted(e["rank"] for e in lst) == list(range(world)) and np.array_equal(total, red)
    if not ok:
        raise RuntimeError(f"count reduce check failed: communicator size {size} (expected {world}), ranks "
                           f"{sorted(e['rank'] for e in lst)}, sum of shards {total.tolist()} != reduced {red.tolist()}")
    return {"backend": str(dist.get_backend()), "world_size": size, "shards_sum_equals_reduced": True,
            "rank_shards": [e["counts"] for e in sorted(lst, key=lambda e: e["rank"])], "sharding": sharding}


def _json_default(o):
    """numpy scalars (counts, flags) in the output line"""
    if hasattr(o, "item"):
        return o.item()
    raise TypeError(f"not JSON serializable: {type(o).__name__}")


def host_info(threads=None):
    """The host cores the CPU legs use: every CPU this process may run on, capped by
    OMP_NUM_THREADS when set (the GPU box exports its CPU share there; os.cpu_count()
    reports the whole machine)."""
    allowed = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = os.environ.get("OMP_NUM_THREADS")
    if threads:
        use = threads
    elif omp and omp.isdigit() and int(omp) > 0:
        use = min(allowed, int(omp))
    else:
        use = allowed
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"threads": int(use), "host_logical_cpus": os.cpu_count(), "affinity_cpus": allowed,
            "omp_num_threads_env": omp, "cpu_model": model}


def _sized_sample(run, threads, seconds, cal_trials):
    """Calibrate with `cal_trials`, then size a sample to ~`seconds` of CPU work (whole
    multiples of the thread count).  Returns the sample's trial count."""
    t0 = time.perf_counter()
    run(0, cal_trials)
    dt = max(time.perf_counter() - t0, 1e-6)
    ntr = max(threads, int(cal_trials * seconds / dt) // threads * threads)
    return ntr


def cpu_baseline(cc, k, n, m, N, seed, learn_len, seconds, host):
    """The oracle's C port of the reference path (oracle/cvd_oracle.c), OpenMP over
    trials on this host's cores, on a bounded sample of the headline workload (p = 0.05)."""
    from oracle import c_oracle as C
    threads = host["threads"]
    c1, c2 = C.Code(cc["gen1"], m, k, n), C.Code(cc["gen2"], m, k, n)
    p = 0.05
    mod = C.Model(c1, p, learn_len if m == 6 else None, 200, 1.0, seed)
    ntr = _sized_sample(lambda lo, hi: mod.run_trials(c1, c2, N, p, seed, lo, hi, nthreads=threads),
                        threads, seconds, threads)
    t0 = time.perf_counter()
    c_smp, _ = mod.run_trials(c1, c2, N, p, seed, 0, ntr, nthreads=threads)
    dt = time.perf_counter() - t0
    basis = ("threads = OMP_NUM_THREADS (the GPU box's CPU share for one GPU, set by the pool; the "
             f"process affinity allows {host['affinity_cpus']} CPUs of the host, which the pool's rules "
             "reserve for other jobs)") if host["omp_num_threads_env"] else \
        f"threads = every CPU in this process's affinity ({host['affinity_cpus']})"
    return {"value": ntr / dt, "unit": "trials/s", "cores": threads, "kind": "port",
            "per_core_value": ntr / dt / threads,
            "sample": f"{ntr} trials (H1+H2, N={N}) at p={p} of the headline sweep, C oracle "
                      f"(oracle/cvd_oracle.c, OpenMP), {threads} threads, {dt:.1f} s",
            "basis": basis, "seconds": dt, "host": host}, [int(x) for x in c_smp]


def pd_match(pkg, det, cc, config, k, n, m, seed, seconds, host):
    """The metric's "Pd match vs CPU" at the config's informative grid point
    (Pd neither 0 nor 1; PD_POINTS).  Outside the timed region.

    (1) exact: the GPU path on the CPU sample's own trial ids (same learned model,
        same streams) gives the same success counts, and the per-trial fp64
        log-likelihood sums of the first trials are bit-identical;
    (2) statistical: Pd of a large independent GPU sample (other trial ids) agrees
        with the CPU sample's Pd within 3 binomial standard deviations of the
        difference (pooled Pd).  Pc is checked the same way."""
    from oracle import c_oracle as C
    import numpy as np
    pt = PD_POINTS[config]
    N, p, ll = pt["N"], pt["p"], pt["learn_len"]
    threads = host["threads"]
    t0 = time.perf_counter()
    c1, c2 = C.Code(cc["gen1"], m, k, n), C.Code(cc["gen2"], m, k, n)
    cm = C.Model(c1, p, ll, 200, 1.0, seed)
    t_cpu_learn = time.perf_counter() - t0
    a0 = PD_SAMPLE_START
    ntr = _sized_sample(lambda lo, hi: cm.run_trials(c1, c2, N, p, seed, a0 + lo, a0 + hi, nthreads=threads),
                        threads, seconds, threads)
    ntr = max(ntr, 64)
    t0 = time.perf_counter()
    c_cpu, _ = cm.run_trials(c1, c2, N, p, seed, a0, a0 + ntr, nthreads=threads)
    c_cpu = [int(x) for x in c_cpu]
    t_cpu = time.perf_counter() - t0
    ncal = min(16, ntr)
    _, s_cpu = cm.run_trials(c1, c2, N, p, seed, a0, a0 + ncal, sums=True, nthreads=threads)
    t0 = time.perf_counter()
    model = det.model(p, ll, 200, 1.0, seed)
    t_gpu_learn = time.perf_counter() - t0
    got = det.run_trials(model, cc["gen1"], cc["gen2"], N, p, seed, a0, a0 + ntr)["counts"].cpu().tolist()
    sums = det.run_trials(model, cc["gen1"], cc["gen2"], N, p, seed, a0, a0 + ncal, return_sums=True)["sums"]
    big = {"m6": 131_072, "m2": 1_048_576, "r23_m4": 131_072}[config]
    gb = det.run_trials(model, cc["gen1"], cc["gen2"], N, p, seed, 1 << 40, (1 << 40) + big)["counts"].cpu().tolist()
    n1, n2 = ntr, big

    def ztest(x1, x2, t1, t2):
        pool = (x1 + x2) / (t1 + t2)
        sd = math.sqrt(max(pool * (1 - pool), 1e-12) * (1 / t1 + 1 / t2))
        return abs(x1 / t1 - x2 / t2) / sd, 3.0 * sd

    z_pd, tol_pd = ztest(c_cpu[0], gb[0], n1, n2)
    z_pc, tol_pc = ztest(c_cpu[0] + c_cpu[1], gb[0] + gb[1], 2 * n1, 2 * n2)
    exact = [int(x) for x in c_cpu] == got and bool(np.array_equal(sums, s_cpu))
    pd_cpu, pd_gpu = c_cpu[0] / n1, gb[0] / n2
    return {"point": {"N": N, "p": p, "learn_len": ll if ll else model.info()["learn_len_eff"],
                      "model_rows": model.info()["n_rows"]},
            "cpu": {"trials": n1, "first_trial": a0, "counts": [int(x) for x in c_cpu], "Pd": pd_cpu,
                    "Pc": (c_cpu[0] + c_cpu[1]) / (2 * n1), "seconds": t_cpu, "learn_s": t_cpu_learn,
                    "threads": threads},
            "gpu_same_trials": {"counts": got, "sums_bit_exact_trials": ncal, "learn_s": t_gpu_learn},
            "gpu_large_sample": {"trials": n2, "first_trial": 1 << 40, "counts": gb, "Pd": pd_gpu,
                                 "Pc": (gb[0] + gb[1]) / (2 * n2)},
            "tolerance": "3 sigma of the difference of two binomial proportions (pooled)",
            "pd_abs_diff": abs(pd_cpu - pd_gpu), "pd_tol": tol_pd, "pd_z": z_pd,
            "pc_tol": tol_pc, "pc_z": z_pc,
            "informative": bool(0.05 < pd_gpu < 0.95),
            "exact_match": bool(exact),
            "match": bool(exact and z_pd <= 3.0 and z_pc <= 3.0)}


def c0_demo(pkg, host):
    """BASELINE.json configs[0], run in full: the demo preset (7,5) vs (5,7), m = 2,
    N = 1e3, 1e3 trials over the demo's p grid -- the C oracle on this host (the CPU
    path) and the product's run_experiment on the GPU; the Pd/Pc tables must be equal."""
    from oracle import c_oracle as C
    c = C0
    threads = host["threads"]
    c1, c2 = C.Code(c["gen1"], 2, 1, 2), C.Code(c["gen2"], 2, 1, 2)
    rows_cpu = []
    t0 = time.perf_counter()
    for p in c["p_vec"]:
        cnt, _ = C.Model(c1, p, None, 200, 1.0, c["seed"]).run_trials(c1, c2, c["N"], p, c["seed"], 0,
                                                                       c["trials"], nthreads=threads)
        rows_cpu.append({"N": c["N"], "p": p, "Pd": int(cnt[0]) / c["trials"],
                         "Pc": (int(cnt[0]) + int(cnt[1])) / (2 * c["trials"])})
    t_cpu = time.perf_counter() - t0
    t0 = time.perf_counter()
    df = pkg.run_experiment(1, 2, 2, c["gen1"], c["gen2"], c["trials"], c["p_vec"], None, 200, 1.0, c["seed"],
                            N_list=[c["N"]])
    t_gpu = time.perf_counter() - t0
    rows_gpu = df.to_dict(orient="records")
    return {"config": "demo preset (7,5) vs (5,7), m=2, N=1e3, 1e3 trials, p " + str(c["p_vec"]),
            "cpu_seconds": t_cpu, "cpu_trials_per_s": len(c["p_vec"]) * c["trials"] / t_cpu, "cpu_threads": threads,
            "gpu_seconds_incl_setup": t_gpu, "rows": rows_gpu, "match": bool(rows_gpu == rows_cpu)}


def reference_call(pkg, cc, k, n, m, N, p_grid, learn_len, seed, num_iter=10_000):
    """The headline workload at the reference's own call shape: run_experiment with its
    default num_iter = 10,000 trials per p (Pd_plotter.py:176-235, 242-264) over the C2 p grid
    at N, through the product's drop-in (cvd_mc_run_grid: per N, each p's batch and one
    multi-model detector launch for the row).  The first call includes the
    models' learning and table builds and the kernel JIT (setup); the second finds them cached
    and times the trials alone; both run every step of every trial (early_decision=False) and
    must give the same DataFrame."""
    import torch
    args = (k, n, m, cc["gen1"], cc["gen2"], num_iter, list(p_grid), learn_len, 200, 1.0, seed)

    def timed(early, chunk=None):
        old = os.environ.get("CVD_CHUNK")
        if chunk is not None:
            os.environ["CVD_CHUNK"] = str(chunk)
        try:
            t0 = time.perf_counter()
            df = pkg.run_experiment(*args, N_list=[N], early_decision=early)
            torch.cuda.synchronize()
            return df, time.perf_counter() - t0, pkg._lib.chunk_last()
        finally:
            if chunk is not None:
                if old is None:
                    os.environ.pop("CVD_CHUNK", None)
                else:
                    os.environ["CVD_CHUNK"] = old

    df1, t_first, _ = timed(False)
    df2, t_second, ck = timed(False)                 # chunked, the default
    df_seq, t_seq, _ = timed(False, chunk=0)         # one lane per sequence, for comparison
    df_early, t_early, _ = timed(True)               # run_experiment's default: early decision
    trials = num_iter * len(p_grid)
    return {"call": f"run_experiment(num_iter={num_iter}, p_vec={list(p_grid)}, N_list=[{N}], learn_len={learn_len})",
            "trials": trials, "first_call_s_incl_setup": t_first, "second_call_s": t_second,
            "trials_per_s_second_call": trials / t_second, "chunked": ck,
            "unchunked_second_call_s": t_seq, "early_decision_second_call_s": t_early,
            "note": "second_call_s: every step of every trial (early_decision=False), chunked launches; "
                    "unchunked: CVD_CHUNK=0 (one lane per sequence); early_decision: run_experiment's "
                    "default (counts only, each trial stops once certain); all four DataFrames equal",
            "dataframes_equal": bool(df1.equals(df2) and df2.equals(df_seq) and df2.equals(df_early)),
            "rows": df2.to_dict(orient="records")}


if __name__ == "__main__":
    main()
