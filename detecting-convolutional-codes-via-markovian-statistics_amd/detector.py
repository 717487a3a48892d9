"""Host driver of the MI355X detector, mirroring the reference's call surface.

Reference (So-bonkers/Detecting-Convolutional-Codes-Via-Markovian-Statistics):
  Pd_plotter.run_experiment(k, n, m, gen1, gen2, num_iter, p_vec, learn_len,
                            learn_burn, laplace, seed) -> DataFrame[N, p, Pd, Pc]
                                                                    (Pd_plotter.py:176-235)
  Pd_plotter.learn_P1_empirical(...)                               (Pd_plotter.py:123-169)
  viterbi_markov.enumerate_markov_states_allzero / build_trellis /
  viterbi_metric_step / branch_output_and_next_state               (viterbi_markov.py:82-195)
  viterbi_markov.simulate_markov_sequence (missing; spec SURVEY.md §8 A5)

The trial loop (Pd_plotter.py:198-233) runs on the GPU through libcvd.so:
cvd_generate (encoder + BSC into bit-packed HBM streams) and cvd_detect
(Eq. 4-5 recursion + log-likelihood sums + decisions + counts).  There is no
CPU fallback: without a GPU or without libcvd.so the calls raise.
"""
import ctypes
import hashlib
import itertools
import os
import warnings
from collections import OrderedDict

import numpy as np
import torch

from . import _lib
from .codes import Code, as_code

# Pd_plotter.py:67-83
DEFAULTS = {
    "num_iter": 10000,
    "p_vec": [0.001, 0.01, 0.1, 0.2, 0.3, 0.4, 0.5],
    "seed": 12345,
    "learn_len": None,
    "learn_burn": 200,
    "laplace": 1.0,
    "save_dir": "results_experiments",
}
N_SPECTRUM_BY_M = {1: [5, 10, 20, 50, 100, 200], 2: [500], 3: [500], 4: [50, 100, 200, 300, 500]}

# Non-enumerable codes (m = 6: > 2e8 metric states) learn on a chain of this
# length when learn_len is None; the reference's max(5000, 200*S) needs S.
DEFAULT_ENUM_CAP = 500_000
DEFAULT_SPARSE_LEARN_LEN = 1_000_000


LEARN_TAG = 0xC0DE1EA7   # CVD_LEARN_TAG: stream tag of the P̂1 learning chain


def grid_tag(N, p):
    """Stream tag of an (N, p) grid point (cvd_grid_tag)."""
    return int(_lib.lib().cvd_grid_tag(int(N), float(p)))


def _require_gpu(device):
    if not torch.cuda.is_available():
        raise RuntimeError("the detector runs on the GPU (HIP); no GPU is visible")
    return torch.device("cuda", torch.cuda.current_device() if device is None else device)


def _stream_ptr(stream=None):
    s = torch.cuda.current_stream() if stream is None else stream
    return ctypes.c_void_p(s.cuda_stream)


def model_cache_dir(explicit=None):
    """Directory of the on-disk model cache: `explicit`, else $CVD_MODEL_CACHE; None
    (no cache) when neither is set or the value is "off"."""
    d = explicit if explicit is not None else os.environ.get("CVD_MODEL_CACHE")
    if not d or d == "off":
        return None
    os.makedirs(d, exist_ok=True)
    return d


def model_cache_key(dec, p, learn_len, learn_burn, laplace, seed, enum_cap, default_learn_len, laplace_states=None):
    """File name of a learned model: a hash of everything the learning depends on,
    the reference's lru_cache key (Pd_plotter.py:123-127: gens, k, n, m, p,
    learn_len, learn_burn, laplace, seed) plus this build's enumeration policy and
    stream spec."""
    key = (dec.key, float(p).hex(), learn_len, int(learn_burn), float(laplace).hex(), int(seed),
           int(enum_cap), int(default_learn_len), _lib.ABI_VERSION, "philox4x32-10/D1-D4")
    if laplace_states:
        key = key + (int(laplace_states),)
    txt = repr(key)
    return "cvdm_" + hashlib.sha256(txt.encode()).hexdigest()[:40] + ".bin"


class Model:
    """Decoder trellis (G1) + learned P̂1 + T_ref(1/2) tables (a cvd_model)."""

    def __init__(self, dec, p, learn_len=None, learn_burn=200, laplace=1.0, seed=12345,
                 enum_cap=DEFAULT_ENUM_CAP, default_learn_len=DEFAULT_SPARSE_LEARN_LEN, cache_dir=None,
                 learn_device=None, laplace_states=None):
        """learn_device: run the learning chain on this GPU (cvd_model_create_device,
        bit-identical to the host chain); None: on the host (cvd_model_create).
        laplace_states (non-enumerable codes): the S of the reference's Laplace
        denominator S * laplace (Pd_plotter.py:166-167), e.g. the certified lower bound
        enumerate_states_device gives for m = 6; None: the visited rows."""
        self.dec = dec
        self.p = float(p)
        self._lib = _lib.lib()
        self.from_cache = False
        self.learn_stats = None
        path = None
        d = model_cache_dir(cache_dir)
        if d is not None:
            path = os.path.join(d, model_cache_key(dec, p, learn_len, learn_burn, laplace, seed, enum_cap,
                                                   default_learn_len, laplace_states))
            if os.path.exists(path):
                h = ctypes.c_void_p()
                if self._lib.cvd_model_load(path.encode(), ctypes.byref(h)) == 0:
                    self._h = h
                    if self.code_key() == dec.key:
                        self.from_cache = True
                        return
                    self._lib.cvd_model_destroy(h)   # a stale file under this key: learn again
                    self._h = None
        prm = _lib.cvd_learn_params(float(p), -1 if learn_len is None else int(learn_len),
                                    int(learn_burn), float(laplace), int(seed) & 0xFFFFFFFFFFFFFFFF,
                                    int(enum_cap), int(default_learn_len), int(laplace_states or 0))
        h = ctypes.c_void_p()
        if learn_device is None:
            _lib.check(self._lib.cvd_model_create(dec.c, ctypes.byref(prm), ctypes.byref(h)))
        else:
            st = (ctypes.c_double * 7)()
            _lib.check(self._lib.cvd_model_create_device(dec.c, ctypes.byref(prm), int(learn_device), None,
                                                         ctypes.byref(h), ctypes.cast(st, ctypes.c_void_p)))
            self.learn_stats = dict(zip(("seconds", "mismatched_blocks", "fix_passes", "sequential_blocks",
                                         "hash_attempts", "host_fallback", "sequential_seconds"), list(st)))
        self._h = h
        if path is not None:
            # best effort: a cache that cannot be written (read-only or full disk) never
            # fails the run; concurrent writers are safe (unique tmp + atomic rename)
            if self._lib.cvd_model_save(self._h, path.encode()) != 0:
                warnings.warn(f"model cache not written ({path}): "
                              f"{self._lib.cvd_last_error().decode(errors='replace')}", RuntimeWarning, stacklevel=2)

    def save(self, path):
        _lib.check(self._lib.cvd_model_save(self._h, os.fspath(path).encode()))

    @classmethod
    def load(cls, dec, path):
        """A model written by save() (host tables; call upload(device) before use)."""
        self = cls.__new__(cls)
        self.dec, self._lib, self.from_cache = dec, _lib.lib(), True
        h = ctypes.c_void_p()
        _lib.check(self._lib.cvd_model_load(os.fspath(path).encode(), ctypes.byref(h)))
        self._h = h
        self.p = float("nan")
        if self.code_key() != dec.key:
            raise _lib.CvdError(f"model file {os.fspath(path)} was learned for another code "
                                f"(k, n, m, taps) than {dec!r}")
        return self

    def code_key(self):
        """(k, n, m, taps bytes) of the model's decoder, comparable with Code.key."""
        inf = self.info()
        k, n, m = inf["k"], inf["n"], inf["m"]
        taps = np.zeros(n * k * (m + 1), np.uint8)
        _lib.check(self._lib.cvd_model_taps(self._h, taps.ctypes.data, taps.size))
        return (k, n, m, taps.tobytes())

    @property
    def handle(self):
        return self._h

    def info(self):
        inf = _lib.cvd_model_info()
        _lib.check(self._lib.cvd_model_info_get(self._h, ctypes.byref(inf)))
        return {f: getattr(inf, f) for f, _ in inf._fields_}

    def dense_P1(self):
        S = self.info()["S"]
        P = np.zeros((S, S), np.float64)
        _lib.check(self._lib.cvd_model_dense_P1(self._h, P.ctypes.data, S))
        return P

    def rows(self):
        inf = self.info()
        R, M = 1 << inf["n"], 1 << inf["m"]
        lp = np.zeros((inf["n_rows"], R), np.float64)
        keys = np.zeros((inf["n_rows"], M), np.uint8)
        _lib.check(self._lib.cvd_model_rows(self._h, lp.ctypes.data, keys.ctypes.data, inf["n_rows"]))
        return lp, keys

    def upload(self, device):
        _lib.check(self._lib.cvd_model_upload(self._h, int(device)))
        st, msg = self.jit_status()
        if st < 0:
            warnings.warn("code-specialised detector kernel unavailable, running the table-driven "
                          f"butterfly kernel (same results, slower): {msg}", RuntimeWarning, stacklevel=2)
        return self

    def device_error(self):
        """Raise if a launch on this model set a kernel error flag since the last check
        (cvd_model_device_error: walk mode's scheduler guard; synchronises the device)."""
        flags = ctypes.c_int32()
        _lib.check(self._lib.cvd_model_device_error(self._h, ctypes.byref(flags)))
        return int(flags.value)

    def jit_status(self):
        """(1 built | -1 unavailable | 0 not applicable, reason) of the code-specialised kernel."""
        buf = ctypes.create_string_buffer(4096)
        st = self._lib.cvd_model_jit_status(self._h, buf, len(buf))
        return st, buf.value.decode(errors="replace")

    def __del__(self):
        h = getattr(self, "_h", None)
        if h and h.value:
            try:
                self._lib.cvd_model_destroy(h)
            except Exception:
                pass
            self._h = None


class Detector:
    """One decoder (G1) on one GPU; caches learned models per (p, learning args)
    like the reference's @lru_cache(maxsize=128) (Pd_plotter.py:123)."""

    def __init__(self, k, n, m, gen1, device=None, enum_cap=DEFAULT_ENUM_CAP,
                 default_learn_len=DEFAULT_SPARSE_LEARN_LEN, model_cache=None):
        self.k, self.n, self.m = int(k), int(n), int(m)
        self.dec = as_code(gen1, m, k, n)
        self.device = _require_gpu(device)
        self.enum_cap = enum_cap
        self.default_learn_len = default_learn_len
        self.model_cache = model_cache   # on-disk cache dir (None: $CVD_MODEL_CACHE if set)
        # the learning chain runs on this GPU (bit-identical to the host chain);
        # CVD_LEARN_HOST=1 keeps it on the host
        self.learn_device = None if os.environ.get("CVD_LEARN_HOST", "0") not in ("", "0") else self.device.index
        self._models = OrderedDict()

    def model(self, p, learn_len=None, learn_burn=200, laplace=1.0, seed=12345, laplace_states=None):
        key = (float(p), learn_len, int(learn_burn), float(laplace), int(seed), laplace_states)
        if key in self._models:
            self._models.move_to_end(key)
            return self._models[key]
        mod = Model(self.dec, p, learn_len, learn_burn, laplace, seed, self.enum_cap,
                    self.default_learn_len, self.model_cache, self.learn_device,
                    laplace_states).upload(self.device.index)
        self._models[key] = mod
        while len(self._models) > 128:
            self._models.popitem(last=False)
        return mod

    def prepare_models(self, p_list, learn_len=None, learn_burn=200, laplace=1.0, seed=12345, workers=None):
        """Learn the models of several p at once (host threads; cvd_model_create
        runs without the GIL), then upload them in order.  The learning chain of
        one model is sequential, so a p sweep's setup costs about its slowest
        model instead of the sum."""
        from concurrent.futures import ThreadPoolExecutor
        keys = {}
        for p in p_list:
            key = (float(p), learn_len, int(learn_burn), float(laplace), int(seed), None)
            if key not in self._models:
                keys[key] = float(p)
        if len(keys) > 1:
            nw = workers or min(len(keys), 8)
            with ThreadPoolExecutor(max_workers=nw) as ex:
                built = list(ex.map(lambda p: Model(self.dec, p, learn_len, learn_burn, laplace, seed,
                                                    self.enum_cap, self.default_learn_len, self.model_cache,
                                                    self.learn_device),
                                    keys.values()))
            for key, mod in zip(keys, built):
                self._models[key] = mod.upload(self.device.index)
        return [self.model(p, learn_len, learn_burn, laplace, seed) for p in p_list]

    def words_per_seq(self, N):
        """Received words per sequence, padded to whole 16-byte chunks."""
        spw = 32 // self.n
        return ((int(N) + spw - 1) // spw + 3) // 4 * 4

    def stream_buffer(self, N, pitch):
        """Device buffer for `pitch` sequences: [W/4, pitch, 4] words (include/cvd.h layout)."""
        return torch.empty((self.words_per_seq(N) // 4, int(pitch), 4), dtype=torch.int32, device=self.device)

    def generate(self, enc, N, p, seed, tag, seq_base, seq_stride, count, out=None, q0=0, pitch=None,
                 random_input=True, stream=None):
        """Received words (int32 view of uint32) [W/4, pitch, 4] for `count` sequences."""
        enc = as_code(enc, self.m, self.k, self.n)
        pitch = count if pitch is None else pitch
        if out is None:
            out = self.stream_buffer(N, pitch)
        _lib.check(_lib.lib().cvd_generate(enc.c, int(seed) & 0xFFFFFFFFFFFFFFFF, int(tag), float(p),
                                           int(N), int(bool(random_input)), int(seq_base),
                                           int(seq_stride), ctypes.c_void_p(out.data_ptr()), int(pitch),
                                           int(q0), int(count), _stream_ptr(stream)))
        return out

    def detect(self, model, r, N, nseq, n_h1, sums=None, counts=None, path=_lib.PATH_AUTO, stream=None,
               early_decision=False):
        """early_decision: counts only; a trial stops once its decision is certain
        (CVD_DETECT_EARLY_DECISION; same counts, no sums)."""
        if counts is None:
            counts = torch.zeros(2, dtype=torch.int64, device=self.device)
        if early_decision:
            path = int(path) | _lib.DETECT_EARLY_DECISION
        _lib.check(_lib.lib().cvd_detect(model.handle, ctypes.c_void_p(r.data_ptr()), int(N), int(nseq),
                                         int(n_h1),
                                         ctypes.c_void_p(sums.data_ptr() if sums is not None else 0),
                                         ctypes.c_void_p(counts.data_ptr()), int(path),
                                         _stream_ptr(stream)))
        return counts

    def detect_multi(self, models, bufs, N, nseq, n_h1, counts, sums=None, path=_lib.PATH_AUTO, stream=None,
                     early_decision=False):
        """len(models) detect() calls in as few launches as possible (cvd_detect_multi):
        model i over stream buffer bufs[i] (nseq[i] sequences, the first n_h1[i] H1),
        accumulating counts[i] (and sums[i] if given); models that share the specialised
        kernel variant run in one launch, so a p sweep pays one last-round tail."""
        k = len(models)
        if not (len(bufs) == len(nseq) == len(n_h1) == len(counts) == k) or (sums is not None and len(sums) != k):
            raise ValueError("one buffer, nseq, n_h1 and counts entry per model")
        if early_decision:
            path = int(path) | _lib.DETECT_EARLY_DECISION
        P = ctypes.c_void_p * max(k, 1)
        hs = P(*[m.handle.value for m in models])
        rs = P(*[r.data_ptr() for r in bufs])
        cs = P(*[c.data_ptr() for c in counts])
        ss = P(*[(x.data_ptr() if x is not None else 0) for x in sums]) if sums is not None else None
        nv = (ctypes.c_int64 * max(k, 1))(*[int(x) for x in nseq])
        hv = (ctypes.c_int64 * max(k, 1))(*[int(x) for x in n_h1])
        _lib.check(_lib.lib().cvd_detect_multi(hs, k, rs, int(N), nv, hv, ss, cs, int(path), _stream_ptr(stream)))
        return counts

    @staticmethod
    def multi_groups(models, nseq=None):
        """Index runs of `models` that cvd_detect_multi merges into one launch (the same
        specialised kernel variant, as the library reports it: cvd_model_info.multi_variant;
        at most 8 per launch; a model whose launch over nseq[i] sequences is persistent,
        nseq[i] > cvd_model_info.persist_seqs > 0, alone) -- for per-launch timing."""
        groups, cur, key = [], [], None
        for i, m in enumerate(models):
            inf = m.info()
            k = inf["multi_variant"] or None
            if k is not None and nseq is not None and 0 < inf["persist_seqs"] < int(nseq[i]):
                k = None
            if cur and (k is None or k != key or len(cur) == 8 or os.environ.get("CVD_NO_MULTI")):
                groups.append(cur)
                cur = []
            cur.append(i)
            key = k
        if cur:
            groups.append(cur)
        return groups

    def trace(self, model, r, N, nseq, stream=None):
        """D_0..D_N of every sequence on the explicit path: uint8 [N+1, nseq, 2^m]."""
        D = torch.empty((int(N) + 1, int(nseq), 1 << self.m), dtype=torch.uint8, device=self.device)
        _lib.check(_lib.lib().cvd_trace(model.handle, ctypes.c_void_p(r.data_ptr()), int(N), int(nseq),
                                        ctypes.c_void_p(D.data_ptr()), _stream_ptr(stream)))
        return D

    # one residency round of the butterfly kernel: 4 waves/SIMD x 1024 SIMDs x 64
    # lanes = 262,144 sequences = 131,072 trials (H1 + H2)
    FULL_ROUND_TRIALS = 131_072

    def default_batch(self, N, trial_count, budget_bytes=None):
        """Trials per launch: as many as a third of the free HBM (at most 96 GiB)
        holds, rounded down to whole residency rounds when that is >= one round."""
        per_trial = 2 * self.words_per_seq(N) * 4
        if budget_bytes is None:
            free, _ = torch.cuda.mem_get_info(self.device)
            budget_bytes = min(free // 3, 96 << 30)
        b = max(1024, budget_bytes // max(per_trial, 1))
        if b >= self.FULL_ROUND_TRIALS:
            b -= b % self.FULL_ROUND_TRIALS
        return int(max(1, min(trial_count, b)))

    def run_trials(self, model, gen1, gen2, N, p, seed, trial_begin, trial_end, batch=None,
                   path=_lib.PATH_AUTO, return_sums=False, counts=None, stream=None, early_decision=False,
                   fused=False, check=None):
        """Global trials [trial_begin, trial_end) of one (N, p) grid point
        (Pd_plotter.py:198-223).  Returns {"counts": (s1, s2), "sums": [T, 4]?}
        with sums per trial = (logp1, logp1_ref, logp2, logp2_ref).
        early_decision (counts only): stop each trial once its decision is certain.
        fused: generator and table automaton in one kernel (cvd_mc_fused; dense
        LDS-resident models), sums included; the counts-only path uses it on its own
        (cvd_mc_run, PATH_AUTO) whenever it applies.
        check: read the model's kernel error flags afterwards (cvd_model_device_error,
        which synchronises) and raise if a launch set one; default: when sums are returned
        (the call synchronises anyway), not for counts-only calls, whose caller checks once
        after its launches (model.device_error())."""
        if check is None:
            check = return_sums
        if early_decision and return_sums:
            raise ValueError("early_decision gives counts only; per-trial sums need the full run")
        g1 = as_code(gen1, self.m, self.k, self.n)
        g2 = as_code(gen2, self.m, self.k, self.n)
        T = int(trial_end) - int(trial_begin)
        if counts is None:
            counts = torch.zeros(2, dtype=torch.int64, device=self.device)
        if T <= 0:
            return {"counts": counts, "sums": np.zeros((0, 4))} if return_sums else {"counts": counts}
        if fused:
            sums = torch.full((T, 4), float("nan"), dtype=torch.float64, device=self.device) if return_sums else None
            flags = _lib.DETECT_EARLY_DECISION if early_decision else 0
            _lib.check(_lib.lib().cvd_mc_fused(model.handle, g1.c, g2.c, float(p), int(N),
                                               int(seed) & 0xFFFFFFFFFFFFFFFF, int(trial_begin), int(trial_end),
                                               ctypes.c_void_p(sums.data_ptr() if sums is not None else 0),
                                               ctypes.c_void_p(counts.data_ptr()), flags, _stream_ptr(stream)))
            if check:
                model.device_error()
            if return_sums:
                return {"counts": counts, "sums": sums.cpu().numpy()}
            return {"counts": counts}
        batch = self.default_batch(N, T) if batch is None else int(batch)
        lib = _lib.lib()
        if not return_sums:
            # the fused kernel (PATH_AUTO on an mc_fused model) needs no stream workspace
            fused_auto = int(path) == _lib.PATH_AUTO and bool(model.info()["mc_fused"])
            work = None
            if not fused_auto:
                wsz = lib.cvd_mc_workspace_bytes(g1.c, int(N), batch)
                work = torch.empty(max(wsz, 4) // 4, dtype=torch.int32, device=self.device)
            flags = _lib.DETECT_EARLY_DECISION if early_decision else 0
            _lib.check(lib.cvd_mc_run(model.handle, g1.c, g2.c, float(p), int(N),
                                      int(seed) & 0xFFFFFFFFFFFFFFFF, int(trial_begin), int(trial_end),
                                      batch, ctypes.c_void_p(work.data_ptr() if work is not None else 0),
                                      ctypes.c_void_p(counts.data_ptr()), int(path) | flags, _stream_ptr(stream)))
            if check:
                model.device_error()
            return {"counts": counts}
        tag = grid_tag(N, p)
        out = []
        for b in range(int(trial_begin), int(trial_end), batch):
            Tb = min(batch, int(trial_end) - b)
            r = self.stream_buffer(N, 2 * Tb)
            self.generate(g1, N, p, seed, tag, 2 * b, 2, Tb, out=r, q0=0, pitch=2 * Tb, stream=stream)
            self.generate(g2, N, p, seed, tag, 2 * b + 1, 2, Tb, out=r, q0=Tb, pitch=2 * Tb, stream=stream)
            # NaN-filled: a sequence the kernel never wrote cannot pass for a result (the
            # allocator hands back the previous call's buffer)
            sums = torch.full((2 * Tb, 2), float("nan"), dtype=torch.float64, device=self.device)
            self.detect(model, r, N, 2 * Tb, Tb, sums=sums, counts=counts, path=path, stream=stream)
            s = sums.cpu().numpy()
            out.append(np.concatenate([s[:Tb], s[Tb:]], axis=1))
        if check:
            model.device_error()
        return {"counts": counts, "sums": np.concatenate(out, axis=0)}


    def run_grid(self, models, gen1, gen2, p_list, N_list, seed, trial_begin, trial_end, batch=None,
                 path=_lib.PATH_AUTO, counts=None, stream=None, early_decision=False, budget=None):
        """The (N, p) grid of Pd_plotter.py:196-233 in ONE library call (cvd_mc_run_grid,
        SURVEY.md §8(b)): models[i] learned at p_list[i]; global trials [trial_begin,
        trial_end) at every point; returns the int64 counts [len(N_list), len(p_list), 2].

        `batch` is trials per launch PER GRID POINT of a p row: the p row's batches are
        generated into one stream slot each, so the workspace is about len(p_list) times one
        point's.  An explicit batch is clamped so that the workspace stays within `budget`
        bytes (default: the free-memory budget batch=None uses; clamp_grid_batch)."""
        g1 = as_code(gen1, self.m, self.k, self.n)
        g2 = as_code(gen2, self.m, self.k, self.n)
        npn, nN = len(p_list), len(N_list)
        if len(models) != npn:
            raise ValueError("one model per p")
        if counts is None:
            counts = torch.zeros((nN, npn, 2), dtype=torch.int64, device=self.device)
        T = int(trial_end) - int(trial_begin)
        if T <= 0:
            return counts
        if budget is None:
            free, _ = torch.cuda.mem_get_info(self.device)
            budget = min(free // 3, 96 << 30)
        if batch is None:
            # the p row's batches share the HBM budget (one stream slot per point)
            batch = self.default_batch(max(N_list), T, budget // max(1, npn))
        hs = (ctypes.c_void_p * npn)(*[m.handle.value for m in models])
        pv = (ctypes.c_double * npn)(*[float(p) for p in p_list])
        Nv = (ctypes.c_int64 * nN)(*[int(N) for N in N_list])
        lib = _lib.lib()
        flags = _lib.DETECT_EARLY_DECISION if early_decision else 0
        batch = clamp_grid_batch(models, g1, N_list, batch, int(path) | flags, budget)
        wsz = lib.cvd_mc_grid_workspace_bytes(hs, npn, g1.c, Nv, nN, batch, int(path) | flags)
        if wsz < 0:
            raise _lib.CvdError("cvd_mc_grid_workspace_bytes: bad arguments")
        work = torch.empty(max(wsz, 4) // 4, dtype=torch.int32, device=self.device) if wsz > 0 else None
        _lib.check(lib.cvd_mc_run_grid(hs, g1.c, g2.c, pv, npn, Nv, nN, int(seed) & 0xFFFFFFFFFFFFFFFF,
                                       int(trial_begin), int(trial_end), batch,
                                       ctypes.c_void_p(work.data_ptr() if work is not None else 0),
                                       ctypes.c_void_p(counts.data_ptr()), int(path) | flags, _stream_ptr(stream)))
        return counts


def grid_workspace_bytes(models, g1, N_list, batch, flags):
    """cvd_mc_grid_workspace_bytes of a p row of `models` (host call, no GPU needed)."""
    npn, nN = len(models), len(N_list)
    hs = (ctypes.c_void_p * npn)(*[m.handle.value for m in models])
    Nv = (ctypes.c_int64 * nN)(*[int(N) for N in N_list])
    wsz = _lib.lib().cvd_mc_grid_workspace_bytes(hs, npn, g1.c, Nv, nN, int(batch), int(flags))
    if wsz < 0:
        raise _lib.CvdError("cvd_mc_grid_workspace_bytes: bad arguments")
    return int(wsz)


def clamp_grid_batch(models, g1, N_list, batch, flags, budget):
    """The largest batch <= `batch` whose grid workspace (one stream slot per p of the row)
    fits `budget` bytes (at least 1 trial): the per-point batch a caller gives would
    otherwise cost len(models) times its slot."""
    batch = max(1, int(batch))
    while batch > 1 and grid_workspace_bytes(models, g1, N_list, batch, flags) > budget:
        batch = max(1, batch * budget // max(1, grid_workspace_bytes(models, g1, N_list, batch, flags)) - 1)
    return batch


# ───────────────────── reference-mirroring functions ────────────────────────

_DETECTORS = {}


def _detector(k, n, m, gen1, device=None):
    code = as_code(gen1, m, k, n)
    key = (code.key, device)
    if key not in _DETECTORS:
        _DETECTORS[key] = Detector(k, n, m, code, device=device)
    return _DETECTORS[key]


def run_experiment(k, n, m, gen1, gen2, num_iter, p_vec, learn_len, learn_burn, laplace, seed,
                   N_list=None, device=None, batch=None, path=_lib.PATH_AUTO, early_decision=True):
    """Drop-in for Pd_plotter.run_experiment (Pd_plotter.py:176-235).

    Extra keyword arguments: N_list (defaults to the reference's
    N_SPECTRUM_BY_M.get(m, [50, 100, 200]), Pd_plotter.py:196), device, batch,
    path, early_decision (default on: the table needs only each trial's
    decision, so a trial stops once it is certain -- identical Pd/Pc, see
    CVD_DETECT_EARLY_DECISION).  When a torch.distributed default group is initialised (one process
    per GPU), trials are sharded by global trial id over the ranks and the
    success counts reduced with ONE all_reduce (RCCL on ROCm); every rank
    returns the same DataFrame.
    """
    import pandas as pd
    from .distributed import run_sharded_grid, pd_rows

    det = _detector(k, n, m, gen1, device)
    N_spectrum = list(N_SPECTRUM_BY_M.get(m, [50, 100, 200]) if N_list is None else N_list)

    models = det.prepare_models(list(p_vec), learn_len, learn_burn, laplace, seed)

    def grid_fn(lo, hi, out):
        # the whole (N, p) grid of this rank's trial block in one library call
        # (cvd_mc_run_grid: per N, the p row's batches in multi-model launches)
        det.run_grid(models, gen1, gen2, list(p_vec), N_spectrum, seed, lo, hi, batch=batch, path=path,
                     counts=out, early_decision=early_decision)

    counts = run_sharded_grid(grid_fn, N_spectrum, list(p_vec), num_iter, det.device)
    for mdl in models:
        mdl.device_error()
    return pd.DataFrame(pd_rows(counts, N_spectrum, list(p_vec), num_iter))


def learn_P1_empirical(gens_tuple, k, n, m, p, learn_len, learn_burn, laplace, seed):
    """Mirror of Pd_plotter.py:123-169 for enumerable codes: (states, state_index, P)."""
    gen = [[list(x) for x in row] for row in gens_tuple]
    mod = Model(Code(gen, m, k, n), p, learn_len, learn_burn, laplace, seed)
    if mod.info()["kind"] != 0:
        raise _lib.CvdError("learn_P1_empirical: code is not enumerable; use Detector.model()")
    _, keys = mod.rows()
    states = [tuple(int(v) for v in row) for row in keys]
    return states, {s: i for i, s in enumerate(states)}, mod.dense_P1()


def enumerate_markov_states_allzero(generator_matrix, m, k, n, cap=DEFAULT_ENUM_CAP):
    """Mirror of viterbi_markov.py:166-195 (native BFS): (states, transitions, all_r)."""
    code = as_code(generator_matrix, m, k, n)
    lib = _lib.lib()
    S = ctypes.c_int64()
    _lib.check(lib.cvd_enumerate(code.c, int(cap), ctypes.byref(S), None, None))
    M, R = 1 << m, 1 << n
    st = np.zeros((S.value, M), np.uint8)
    nx = np.zeros((S.value, R), np.int32)
    _lib.check(lib.cvd_enumerate(code.c, int(cap), ctypes.byref(S), st.ctypes.data, nx.ctypes.data))
    all_r = list(itertools.product([0, 1], repeat=n))
    states = [tuple(int(v) for v in row) for row in st]
    transitions = {}
    for i in range(S.value):
        d = {}
        for ri, r in enumerate(all_r):
            rint = sum(b << j for j, b in enumerate(r))
            d.setdefault(int(nx[i, rint]), []).append(r)
        transitions[i] = d
    return states, transitions, all_r


def enumerate_states_device(generator_matrix, m, k, n, device=0, cap=1 << 40, mem_bytes=0, with_tables=False,
                            max_levels=1 << 16):
    """viterbi_markov.py:166-195 on the GPU (cvd_enumerate_device).

    Returns {"S", "complete", "level_sizes", "states"?, "next"?}: complete = False when
    the state count passed `cap` or the device memory budget, and S is then a certified
    lower bound (distinct reachable states found).  with_tables: also the states in
    discovery order ([S, 2^m] uint8) and next[S, 2^n] (int32, by received word)."""
    code = as_code(generator_matrix, m, k, n)
    lib = _lib.lib()
    S = ctypes.c_int64()
    nl = ctypes.c_int32()
    lv = np.zeros(max_levels, np.int64)
    rc = lib.cvd_enumerate_device(code.c, int(device), int(cap), int(mem_bytes), ctypes.byref(S), None, None,
                                  lv.ctypes.data, int(max_levels), ctypes.byref(nl), None)
    if rc not in (0, -3):
        _lib.check(rc)
    if rc == -3 and S.value < 1:   # CVD_E_CAPACITY certifies S_out >= 1; anything else is a failure
        _lib.check(rc)
    out = {"S": int(S.value), "complete": rc == 0, "level_sizes": lv[:min(nl.value, max_levels)].tolist()}
    if with_tables and rc == 0:
        st = np.zeros((S.value, 1 << m), np.uint8)
        nx = np.zeros((S.value, 1 << n), np.int32)
        _lib.check(lib.cvd_enumerate_device(code.c, int(device), int(S.value), int(mem_bytes), ctypes.byref(S),
                                            st.ctypes.data, nx.ctypes.data, None, 0, ctypes.byref(nl), None))
        out["states"], out["next"] = st, nx
    return out


class Trellis(dict):
    """build_trellis result (viterbi_markov.py:118-132) that also carries the code."""

    def __init__(self, code):
        super().__init__()
        self.code = code
        out, nxt = code.tables()
        for ns in range(1 << code.m):
            self[ns] = []
        for s in range(1 << code.m):
            for U in range(1 << code.k):
                u = tuple((U >> i) & 1 for i in range(code.k))
                o = tuple((int(out[s, U]) >> j) & 1 for j in range(code.n))
                self[int(nxt[s, U])].append((s, u, o))


def build_trellis(generator_matrix, m, k, n=None):
    n = len(generator_matrix) if n is None else n
    return Trellis(as_code(generator_matrix, m, k, n))


def branch_output_and_next_state(state_int, input_bits, generator_matrix, m, k):
    code = as_code(generator_matrix, m, k, len(generator_matrix))
    out, nxt = code.tables()
    U = sum(int(b) << i for i, b in enumerate(input_bits))
    o = int(out[state_int, U])
    return tuple((o >> j) & 1 for j in range(code.n)), int(nxt[state_int, U])


def viterbi_metric_step(D_prev, trellis, y_t):
    """Mirror of viterbi_markov.py:139-159 (native host step)."""
    code = trellis.code
    D = np.asarray(D_prev, dtype=np.uint8)
    out = np.zeros(1 << code.m, np.uint8)
    r = sum(int(b) << j for j, b in enumerate(y_t))
    _lib.check(_lib.lib().cvd_metric_step(code.c, D.ctypes.data, r, out.ctypes.data))
    return tuple(int(v) for v in out)


def simulate_markov_sequence(generator_matrix, m, k, n, N, p_val, random_input=True, seed=None,
                             decoder=None, tag=LEARN_TAG, seq_id=0, device=None):
    """The reference's missing simulator (called at Pd_plotter.py:149-155, 212, 219),
    on the GPU: encoder -> BSC(p) (cvd_generate) -> D_0..D_N on trellis(decoder)
    (cvd_trace).  Returns {"metrics": [tuple, ...], "received": np.ndarray}."""
    dec = as_code(decoder if decoder is not None else generator_matrix, m, k, n)
    det = _detector(k, n, m, dec, device)
    model = det.model(0.0, learn_len=0, learn_burn=0, laplace=1.0, seed=0)
    sd = 0 if seed is None else int(seed)
    r = det.generate(generator_matrix, N, p_val, sd, tag, seq_id, 1, 1, random_input=random_input)
    D = det.trace(model, r, N, 1)[:, 0, :].cpu().numpy()
    spw = 32 // n
    words = r[:, 0, :].reshape(-1).cpu().numpy().astype(np.uint32)
    t = np.arange(N)
    recv = (words[t // spw] >> ((t % spw) * n).astype(np.uint32)) & ((1 << n) - 1)
    return {"metrics": [tuple(int(v) for v in row) for row in D], "received": recv.astype(np.int64)}


def log_likelihood_ratio(sums):
    """Λ_N = log P̂1(D_0^N) - log T_ref(D_0^N) per sequence (Pd_plotter.py:38)."""
    return sums[..., 0] - sums[..., 1]

