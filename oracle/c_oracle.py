"""ctypes binding of oracle/_build/liboracle.so (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use it."""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_PATH = os.path.join(_HERE, "_build", "liboracle.so")
_L = None


class oc_code(ctypes.Structure):
    _fields_ = [("k", ctypes.c_int32), ("n", ctypes.c_int32), ("m", ctypes.c_int32),
                ("taps", ctypes.POINTER(ctypes.c_uint8))]


def lib():
    global _L
    if _L is None:
        if not os.path.exists(_PATH):
            subprocess.check_call(["make", "-s", "-C", _HERE])
        L = ctypes.CDLL(_PATH)
        L.oc_model_create.restype = ctypes.c_void_p
        L.oc_model_create.argtypes = [ctypes.POINTER(oc_code), ctypes.c_double, ctypes.c_int64,
                                      ctypes.c_int64, ctypes.c_double, ctypes.c_uint64,
                                      ctypes.c_int64, ctypes.c_int64, ctypes.c_int64]
        L.oc_model_S.restype = ctypes.c_int64
        L.oc_model_S.argtypes = [ctypes.c_void_p]
        L.oc_model_kind.argtypes = [ctypes.c_void_p]
        L.oc_model_learn_len.restype = ctypes.c_int64
        L.oc_model_learn_len.argtypes = [ctypes.c_void_p]
        L.oc_model_rows.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        L.oc_model_destroy.argtypes = [ctypes.c_void_p]
        L.oc_run_trials.argtypes = [ctypes.c_void_p, ctypes.POINTER(oc_code), ctypes.POINTER(oc_code),
                                    ctypes.c_int64, ctypes.c_double, ctypes.c_uint64, ctypes.c_int64,
                                    ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        L.oc_stream.argtypes = [ctypes.POINTER(oc_code), ctypes.c_int64, ctypes.c_double,
                                ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_void_p]
        L.oc_grid_tag.restype = ctypes.c_uint32
        L.oc_grid_tag.argtypes = [ctypes.c_int64, ctypes.c_double]
        _L = L
    return _L


class Code:
    def __init__(self, gen, m, k, n):
        t = np.zeros((n, k, m + 1), np.uint8)
        for j in range(n):
            for i in range(k):
                v = list(gen[j][i])[: m + 1]
                t[j, i, : len(v)] = v
        self.taps = t
        self.c = oc_code(k, n, m, t.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)))
        self.k, self.n, self.m = k, n, m


class Model:
    def __init__(self, dec, p, learn_len=None, learn_burn=200, laplace=1.0, seed=12345,
                 enum_cap=500_000, sparse_default_len=1_000_000, laplace_states=0):
        self.dec = dec
        self.h = lib().oc_model_create(ctypes.byref(dec.c), p, -1 if learn_len is None else learn_len,
                                       learn_burn, laplace, seed, enum_cap, sparse_default_len,
                                       int(laplace_states or 0))

    @property
    def S(self):
        return lib().oc_model_S(self.h)

    @property
    def kind(self):
        return lib().oc_model_kind(self.h)

    def rows(self):
        S, R, M = self.S, 1 << self.dec.n, 1 << self.dec.m
        lp = np.zeros((S, R)); keys = np.zeros((S, M), np.uint8)
        lib().oc_model_rows(self.h, lp.ctypes.data, keys.ctypes.data)
        return lp, keys

    def run_trials(self, enc1, enc2, N, p, seed, t0, t1, sums=False, nthreads=0):
        counts = np.zeros(2, np.int64)
        out = np.zeros((t1 - t0, 4)) if sums else None
        lib().oc_run_trials(self.h, ctypes.byref(enc1.c), ctypes.byref(enc2.c), N, p, seed, t0, t1,
                            out.ctypes.data if sums else None, counts.ctypes.data, nthreads)
        return counts, out

    def __del__(self):
        if getattr(self, "h", None):
            lib().oc_model_destroy(self.h)
            self.h = None


def stream(enc, N, p, seed, tag, sid):
    out = np.zeros(N, np.int32)
    lib().oc_stream(ctypes.byref(enc.c), N, p, seed, tag, sid, out.ctypes.data)
    return out.astype(np.int64)


def max_threads():
    return lib().oc_max_threads()
