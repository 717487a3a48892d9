"""ctypes binding of libcvd.so (include/cvd.h).

torch is imported before the library is opened: libcvd.so needs
libamdhip64.so.7, and when torch has already loaded its own copy (same soname)
the dynamic linker binds libcvd.so to that one, so torch's device buffers and
streams and our kernels share one HIP runtime.
"""
import ctypes
import os

import torch  # noqa: F401  (load torch's HIP runtime first)

_HERE = os.path.dirname(os.path.abspath(__file__))
# CVD_LIB_PATH: another build of the same ABI (A/B builds, profiles/build_ab.sh)
LIB_PATH = os.environ.get("CVD_LIB_PATH") or os.path.join(_HERE, "lib", "libcvd.so")
ABI_VERSION = 11

PATH_AUTO, PATH_TABLE, PATH_EXPLICIT, PATH_EXPLICIT_GENERIC, PATH_EXPLICIT_ORBIT, PATH_EXPLICIT_BUTTERFLY = 0, 1, 2, 3, 4, 5
DETECT_EARLY_DECISION = 0x100   # OR'ed into path: counts only, stop once every decision is certain


class CvdError(RuntimeError):
    """Raised when a libcvd call returns a negative status."""


class cvd_code(ctypes.Structure):
    _fields_ = [("k", ctypes.c_int32), ("n", ctypes.c_int32), ("m", ctypes.c_int32),
                ("taps", ctypes.POINTER(ctypes.c_uint8))]


class cvd_learn_params(ctypes.Structure):
    _fields_ = [("p", ctypes.c_double), ("learn_len", ctypes.c_int64),
                ("learn_burn", ctypes.c_int64), ("laplace", ctypes.c_double),
                ("seed", ctypes.c_uint64), ("enum_cap", ctypes.c_int64),
                ("default_learn_len", ctypes.c_int64), ("laplace_states", ctypes.c_int64)]


class cvd_model_info(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int32), ("k", ctypes.c_int32), ("n", ctypes.c_int32),
                ("m", ctypes.c_int32), ("S", ctypes.c_int64), ("n_rows", ctypes.c_int64),
                ("learn_len_eff", ctypes.c_int64), ("hash_capacity", ctypes.c_int64),
                ("max_probe", ctypes.c_int32), ("device", ctypes.c_int32),
                ("logp1_unseen", ctypes.c_double), ("explicit_kernel", ctypes.c_int32),
                ("mc_fused", ctypes.c_int32), ("walk", ctypes.c_int32), ("lds_filter", ctypes.c_int32),
                ("walk_compact", ctypes.c_int32), ("multi_variant", ctypes.c_int64), ("persist_seqs", ctypes.c_int64)]


KERNEL_NAMES = {0: "none", 1: "detect_explicit_kernel (generic explicit path)",
                2: "detect_k1_kernel (k=1 orbit explicit path)",
                3: "detect_k1b_kernel (k=1 butterfly explicit path, table-driven)",
                4: "cvd_k1b_spec (k=1 butterfly explicit path, code-specialised at model upload)",
                5: "cvd_k1b_spec (m=6 bit-sliced form k1s, code-specialised at model upload)"}


EXPORTS = {
    # name: (restype, argtypes)
    "cvd_version": (ctypes.c_int, []),
    "cvd_last_error": (ctypes.c_char_p, []),
    "cvd_grid_tag": (ctypes.c_uint32, [ctypes.c_int64, ctypes.c_double]),
    "cvd_code_tables": (ctypes.c_int, [ctypes.POINTER(cvd_code), ctypes.c_void_p, ctypes.c_void_p]),
    "cvd_metric_step": (ctypes.c_int, [ctypes.POINTER(cvd_code), ctypes.c_void_p, ctypes.c_int32,
                                       ctypes.c_void_p]),
    "cvd_enumerate": (ctypes.c_int, [ctypes.POINTER(cvd_code), ctypes.c_int64,
                                     ctypes.POINTER(ctypes.c_int64), ctypes.c_void_p, ctypes.c_void_p]),
    "cvd_enumerate_device": (ctypes.c_int, [ctypes.POINTER(cvd_code), ctypes.c_int32, ctypes.c_int64, ctypes.c_int64,
                                            ctypes.POINTER(ctypes.c_int64), ctypes.c_void_p, ctypes.c_void_p,
                                            ctypes.c_void_p, ctypes.c_int32, ctypes.POINTER(ctypes.c_int32),
                                            ctypes.c_void_p]),
    "cvd_model_create": (ctypes.c_int, [ctypes.POINTER(cvd_code), ctypes.POINTER(cvd_learn_params),
                                        ctypes.POINTER(ctypes.c_void_p)]),
    "cvd_model_create_device": (ctypes.c_int, [ctypes.POINTER(cvd_code), ctypes.POINTER(cvd_learn_params),
                                               ctypes.c_int32, ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p),
                                               ctypes.c_void_p]),
    "cvd_model_info_get": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(cvd_model_info)]),
    "cvd_model_dense_P1": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64]),
    "cvd_model_rows": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64]),
    "cvd_model_taps": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64]),
    "cvd_model_upload": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "cvd_model_destroy": (None, [ctypes.c_void_p]),
    "cvd_model_save": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p]),
    "cvd_model_load": (ctypes.c_int, [ctypes.c_char_p, ctypes.POINTER(ctypes.c_void_p)]),
    "cvd_model_jit_status": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int64]),
    "cvd_allreduce_counts": (ctypes.c_int, [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int64, ctypes.c_int32,
                                            ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_void_p)]),
    "cvd_comm_unique_id": (ctypes.c_int, [ctypes.c_char_p]),
    "cvd_comm_init": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                     ctypes.POINTER(ctypes.c_void_p)]),
    "cvd_comm_allreduce_counts": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]),
    "cvd_comm_destroy": (None, [ctypes.c_void_p]),
    "cvd_generate": (ctypes.c_int, [ctypes.POINTER(cvd_code), ctypes.c_uint64, ctypes.c_uint32,
                                    ctypes.c_double, ctypes.c_int64, ctypes.c_int32, ctypes.c_int64,
                                    ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64,
                                    ctypes.c_int64, ctypes.c_void_p]),
    "cvd_detect": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64,
                                  ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32,
                                  ctypes.c_void_p]),
    "cvd_detect_multi": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_int64,
                                        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_int32, ctypes.c_void_p]),
    "cvd_trace": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64,
                                 ctypes.c_void_p, ctypes.c_void_p]),
    "cvd_mc_workspace_bytes": (ctypes.c_int64, [ctypes.POINTER(cvd_code), ctypes.c_int64, ctypes.c_int64]),
    "cvd_mc_run": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(cvd_code), ctypes.POINTER(cvd_code),
                                  ctypes.c_double, ctypes.c_int64, ctypes.c_uint64, ctypes.c_int64,
                                  ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p,
                                  ctypes.c_int32, ctypes.c_void_p]),
    "cvd_mc_grid_workspace_bytes": (ctypes.c_int64, [ctypes.c_void_p, ctypes.c_int32, ctypes.POINTER(cvd_code),
                                                     ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_int32]),
    "cvd_mc_run_grid": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(cvd_code), ctypes.POINTER(cvd_code),
                                       ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_int32,
                                       ctypes.c_uint64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
                                       ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p]),
    "cvd_model_device_error": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int32)]),
    "cvd_chunk_last": (ctypes.c_int, [ctypes.POINTER(ctypes.c_int64)]),
    "cvd_jit_prebuild": (ctypes.c_int, [ctypes.POINTER(cvd_code), ctypes.c_char_p, ctypes.c_char_p,
                                        ctypes.POINTER(ctypes.c_int32)]),
    "cvd_mc_fused": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(cvd_code), ctypes.POINTER(cvd_code),
                                    ctypes.c_double, ctypes.c_int64, ctypes.c_uint64, ctypes.c_int64,
                                    ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32,
                                    ctypes.c_void_p]),
    "cvd_parity_detect": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_int64,
                                         ctypes.c_int64, ctypes.c_void_p, ctypes.c_int32, ctypes.c_double,
                                         ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "cvd_count_transitions": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64,
                                             ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p]),
    "cvd_chernoff_build": (ctypes.c_int, [ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.c_double, ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p,
                                          ctypes.c_void_p, ctypes.c_void_p]),
    "cvd_chernoff_build_dense": (ctypes.c_int, [ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p,
                                                ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p]),
    "cvd_spectral_radius": (ctypes.c_int, [ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p,
                                           ctypes.c_void_p, ctypes.c_int32, ctypes.c_double, ctypes.c_int32,
                                           ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
}

_lib = None


def lib():
    """Open libcvd.so (fails loudly if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise CvdError(f"{LIB_PATH} is missing: run `python __graft_entry__.py` (build) first")
    L = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in EXPORTS.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    if L.cvd_version() != ABI_VERSION:
        raise CvdError(f"libcvd ABI {L.cvd_version()} != expected {ABI_VERSION}")
    _lib = L
    return L


def check(rc):
    if rc != 0:
        msg = lib().cvd_last_error().decode(errors="replace")
        raise CvdError(f"libcvd error {rc}: {msg}")
    return rc


def chunk_last():
    """The chunked launches of this process's last detect call (cvd_chunk_last): groups (0:
    the call ran unchunked), chunks per sequence C, steps per chunk L, and the sequences left
    to the sequential rerun."""
    out = (ctypes.c_int64 * 4)()
    check(lib().cvd_chunk_last(out))
    return {"groups": int(out[0]), "C": int(out[1]), "L": int(out[2]), "reruns": int(out[3])}
