"""ctypes binding of libace.so (the C-ABI declared in include/ace.h).

The product path has no CPU fallback: if the HIP library is missing this
module raises at import time, and every solver entry point goes through it.
"""
from __future__ import annotations

import ctypes as C
import os
import pathlib

_HERE = pathlib.Path(__file__).resolve().parent
LIB_PATH = pathlib.Path(os.environ.get("ACE_LIB", _HERE / "libace.so"))

ACE_OK = 0
ACE_ERR_ARG = -1
ACE_ERR_UNSUPPORTED = -2
ACE_ERR_HIP = -3
ACE_ERR_WORKSPACE = -4

ACE_VARIANT_A2ONLY = 0
ACE_VARIANT_NUCLEAR = 1

ACE_ST_CONVERGED = 1
ACE_ST_NO_OPT = 2
ACE_ST_EIG_NOCONV = 4
ACE_ST_ROLLBACK = 8
ACE_ST_RANK_ONE = 128

ACE_TRAIN_SHARED = 0
ACE_TRAIN_PER_REALISATION = 1

KERNEL_CLASSES = ["setup", "init", "pre", "apply_A", "apply_G", "ystep", "apply_K", "apply_AH", "zstep", "final", "msr"]


class AceError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"ace error {code}: {msg}")
        self.code = code


class AdmmCfg(C.Structure):
    """Mirror of ``ace_admm_cfg`` (include/ace.h)."""
    _fields_ = [
        ("variant", C.c_int),
        ("scale_by_row", C.c_int),
        ("use_rank_one", C.c_int),
        ("maxiter", C.c_int),
        ("fixed_iters", C.c_int),
        ("a_shared", C.c_int),
        ("eig_warm", C.c_int),
        ("f64_applies", C.c_int),
        ("mu0", C.c_double),
        ("rho", C.c_double),
        ("tol_rel", C.c_double),
        ("tol_abs", C.c_double),
        ("r", C.c_int),
        ("reserved", C.c_int),
        ("rank_one", C.c_void_p),
    ]


class PipelineCfg(C.Structure):
    """Mirror of ``ace_pipeline_cfg`` (include/ace.h)."""
    _fields_ = [
        ("variant", C.c_int),
        ("restarts", C.c_int),
        ("r", C.c_int),
        ("maxiter", C.c_int),
        ("eig_warm", C.c_int),
        ("stop_before_refine", C.c_int),
        ("train_layout", C.c_int),
        ("train_seed", C.c_int),
        ("mu0", C.c_double),
        ("rho", C.c_double),
        ("cc_frac", C.c_double),
        ("tol_rel", C.c_double),
        ("tol_abs", C.c_double),
    ]


def _load():
    if not LIB_PATH.exists():
        raise ImportError(
            f"ace_amd: HIP library {LIB_PATH} not found -- build it with "
            f"`make -C 2ace-mmwave-channel-estimation_amd/csrc` (or __graft_entry__.build()). "
            f"There is no CPU fallback on the product path.")
    lib = C.CDLL(str(LIB_PATH))
    vp, dp, ip, up = C.c_void_p, C.POINTER(C.c_double), C.POINTER(C.c_int32), C.POINTER(C.c_uint32)
    cfgp = C.POINTER(AdmmCfg)
    lib.ace_admm_cfg_default.argtypes = [cfgp]
    lib.ace_admm_cfg_default.restype = None
    lib.ace_admm_workspace_size.argtypes = [cfgp, C.c_int, C.c_int, C.c_int]
    lib.ace_admm_workspace_size.restype = C.c_size_t
    lib.ace_admm_solve_batch.argtypes = [cfgp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                         vp, vp, vp, vp, vp, vp, vp, vp, vp, C.c_size_t, vp]
    lib.ace_admm_solve_batch.restype = C.c_int
    lib.ace_admm_solve_host.argtypes = [cfgp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                        dp, dp, dp, dp, dp, ip, up, dp]
    lib.ace_admm_solve_host.restype = C.c_int
    pcfgp = C.POINTER(PipelineCfg)
    lib.ace_pipeline_cfg_default.argtypes = [pcfgp, C.c_int]
    lib.ace_pipeline_cfg_default.restype = None
    lib.ace_pipeline_workspace_size.argtypes = [pcfgp, C.c_int, C.c_int, C.c_int]
    lib.ace_pipeline_workspace_size.restype = C.c_size_t
    lib.ace_pipeline_solve_batch.argtypes = [pcfgp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                             vp, vp, ip, vp, vp, vp, vp, vp, vp, C.c_size_t, vp]
    lib.ace_pipeline_solve_batch.restype = C.c_int
    lib.ace_pipeline_solve_host.argtypes = [pcfgp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                            dp, dp, ip, dp, dp, dp, ip, up]
    lib.ace_pipeline_solve_host.restype = C.c_int
    lib.ace_synth_codebook.argtypes = [C.c_uint64, C.c_int64, C.c_int, C.c_int, C.c_int, vp, vp]
    lib.ace_synth_codebook.restype = C.c_int
    lib.ace_synth_channels.argtypes = [C.c_uint64, C.c_int64, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                       C.c_double, C.c_double, vp, C.c_int, vp, vp, vp, vp]
    lib.ace_synth_channels.restype = C.c_int
    lib.ace_prof_start.argtypes = [C.c_int]
    lib.ace_prof_start.restype = C.c_int
    lib.ace_prof_sample.argtypes = [C.c_int, C.c_uint32]
    lib.ace_prof_sample.restype = C.c_int
    lib.ace_prof_stop.argtypes = [dp, ip]
    lib.ace_prof_stop.restype = C.c_int
    lib.ace_prof_msp_steps.argtypes = [C.POINTER(C.c_longlong)]
    lib.ace_prof_msp_steps.restype = C.c_int
    lib.ace_prof_work.argtypes = [dp]
    lib.ace_prof_work.restype = C.c_int
    lib.ace_prof_work_ex.argtypes = [dp, dp, dp]
    lib.ace_prof_work_ex.restype = C.c_int
    lib.ace_nuclear_prox_batch.argtypes = [C.c_int, C.c_int, C.c_int, vp, C.c_double, vp, vp]
    lib.ace_nuclear_prox_batch.restype = C.c_int
    lib.ace_spectral_init_host.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, vp, vp, vp, vp]
    lib.ace_spectral_init_host.restype = C.c_int
    lib.ace_path_counts.argtypes = [C.POINTER(C.c_int64), C.c_int]
    lib.ace_path_counts.restype = C.c_int
    lib.ace_lds_request.argtypes = [C.c_char_p, C.c_int, C.POINTER(C.c_size_t)]
    lib.ace_lds_request.restype = C.c_int
    lib.ace_last_error.argtypes = []
    lib.ace_last_error.restype = C.c_char_p
    lib.ace_version.argtypes = []
    lib.ace_version.restype = C.c_char_p
    return lib


LIB = _load()


def check(rc):
    if rc != ACE_OK:
        raise AceError(rc, LIB.ace_last_error().decode())
    return rc


PATHS = ("int8_shared", "codes_private", "f64_shared", "f64_private")


def path_counts(reset=False):
    """InferADMM solves per apply path since the last reset (ace_path_counts)."""
    v = (C.c_int64 * 4)()
    check(LIB.ace_path_counts(v, int(bool(reset))))
    return dict(zip(PATHS, v))


def lds_request(kernel: str, m: int) -> int:
    """Dynamic LDS bytes the launcher of ``kernel`` requests at size m (ace_lds_request; no GPU call)."""
    v = C.c_size_t()
    check(LIB.ace_lds_request(kernel.encode(), int(m), C.byref(v)))
    return v.value


def default_cfg(**kw) -> AdmmCfg:
    cfg = AdmmCfg()
    LIB.ace_admm_cfg_default(C.byref(cfg))
    for k, v in kw.items():
        if not hasattr(cfg, k):
            raise TypeError(f"unknown ace_admm_cfg field {k!r}")
        setattr(cfg, k, v)
    return cfg


def pipeline_cfg(variant, **kw) -> PipelineCfg:
    cfg = PipelineCfg()
    LIB.ace_pipeline_cfg_default(C.byref(cfg), int(variant))
    for k, v in kw.items():
        if not hasattr(cfg, k):
            raise TypeError(f"unknown ace_pipeline_cfg field {k!r}")
        setattr(cfg, k, v)
    return cfg
