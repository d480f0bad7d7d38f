"""Host-side mirror of the reference solver interface, backed by the HIP library.

Reference: main/src/my_recovery_algorithms/ADMM_v2/inferLowRankV4_multi.m
  InferADMM(A, B, X0, scale_by_row, use_rank_one, tx, rx, lambda, mu0, rho,
            tol_rel, tol_abs, maxiter, U, D)                          (:281)
and inferLowRank_Nuclear.m (:269) for the nuclear-norm variant.

Two entry points:
  * ``InferADMM`` -- same argument names/meaning as the MATLAB function for one
    realisation (numpy in, numpy out); the GPU solves it through
    ``ace_admm_solve_host``.
  * ``infer_admm_batch`` -- the throughput path: torch tensors already resident
    in HBM, one call for a whole batch of realisations, asynchronous on the
    current HIP stream (``ace_admm_solve_batch``).

Errors follow the reference's behaviour where it has one (MATLAB raises on bad
shapes); configurations the GPU path does not implement raise
``NotImplementedError`` -- there is no silent CPU fallback.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _lib
from ._lib import LIB, check, default_cfg, ACE_VARIANT_A2ONLY, ACE_VARIANT_NUCLEAR  # noqa: F401

VARIANTS = {"A2only": ACE_VARIANT_A2ONLY, "A2nuclear": ACE_VARIANT_NUCLEAR,
            "a2only": ACE_VARIANT_A2ONLY, "nuclear": ACE_VARIANT_NUCLEAR,
            ACE_VARIANT_A2ONLY: ACE_VARIANT_A2ONLY, ACE_VARIANT_NUCLEAR: ACE_VARIANT_NUCLEAR}


@dataclass
class BatchResult:
    X: object          # [batch][n] complex128 (torch tensor or numpy)
    Y: object          # [batch][m]
    iters: object      # [batch] int32
    status: object     # [batch] uint32 (ACE_ST_* bits)
    mu: object         # [batch] float64
    rank_one: object = None   # the per-realisation flags the solve was given (device), if any

    @property
    def converged(self):
        return (self.status & _lib.ACE_ST_CONVERGED) != 0


def _cfg(variant, scale_by_row, use_rank_one, mu0, rho, tol_rel, tol_abs, maxiter, fixed_iters, a_shared,
         eig_warm, f64_applies=False, r=1):
    return default_cfg(variant=VARIANTS[variant], scale_by_row=int(bool(scale_by_row)),
                       use_rank_one=int(bool(use_rank_one)), mu0=float(mu0), rho=float(rho),
                       tol_rel=float(tol_rel), tol_abs=float(tol_abs), maxiter=int(maxiter),
                       fixed_iters=int(bool(fixed_iters)), a_shared=int(bool(a_shared)),
                       eig_warm=int(bool(eig_warm)), f64_applies=int(bool(f64_applies)), r=int(r))


def _flags(use_rank_one, batch):
    """use_rank_one as (batch-wide bool, per-realisation uint8 array or None)."""
    shp = getattr(use_rank_one, "shape", None)
    if shp is None and isinstance(use_rank_one, (list, tuple)):
        shp = (len(use_rank_one),)
    if shp is None or len(shp) == 0:
        return bool(use_rank_one), None
    return False, use_rank_one


def _cols(X0, batch, n):
    """X0 [batch][n] or [batch][r][n] -> r (columns per realisation, :281 X0 is n x r)."""
    if X0.ndim == 2 and tuple(X0.shape) == (batch, n):
        return 1
    if X0.ndim == 3 and X0.shape[0] == batch and X0.shape[2] == n and 1 <= X0.shape[1] <= 32:
        return int(X0.shape[1])
    raise ValueError(f"X0 must be [batch][n] or [batch][r][n] with r <= 32, got {tuple(X0.shape)}")


def _dp(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


def InferADMM(A, B, X0, scale_by_row, use_rank_one, tx, rx, lambda_=0.0, mu0=1e-3, rho=1.03,
              tol_rel=1e-4, tol_abs=1e-8, maxiter=500, U=None, D=None, *, variant="A2only",
              fixed_iters=False, eig_warm=True):
    """[X, Y, converged] = InferADMM(...) (inferLowRankV4_multi.m:281-386) on the GPU.

    ``U``/``D`` are accepted for signature parity and ignored: the GPU path forms
    its own (I + A A^H)^{-1} (algebraically identical to U = inv(A'A + I)).
    Only lambda = 0 (the value every reference driver reaches) runs on the GPU.  X0 is n x r
    (r <= 32): r = 1 is the refinement stage (:92/:100), r = 20 the stages of inferLowRankImpl
    (:258 with scale_by_row, :270 without: X, Y are then the best column, :352-361).
    """
    if lambda_ != 0:
        raise NotImplementedError("lambda != 0 is unreachable from the reference drivers and not implemented")
    A = np.ascontiguousarray(A, dtype=np.complex128)
    m, n = A.shape
    X0 = np.asarray(X0, dtype=np.complex128)
    X0 = X0.reshape(n, -1)
    r = X0.shape[1]
    if r > 32:
        raise NotImplementedError("GPU InferADMM implements r <= 32 columns")
    X0 = np.ascontiguousarray(X0.T)[None]                   # [1][r][n]: column j contiguous
    B = np.ascontiguousarray(np.asarray(B, dtype=np.float64).reshape(m))
    res = infer_admm_host(A[None], B[None], X0 if r > 1 else X0[:, 0], tx, rx, variant=variant,
                          scale_by_row=scale_by_row, use_rank_one=use_rank_one, mu0=mu0, rho=rho, tol_rel=tol_rel,
                          tol_abs=tol_abs, maxiter=maxiter, fixed_iters=fixed_iters, eig_warm=eig_warm)
    R = r if scale_by_row else 1
    return res.X[0].reshape(R, n).T.copy(), res.Y[0].reshape(R, m).T.copy(), bool(res.converged[0])


def infer_admm_host(A, B, X0, tx, rx, *, variant="A2only", scale_by_row=True, use_rank_one=False, mu0=1e-3,
                    rho=1.03, tol_rel=1e-4, tol_abs=1e-8, maxiter=500, fixed_iters=False, eig_warm=True,
                    f64_applies=False):
    """Batch solve on host numpy arrays: A [1|batch][m][n], B [batch][m], X0 [batch][n] or
    [batch][r][n] (r > 1: shared A).  ``use_rank_one``: one flag for the batch or one per
    realisation (the refinement of a batch of pipelines, inferLowRankV4_multi.m:92/:100).
    ``f64_applies`` keeps the f64 matrix-core applies for phase-code codebooks too.
    X, Y: [batch][n] / [batch][m] at r = 1, else [batch][R][n] / [batch][R][m] with
    R = r (scale_by_row) or 1 (per-column mode: the best column)."""
    A = np.ascontiguousarray(A, dtype=np.complex128)
    B = np.ascontiguousarray(B, dtype=np.float64)
    X0 = np.ascontiguousarray(X0, dtype=np.complex128)
    batch, m = B.shape
    n = X0.shape[-1]
    r = _cols(X0, batch, n)
    if A.ndim != 3 or A.shape[1:] != (m, n) or A.shape[0] not in (1, batch):
        raise ValueError(f"shape mismatch: A{A.shape} B{B.shape} X0{X0.shape}")
    a_shared = A.shape[0] == 1
    uro, flags = _flags(use_rank_one, batch)
    cfg = _cfg(variant, scale_by_row, uro, mu0, rho, tol_rel, tol_abs, maxiter, fixed_iters, a_shared,
               eig_warm, f64_applies, r)
    if flags is not None:
        flags = np.ascontiguousarray(np.asarray(flags).reshape(-1) != 0, dtype=np.uint8)
        if flags.shape != (batch,):
            raise ValueError(f"use_rank_one must be a scalar or one flag per realisation ({batch})")
        cfg.rank_one = flags.ctypes.data
    R = r if scale_by_row else 1
    shp = (batch,) if X0.ndim == 2 else (batch, R)
    X = np.empty(shp + (n,), np.complex128)
    Y = np.empty(shp + (m,), np.complex128)
    it = np.empty(batch, np.int32)
    stt = np.empty(batch, np.uint32)
    mu = np.empty(batch, np.float64)
    check(LIB.ace_admm_solve_host(C.byref(cfg), batch, m, n, tx, rx, _dp(A.view(np.float64)),
                                  _dp(B), _dp(X0.view(np.float64)), _dp(X.view(np.float64)),
                                  _dp(Y.view(np.float64)), it.ctypes.data_as(C.POINTER(C.c_int32)),
                                  stt.ctypes.data_as(C.POINTER(C.c_uint32)), _dp(mu)))
    return BatchResult(X, Y, it, stt, mu)


class Workspace:
    """Reusable device workspace for ``infer_admm_batch`` (a torch uint8 tensor)."""

    def __init__(self):
        self.buf = None

    def get(self, nbytes, device):
        import torch
        if self.buf is None or self.buf.numel() < nbytes or self.buf.device != device:
            self.buf = torch.empty(nbytes, dtype=torch.uint8, device=device)
        return self.buf


_DEFAULT_WS = Workspace()


def infer_admm_batch(A, B, X0, tx, rx, *, variant="A2only", scale_by_row=True, use_rank_one=False, mu0=1e-3,
                     rho=1.03, tol_rel=1e-4, tol_abs=1e-8, maxiter=500, fixed_iters=False, eig_warm=True,
                     f64_applies=False, out=None, workspace=None, stream=None):
    """Batched InferADMM on device tensors (torch, complex128 / float64, contiguous).

    A: [1|batch][m][n] (1 = shared codebook), B: [batch][m], X0: [batch][n] or [batch][r][n]
    (r <= 32, shared A).  ``use_rank_one``: a bool for the whole batch, or one flag per
    realisation (a device tensor, or a host array uploaded here) -- the refinement of a batch of
    pipelines passes each realisation's last-restart flag (inferLowRankV4_multi.m:73-77, :92/:100;
    PipelineResult.rank_one).  Returns BatchResult of device tensors; asynchronous on ``stream``
    (default: torch's current stream) except for the convergence polls of early-exit mode.
    """
    import torch
    if not (A.is_cuda and B.is_cuda and X0.is_cuda):
        raise ValueError("infer_admm_batch needs device tensors (use infer_admm_host for numpy arrays)")
    if A.dtype != torch.complex128 or X0.dtype != torch.complex128 or B.dtype != torch.float64:
        raise TypeError("A, X0 must be complex128 and B float64")
    A, B, X0 = A.contiguous(), B.contiguous(), X0.contiguous()
    batch, m = B.shape
    n = X0.shape[-1]
    r = _cols(X0, batch, n)
    if A.dim() != 3 or tuple(A.shape[1:]) != (m, n) or A.shape[0] not in (1, batch):
        raise ValueError(f"shape mismatch: A{tuple(A.shape)} B{tuple(B.shape)} X0{tuple(X0.shape)}")
    a_shared = A.shape[0] == 1
    uro, flags = _flags(use_rank_one, batch)
    cfg = _cfg(variant, scale_by_row, uro, mu0, rho, tol_rel, tol_abs, maxiter, fixed_iters, a_shared,
               eig_warm, f64_applies, r)
    dev = A.device
    if flags is not None:
        flags = torch.as_tensor(flags).reshape(-1).to(device=dev)
        flags = (flags != 0).to(torch.uint8).contiguous()
        if flags.numel() != batch:
            raise ValueError(f"use_rank_one must be a scalar or one flag per realisation ({batch})")
        cfg.rank_one = flags.data_ptr()
    R = r if scale_by_row else 1
    shp = (batch,) if X0.dim() == 2 else (batch, R)
    if out is None:
        out = BatchResult(torch.empty(shp + (n,), dtype=torch.complex128, device=dev),
                          torch.empty(shp + (m,), dtype=torch.complex128, device=dev),
                          torch.empty(batch, dtype=torch.int32, device=dev),
                          torch.empty(batch, dtype=torch.int32, device=dev),
                          torch.empty(batch, dtype=torch.float64, device=dev))
    nbytes = int(LIB.ace_admm_workspace_size(C.byref(cfg), batch, m, n)) + 256
    ws = (workspace or _DEFAULT_WS).get(nbytes, dev)
    if stream is None:
        stream = torch.cuda.current_stream(dev)
    cur = torch.cuda.current_stream(dev)
    if flags is not None and stream != cur:
        # the flags were built on torch's current stream: the solve's stream waits for them, and their
        # memory stays reserved for that stream until the solve has read them
        stream.wait_stream(cur)
        flags.record_stream(stream)
    check(LIB.ace_admm_solve_batch(C.byref(cfg), batch, m, n, tx, rx, A.data_ptr(), B.data_ptr(), X0.data_ptr(),
                                   out.X.data_ptr(), out.Y.data_ptr(), out.iters.data_ptr(),
                                   out.status.data_ptr(), out.mu.data_ptr(), ws.data_ptr(), ws.numel(),
                                   stream.cuda_stream))
    if flags is not None:
        out.rank_one = flags   # (kept alive until the asynchronous solve has read it)
    return out


def nuclear_prox_batch(E, tau, *, out=None, stream=None):
    """Z_b = U Shrink(S, tau) V^H of each n x r matrix E_b (inferLowRank_Nuclear.m:411-439, the
    A2nuclear Z-prox) on the GPU.  E: torch complex128 device tensor [batch][r][n] (column j of
    realisation b contiguous, the solver's state layout), r <= 32."""
    import torch
    if not E.is_cuda or E.dtype != torch.complex128 or E.dim() != 3:
        raise TypeError("E must be a complex128 device tensor [batch][r][n]")
    E = E.contiguous()
    batch, r, n = E.shape
    if out is None:
        out = torch.empty_like(E)
    if stream is None:
        stream = torch.cuda.current_stream(E.device)
    check(LIB.ace_nuclear_prox_batch(batch, n, r, E.data_ptr(), float(tau), out.data_ptr(), stream.cuda_stream))
    return out


def synth_problem(seed, first, count, m, tx, rx, *, a_shared=True, L=3, snr_db=30.0, x0_noise=0.5,
                  device="cuda", stream=None, A=None):
    """Generate a synthetic batch directly in HBM (ace_synth_codebook/ace_synth_channels).
    ``A`` (a device complex128 [1][m][n] tensor) replaces the random phase-code codebook, e.g. by
    rows of a multiresolution codebook (ace_amd.synth.multires_codebook)."""
    import torch
    n = tx * rx
    dev = torch.device(device)
    if stream is None:
        stream = torch.cuda.current_stream(dev)
    na = 1 if a_shared else count
    if A is not None:
        if not a_shared or tuple(A.shape) != (1, m, n) or A.dtype != torch.complex128 or not A.is_cuda:
            raise ValueError("A must be a shared device complex128 [1][m][n] codebook")
        A = A.contiguous()
    else:
        A = torch.empty((na, m, n), dtype=torch.complex128, device=dev)
        check(LIB.ace_synth_codebook(seed, -1 if a_shared else first, na, m, n, A.data_ptr(), stream.cuda_stream))
    H = torch.empty((count, n), dtype=torch.complex128, device=dev)
    B = torch.empty((count, m), dtype=torch.float64, device=dev)
    X0 = torch.empty((count, n), dtype=torch.complex128, device=dev)
    check(LIB.ace_synth_channels(seed, first, count, m, tx, rx, L, snr_db, x0_noise, A.data_ptr(),
                                 int(a_shared), H.data_ptr(), B.data_ptr(), X0.data_ptr(), stream.cuda_stream))
    return A, B, X0, H
