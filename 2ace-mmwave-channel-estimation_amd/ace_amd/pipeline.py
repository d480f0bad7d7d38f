"""Host-side mirror of the reference's full recovery functions, backed by the HIP pipeline.

Reference (main/src/my_recovery_algorithms/ADMM_v2/):
  [X, Y, quality] = inferLowRankV4_multi(A, B, tx, rx, lambda, r, mu0, rho, cc_frac,
                                         tol_rel, tol_abs, maxiter)      (inferLowRankV4_multi.m:5)
  [X, Y, quality] = inferLowRank_Nuclear(...)                            (inferLowRank_Nuclear.m)
  inferLowRankV4 (Numerical_Simulation/src/my_recovery_algorithms/ADMM_v2/inferLowRankV4.m):
  the one-restart form of inferLowRankV4_multi.

MATLAB's ``randsample(m, floor(m*cc_frac))`` (:48), drawn inside every call, is replaced by
explicit train partitions: ``train_idx`` [restarts][m_t] shared by a batch, or
[batch][restarts][m_t] -- each realisation its own, as a Monte-Carlo batch of calls draws them
(ACE_TRAIN_PER_REALISATION: one GPU batch, the stages on the full A in m-space) -- or, when
omitted, random permutation prefixes (the same distribution as randsample without replacement;
MATLAB's stream itself is not reproducible outside MATLAB).

Entry points:
  * ``inferLowRankV4_multi`` / ``inferLowRankV4`` / ``inferLowRank_Nuclear`` -- one
    realisation, MATLAB argument order, numpy in / out ((n,1), (m,1), quality).
  * ``infer_low_rank_pipeline_host`` -- a batch on host arrays, shared or per-realisation
    partitions, one GPU batch (ace_pipeline_solve_host).
  * ``infer_low_rank_pipeline_batch`` -- device tensors already in HBM, shared or
    per-realisation partitions (ace_pipeline_solve_batch); the throughput path.
There is no CPU fallback: every call goes through libace.so.
"""
from __future__ import annotations

import ctypes as C
import math
from dataclasses import dataclass

import numpy as np

from ._lib import (LIB, check, pipeline_cfg, ACE_ST_ROLLBACK, ACE_ST_RANK_ONE, ACE_TRAIN_SHARED,
                   ACE_TRAIN_PER_REALISATION)
from .solver import VARIANTS


@dataclass
class PipelineResult:
    X: object            # [batch][n] complex128
    Y: object            # [batch][m] complex128
    quality: object      # [batch] float64 (last restart's, as the reference returns)
    stage_iters: object  # [batch][4*restarts+1] int32
    status: object       # [batch] uint32 (ACE_ST_* bits)

    @property
    def rolled_back(self):
        return (self.status & ACE_ST_ROLLBACK) != 0

    @property
    def rank_one(self):
        """The refinement's use_rank_one per realisation: the last restart ran the rank-one retry
        (inferLowRankV4_multi.m:73-77, passed at :92/:100)."""
        return (self.status & ACE_ST_RANK_ONE) != 0


def _cfg(variant, restarts, r, mu0, rho, cc_frac, tol_rel, tol_abs, maxiter, eig_warm):
    v = VARIANTS[variant]
    kw = dict(r=int(r), mu0=float(mu0), rho=float(rho), cc_frac=float(cc_frac), tol_rel=float(tol_rel),
              tol_abs=float(tol_abs), maxiter=int(maxiter), eig_warm=int(bool(eig_warm)))
    if restarts is not None:
        kw["restarts"] = int(restarts)
    return pipeline_cfg(v, **kw)


def draw_partitions(rng, m, restarts, cc_frac=0.95, batch=None):
    """randsample(m, floor(m*cc_frac)) per restart (inferLowRankV4_multi.m:48), 0-based:
    [restarts][m_t], or [batch][restarts][m_t] (one draw per call) when ``batch`` is given."""
    mt = math.floor(m * cc_frac)
    if batch is not None:
        return np.stack([np.stack([rng.permutation(m)[:mt] for _ in range(restarts)])
                         for _ in range(batch)]).astype(np.int32)
    return np.stack([rng.permutation(m)[:mt] for _ in range(restarts)]).astype(np.int32)


PART_MAXTE = 96   # test rows per realisation the per-realisation form takes (csrc/ace_common.hpp PART_MAXTE)


def _groups(tr, m):
    """Realisation groups that share their partitions, when a [batch][restarts][m_t] layout exceeds the
    per-realisation form's m - m_t <= PART_MAXTE (each group then runs as one shared-layout call), else None."""
    if tr.ndim != 3 or m - tr.shape[-1] <= PART_MAXTE:
        return None
    groups = {}
    for b in range(tr.shape[0]):
        groups.setdefault(tr[b].tobytes(), []).append(b)
    return list(groups.values())


def _layout(tr, batch):
    """(contiguous int32 train_idx, ACE_TRAIN_*) of a [restarts][m_t] or [batch][restarts][m_t] array."""
    tr = np.ascontiguousarray(np.asarray(tr, dtype=np.int32))
    if tr.ndim == 2:
        return tr, ACE_TRAIN_SHARED
    if tr.ndim == 3 and tr.shape[0] == batch:
        return tr, ACE_TRAIN_PER_REALISATION
    raise ValueError(f"train_idx must be [restarts][m_t] or [batch][restarts][m_t], got {tr.shape}")


def infer_low_rank_pipeline_host(A, B, tx, rx, train_idx, *, variant="A2only", restarts=None, r=20, mu0=1e-3,
                                 rho=1.03, cc_frac=0.95, tol_rel=1e-4, tol_abs=1e-8, maxiter=500,
                                 eig_warm=True) -> PipelineResult:
    """Pipeline on host arrays.  A: [m][n] (one codebook), B: [batch][m],
    train_idx: [restarts][m_t] (shared) or [batch][restarts][m_t]."""
    A = np.ascontiguousarray(A, dtype=np.complex128)
    if A.ndim == 3 and A.shape[0] == 1:
        A = A[0]
    B = np.ascontiguousarray(np.atleast_2d(np.asarray(B, dtype=np.float64)))
    batch, m = B.shape
    if A.ndim != 2 or A.shape[0] != m:
        raise ValueError(f"shape mismatch: A{A.shape} B{B.shape}")
    n = A.shape[1]
    tr, layout = _layout(train_idx, batch)
    grp = _groups(tr, m)
    if grp is not None and len(grp) > 1:   # (m - m_t > PART_MAXTE: one shared-layout call per group)
        parts = [(g, infer_low_rank_pipeline_host(A, B[g], tx, rx, tr[g[0]], variant=variant, restarts=restarts, r=r,
                                                  mu0=mu0, rho=rho, cc_frac=cc_frac, tol_rel=tol_rel,
                                                  tol_abs=tol_abs, maxiter=maxiter, eig_warm=eig_warm))
                 for g in grp]
        p0 = parts[0][1]
        res = PipelineResult(*(np.empty((batch,) + f.shape[1:], f.dtype) for f in
                               (p0.X, p0.Y, p0.quality, p0.stage_iters, p0.status)))
        for g, p in parts:
            for k in ("X", "Y", "quality", "stage_iters", "status"):
                getattr(res, k)[g] = getattr(p, k)
        return res
    if grp is not None:   # one group: every realisation shares the partitions
        tr, layout = tr[0], ACE_TRAIN_SHARED
    nres = tr.shape[-2] if restarts is None else int(restarts)
    cfg = _cfg(variant, nres, r, mu0, rho, cc_frac, tol_rel, tol_abs, maxiter, eig_warm)
    if tr.shape[-2] != cfg.restarts:
        raise ValueError(f"train_idx holds {tr.shape[-2]} partitions, cfg.restarts = {cfg.restarts}")
    cfg.train_layout = layout
    ld = 4 * cfg.restarts + 1
    X = np.empty((batch, n), np.complex128)
    Y = np.empty((batch, m), np.complex128)
    q = np.empty(batch, np.float64)
    its = np.empty((batch, ld), np.int32)
    stt = np.empty(batch, np.uint32)
    dp = lambda a: a.ctypes.data_as(C.POINTER(C.c_double))  # noqa: E731
    check(LIB.ace_pipeline_solve_host(
        C.byref(cfg), batch, m, n, tx, rx, dp(A.view(np.float64)), dp(B),
        tr.ctypes.data_as(C.POINTER(C.c_int32)), dp(X.view(np.float64)), dp(Y.view(np.float64)),
        dp(q), its.ctypes.data_as(C.POINTER(C.c_int32)), stt.ctypes.data_as(C.POINTER(C.c_uint32))))
    return PipelineResult(X, Y, q, its, stt)


def _single(A, B, tx, rx, lambda_, r, mu0, rho, cc_frac, tol_rel, tol_abs, maxiter, train_idx, rng, variant,
            restarts):
    if lambda_ != 0:
        raise NotImplementedError("lambda != 0 is unreachable from the reference drivers and not implemented")
    A = np.asarray(A, dtype=np.complex128)
    m = A.shape[0]
    if train_idx is None:
        train_idx = draw_partitions(rng if rng is not None else np.random.default_rng(), m, restarts, cc_frac)
    res = infer_low_rank_pipeline_host(A, np.asarray(B, dtype=np.float64).reshape(1, m), tx, rx,
                                       np.asarray(train_idx).reshape(restarts, -1), variant=variant,
                                       restarts=restarts, r=r, mu0=mu0, rho=rho, cc_frac=cc_frac,
                                       tol_rel=tol_rel, tol_abs=tol_abs, maxiter=maxiter)
    n = A.shape[1]
    return res.X[0].reshape(n, 1), res.Y[0].reshape(m, 1), float(res.quality[0])


def inferLowRankV4_multi(A, B, tx, rx, lambda_=0.0, r=20, mu0=1e-3, rho=1.03, cc_frac=0.95, tol_rel=1e-4,
                         tol_abs=1e-8, maxiter=500, *, train_idx=None, rng=None):
    """[X, Y, quality] = inferLowRankV4_multi(...) (3 restarts, keep the best)."""
    return _single(A, B, tx, rx, lambda_, r, mu0, rho, cc_frac, tol_rel, tol_abs, maxiter, train_idx, rng,
                   "A2only", 3)


def inferLowRankV4(A, B, tx, rx, lambda_=0.0, r=20, mu0=1e-3, rho=1.03, cc_frac=0.95, tol_rel=1e-4,
                   tol_abs=1e-8, maxiter=500, *, train_idx=None, rng=None):
    """Numerical_Simulation's inferLowRankV4: the one-restart pipeline."""
    return _single(A, B, tx, rx, lambda_, r, mu0, rho, cc_frac, tol_rel, tol_abs, maxiter, train_idx, rng,
                   "A2only", 1)


def inferLowRank_Nuclear(A, B, tx, rx, lambda_=0.0, r=20, mu0=1e-3, rho=1.03, cc_frac=0.95, tol_rel=1e-4,
                         tol_abs=1e-8, maxiter=500, *, train_idx=None, rng=None):
    """[X, Y, quality] = inferLowRank_Nuclear(...) (one restart, nuclear-norm Z-prox)."""
    return _single(A, B, tx, rx, lambda_, r, mu0, rho, cc_frac, tol_rel, tol_abs, maxiter, train_idx, rng,
                   "A2nuclear", 1)


def infer_low_rank_pipeline_batch(A, B, tx, rx, train_idx, *, variant="A2only", restarts=None, r=20, mu0=1e-3,
                                  rho=1.03, cc_frac=0.95, tol_rel=1e-4, tol_abs=1e-8, maxiter=500,
                                  eig_warm=True, stop_before_refine=False, workspace=None,
                                  stream=None) -> PipelineResult:
    """Batched pipeline on device tensors: A [m][n] complex128 (shared codebook),
    B [batch][m] float64, train_idx (host) [restarts][m_t] shared by the batch or
    [batch][restarts][m_t] per realisation.  ``stop_before_refine`` returns X_max, the refinement's
    input (inferLowRankV4_multi.m:90-92), instead of running the refinement stage."""
    import torch
    from .solver import _DEFAULT_WS
    if not (A.is_cuda and B.is_cuda):
        raise ValueError("infer_low_rank_pipeline_batch needs device tensors")
    if A.dtype != torch.complex128 or B.dtype != torch.float64:
        raise TypeError("A must be complex128 and B float64")
    if A.dim() == 3 and A.shape[0] == 1:
        A = A[0]
    A, B = A.contiguous(), B.contiguous()
    batch, m = B.shape
    n = A.shape[1]
    tr, layout = _layout(train_idx, batch)
    grp = _groups(tr, m)
    if grp is not None and len(grp) > 1:   # (m - m_t > PART_MAXTE: one shared-layout call per group)
        cur = torch.cuda.current_stream(B.device)
        if stream is not None and stream != cur:
            # the whole grouped path (the B subsets, the group solves, the scatter of their outputs) runs on
            # `stream` after what the caller queued on its current stream; A and B stay reserved for `stream`
            stream.wait_stream(cur)
            A.record_stream(stream)
            B.record_stream(stream)
            with torch.cuda.stream(stream):
                return infer_low_rank_pipeline_batch(
                    A, B, tx, rx, train_idx, variant=variant, restarts=restarts, r=r, mu0=mu0, rho=rho,
                    cc_frac=cc_frac, tol_rel=tol_rel, tol_abs=tol_abs, maxiter=maxiter, eig_warm=eig_warm,
                    stop_before_refine=stop_before_refine, workspace=workspace, stream=None)
        kw = dict(variant=variant, restarts=restarts, r=r, mu0=mu0, rho=rho, cc_frac=cc_frac, tol_rel=tol_rel,
                  tol_abs=tol_abs, maxiter=maxiter, eig_warm=eig_warm, stop_before_refine=stop_before_refine,
                  workspace=workspace, stream=None)
        outs = []
        for g in grp:
            gi = torch.as_tensor(g, device=B.device)
            outs.append((gi, infer_low_rank_pipeline_batch(A, B.index_select(0, gi).contiguous(), tx, rx,
                                                           tr[g[0]], **kw)))
        o0 = outs[0][1]
        res = PipelineResult(*(torch.empty((batch,) + tuple(f.shape[1:]), dtype=f.dtype, device=f.device) for f in
                               (o0.X, o0.Y, o0.quality, o0.stage_iters, o0.status)))
        for gi, o in outs:
            for k in ("X", "Y", "quality", "stage_iters", "status"):
                getattr(res, k).index_copy_(0, gi, getattr(o, k))
        return res
    if grp is not None:   # one group: every realisation shares the partitions
        tr, layout = tr[0], ACE_TRAIN_SHARED
    nres = tr.shape[-2] if restarts is None else int(restarts)
    cfg = _cfg(variant, nres, r, mu0, rho, cc_frac, tol_rel, tol_abs, maxiter, eig_warm)
    cfg.stop_before_refine = int(bool(stop_before_refine))
    cfg.train_layout = layout
    ld = 4 * cfg.restarts + 1
    dev = A.device
    out = PipelineResult(torch.empty((batch, n), dtype=torch.complex128, device=dev),
                         torch.empty((batch, m), dtype=torch.complex128, device=dev),
                         torch.empty(batch, dtype=torch.float64, device=dev),
                         torch.empty((batch, ld), dtype=torch.int32, device=dev),
                         torch.empty(batch, dtype=torch.int32, device=dev))
    nbytes = int(LIB.ace_pipeline_workspace_size(C.byref(cfg), batch, m, n)) + 256
    if nbytes <= 256:
        raise ValueError(LIB.ace_last_error().decode() or "invalid pipeline configuration")
    ws = (workspace or _DEFAULT_WS).get(nbytes, dev)
    if stream is None:
        stream = torch.cuda.current_stream(dev)
    check(LIB.ace_pipeline_solve_batch(C.byref(cfg), batch, m, n, tx, rx, A.data_ptr(), B.data_ptr(),
                                       tr.ctypes.data_as(C.POINTER(C.c_int32)), out.X.data_ptr(),
                                       out.Y.data_ptr(), out.quality.data_ptr(), out.stage_iters.data_ptr(),
                                       out.status.data_ptr(), ws.data_ptr(), ws.numel(), stream.cuda_stream))
    return out


def SpectralInitialize(A, B, r):
    """X = SpectralInitialize(A, B, r) (inferLowRankV4_multi.m:561-574) on the GPU, the kernels of
    the pipeline's own initialisation.  A: [m, n] complex; B: [m] or [batch, m] magnitudes.
    Returns [n, r] (or [batch, n, r]) complex128: column k = sqrt(s_k) v_k, eigenvectors up to a
    unit phase each."""
    A = np.ascontiguousarray(A, dtype=np.complex128)
    B = np.asarray(B, dtype=np.float64)
    single = B.ndim == 1
    Bb = np.ascontiguousarray(B[None, :] if single else B)
    m, n = A.shape
    batch = Bb.shape[0]
    if Bb.shape[1] != m:
        raise ValueError("B must have m entries per realisation")
    X = np.empty((batch, r, n), np.complex128)
    st = np.zeros(batch, np.uint32)
    check(LIB.ace_spectral_init_host(batch, m, n, int(r), A.ctypes.data, Bb.ctypes.data, X.ctypes.data,
                                     st.ctypes.data))
    X = np.transpose(X, (0, 2, 1))
    return X[0] if single else X

