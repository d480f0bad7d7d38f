"""Host-side mirror of the reference's downstream beamformer, backed by the HIP library.

Reference (main/codebook_library.py):
  * ``svd_beamformer(H)`` (:57-96) -> (wr_out, wt_out): 2-bit code strings of the best
    pair of phase-quantised right singular vectors of H and H^T;
  * ``svd_beamformer_compensation(H, offset)`` (:98-138): the same codes after an
    element-wise phase offset (``compensation * pi/2``);
  * ``codebook_generator`` (:192-213) runs one of them per recovered channel row
    (compensation on row 0 only) before writing the firmware codebook (.brd writing is
    the hardware tool's job and out of scope; ``codebook_beams`` returns the codes).

Entry points (no CPU fallback — every call runs ``beamformer_kernel`` on the GPU):
  * ``svd_beamformer`` / ``svd_beamformer_compensation`` — reference signatures, one H.
  * ``codebook_beams`` — the compute part of ``codebook_generator``, all rows in one launch.
  * ``svd_beamformer_host(H, offset)`` — a batch of host arrays.
  * ``svd_beamformer_batch(H, offset)`` — device tensors already in HBM (throughput path).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from ._lib import LIB, check

ACE_ST_BF_NONFINITE = 16
ACE_ST_BF_NOCONV = 32
ACE_ST_BF_DC = 64

_dp = C.POINTER(C.c_double)
_u8p = C.POINTER(C.c_uint8)
LIB.ace_svd_beamformer_batch.argtypes = [C.c_int, C.c_int, C.c_int] + [C.c_void_p] * 9 + [C.c_void_p]
LIB.ace_svd_beamformer_batch.restype = C.c_int
LIB.ace_svd_beamformer_host.argtypes = [C.c_int, C.c_int, C.c_int, _dp, _dp, _u8p, _u8p, C.POINTER(C.c_int32), _dp,
                                        C.POINTER(C.c_uint32), _dp, _dp]
LIB.ace_svd_beamformer_host.restype = C.c_int


class LinAlgError(np.linalg.LinAlgError):
    """Raised where numpy.linalg.svd raises inside the reference (non-finite H)."""


@dataclass
class BeamResult:
    wr_code: object   # [batch][rx] uint8 (0..3)
    wt_code: object   # [batch][tx] uint8
    beam_idx: object  # [batch][2] int32 (tx_idx, rx_idx)
    rss: object       # [batch] float64 (dB of the winning pair)
    status: object    # [batch] uint32 (ACE_ST_BF_*)
    vh_r: object = None  # [batch][rx][rx] complex128 Vh of svd(H)   (optional)
    vh_t: object = None  # [batch][tx][tx] complex128 Vh of svd(H^T) (optional)


def _codes_str(c):
    return "".join(chr(48 + int(x)) for x in c)


def _offset_len(offset, tx, rx):
    """Length of the per-realisation offset row.  The reference multiplies wr (rx entries) and wt (tx
    entries) by the same ``exp(-1j * offset)`` (codebook_library.py:122, :129), so the row must broadcast
    against both, as numpy requires: a constant, or max(tx, rx) entries when tx == rx."""
    shp = np.shape(offset)
    L = shp[-1] if len(shp) else 1
    if L != 1 and (L != rx or L != tx):
        raise ValueError(f"operands could not be broadcast together: offset of length {L} against "
                         f"wr ({rx},) and wt ({tx},)")
    return L


def svd_beamformer_host(H, offset=None, want_vh=False) -> BeamResult:
    """Batch of svd_beamformer(_compensation) on host arrays.  H [batch][tx][rx] complex (1..32
    antennas each side, tx != rx allowed); offset None, or radians per realisation ([batch][L] / [L] /
    scalar) with L = rx = tx or L = 1 (the C-ABI row is max(tx, rx) entries)."""
    H = np.ascontiguousarray(np.asarray(H, dtype=np.complex128))
    if H.ndim == 2:
        H = H[None]
    if H.ndim != 3:
        raise ValueError(f"H must be [batch][tx][rx], got shape {H.shape}")
    batch, tx, rx = H.shape
    off = None
    if offset is not None:
        L = _offset_len(offset, tx, rx)
        o = np.asarray(offset, dtype=np.float64).reshape(-1, L)
        off = np.ascontiguousarray(np.broadcast_to(o, (batch, L)))
        off = np.ascontiguousarray(np.broadcast_to(off, (batch, max(tx, rx))))
    wr = np.empty((batch, rx), np.uint8)
    wt = np.empty((batch, tx), np.uint8)
    idx = np.empty((batch, 2), np.int32)
    rss = np.empty(batch, np.float64)
    st = np.empty(batch, np.uint32)
    vr = np.empty((batch, rx, rx), np.complex128) if want_vh else None
    vt = np.empty((batch, tx, tx), np.complex128) if want_vh else None
    f64 = lambda a: None if a is None else a.view(np.float64).ctypes.data_as(_dp)  # noqa: E731
    check(LIB.ace_svd_beamformer_host(batch, tx, rx, f64(H), None if off is None else off.ctypes.data_as(_dp),
                                      wr.ctypes.data_as(_u8p), wt.ctypes.data_as(_u8p),
                                      idx.ctypes.data_as(C.POINTER(C.c_int32)), rss.ctypes.data_as(_dp),
                                      st.ctypes.data_as(C.POINTER(C.c_uint32)), f64(vr), f64(vt)))
    return BeamResult(wr, wt, idx, rss, st, vr, vt)


def svd_beamformer_batch(H, offset=None, *, want_vh=False, stream=None) -> BeamResult:
    """Batch on device tensors: H [batch][tx][rx] complex128, offset None or [batch][L] / [L] f64 (L as
    in svd_beamformer_host)."""
    import torch
    if not H.is_cuda:
        raise ValueError("svd_beamformer_batch needs device tensors")
    H = H.contiguous()
    batch, tx, rx = H.shape
    dev = H.device
    if offset is not None:
        L = _offset_len(offset, tx, rx)
        offset = offset.to(device=dev, dtype=torch.float64).reshape(-1, L).expand(batch, L)
        offset = offset.expand(batch, max(tx, rx)).contiguous()
    out = BeamResult(torch.empty((batch, rx), dtype=torch.uint8, device=dev),
                     torch.empty((batch, tx), dtype=torch.uint8, device=dev),
                     torch.empty((batch, 2), dtype=torch.int32, device=dev),
                     torch.empty(batch, dtype=torch.float64, device=dev),
                     torch.empty(batch, dtype=torch.int32, device=dev),
                     torch.empty((batch, rx, rx), dtype=torch.complex128, device=dev) if want_vh else None,
                     torch.empty((batch, tx, tx), dtype=torch.complex128, device=dev) if want_vh else None)
    if stream is None:
        stream = torch.cuda.current_stream(dev)
    ptr = lambda t: None if t is None else t.data_ptr()  # noqa: E731
    check(LIB.ace_svd_beamformer_batch(batch, tx, rx, H.data_ptr(), ptr(offset), out.wr_code.data_ptr(),
                                       out.wt_code.data_ptr(), out.beam_idx.data_ptr(), out.rss.data_ptr(),
                                       out.status.data_ptr(), ptr(out.vh_r), ptr(out.vh_t), stream.cuda_stream))
    return out


def _one(H, offset):
    H = np.asarray(H, dtype=np.complex128)
    if H.ndim != 2:
        raise ValueError(f"H must be 2-D (tx, rx), got shape {H.shape}")
    res = svd_beamformer_host(H[None], None if offset is None else np.asarray(offset, np.float64)[None])
    if res.status[0] & ACE_ST_BF_NONFINITE:
        raise LinAlgError("SVD did not converge")
    return _codes_str(res.wr_code[0]), _codes_str(res.wt_code[0])


def svd_beamformer(H):
    """wr_out, wt_out = svd_beamformer(H) (codebook_library.py:57)."""
    return _one(H, None)


def svd_beamformer_compensation(H, offset):
    """wr_out, wt_out = svd_beamformer_compensation(H, offset) (codebook_library.py:98)."""
    return _one(H, offset)


def codebook_beams(H_est, H_directional, num_tx_ant, num_rx_ant,
                   compensation=np.array([0] * 16)):
    """(wr, wt) code-string lists of codebook_generator (codebook_library.py:192-213) for
    the recovered rows H_est [k][tx*rx] and H_directional [k'][tx*rx]: row 0 of H_est with
    the compensation offset, every other row plain, in one GPU launch."""
    H_est = np.asarray(H_est, dtype=np.complex128).reshape(-1, num_tx_ant * num_rx_ant)
    H_dir = np.asarray(H_directional, dtype=np.complex128).reshape(-1, num_tx_ant * num_rx_ant)
    Hs = np.concatenate([H_est, H_dir]).reshape(-1, num_tx_ant, num_rx_ant)
    if len(Hs) == 0:
        return [], []
    comp = np.asarray(compensation, dtype=np.float64) * (np.pi / 2)
    off = np.zeros((len(Hs), _offset_len(comp, num_tx_ant, num_rx_ant) if len(H_est) else 1))
    if len(H_est):
        off[0] = comp
    res = svd_beamformer_host(Hs, off)
    if np.any(res.status & ACE_ST_BF_NONFINITE):
        raise LinAlgError("SVD did not converge")
    return [_codes_str(c) for c in res.wr_code], [_codes_str(c) for c in res.wt_code]
