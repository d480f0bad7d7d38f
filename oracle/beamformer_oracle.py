"""CPU oracle for the downstream beamformer.

TEST INFRASTRUCTURE ONLY.  Nothing on the product path imports this module: only
``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg use it,
and only as the checker.

Reference: ``main/codebook_library.py:57-96`` (``svd_beamformer``), ``:98-138``
(``svd_beamformer_compensation``) and the compute part of ``codebook_generator``
(``:192-213``: reshape each recovered H row to [tx, rx], compensation on row 0).

The reference's algorithm lives in a third-party dependency: ``numpy.linalg.svd``, i.e.
LAPACK ``zgesdd`` with JOBZ='A' from the numpy wheel's scipy-openblas (OpenBLAS 0.3.29,
Reference-LAPACK 3.12 sources).  The beam codes are NOT invariant to the phase LAPACK
picks for each singular vector (the phases are quantised to 2 bits), so the GPU kernel
reproduces zgesdd's convention.  For square n <= 25 (ilaenv SMLSIZ) zgesdd's path is:

  zgebd2 (upper bidiagonal, Householder via zlarfg)  ->  dbdsdc('U','I') which for
  n <= 25 is dlasdq -> dbdsqr on the real bidiagonal, VT_b from identity  ->
  Vh = VT_b * P^H  (zunmbr('P','R','C')).

``gesdd_vh`` below restates that path (the published LAPACK algorithms, with the 3.10+
``dlartg`` sign convention: c >= 0, r carries the sign of f).  ``test_beamformer_oracle``
checks it against ``numpy.linalg.svd`` itself, which pins the convention the HIP kernel
implements.  For 26 <= n <= 32 zgesdd switches to divide and conquer (dlasd0), whose real
singular vectors are dbdsqr's up to sign; ``dc_merge_signs`` restates the merge's sign
convention (dlasd1 / dlasd3), exact except on vectors the merge deflates (the null space of a
rank-deficient H), where beams agree up to a per-beam sign = code offset 0 or 2.

``svd_beamformer`` itself uses ``numpy.linalg.svd`` exactly as the reference does.
"""
from __future__ import annotations

import math

import numpy as np

REF_BF = "main/codebook_library.py"
EPS = 2.0 ** -53          # dlamch('E')
SAFMIN = 2.0 ** -1022     # dlamch('S')
SAFMAX = 1.0 / SAFMIN
RTMIN = math.sqrt(SAFMIN)
RTMAX = math.sqrt(SAFMAX / 2)
TOL = max(10.0, min(100.0, EPS ** -0.125)) * EPS   # dbdsqr TOLMUL*EPS
MAXITR = 6


# --------------------------------------------------------------------------- codes
def quant_codes(v, offset=None):
    """2-bit code string of a quantised beam column (codebook_library.py:80-88).

    ``v`` is a column of wr_quant/wt_quant (unit-modulus); ``offset`` the compensation
    phase (radians, :122).  Returns an int array with values 0..3."""
    v = np.asarray(v, dtype=np.complex128)
    if offset is not None:
        v = v * np.exp(-1j * np.asarray(offset, dtype=np.float64))
    q = np.around(np.angle(v) / (np.pi / 2))
    q[q < 0] = q[q < 0] + 4
    q[q == 4] = 0
    return q.astype(np.int64)


def quantise_vh(vh):
    """wr_quant = exp(-1j * transpose(around(angle(Vh)/(pi/2))*(pi/2))) (:61-65)."""
    ang = -np.transpose(np.around(np.angle(vh) / (np.pi / 2)) * (np.pi / 2))
    return np.exp(1j * ang)


def svd_beamformer(H, offset=None, vh_fn=None):
    """svd_beamformer / svd_beamformer_compensation (codebook_library.py:57-138).

    Returns (wr_code, wt_code, tx_idx, rx_idx, rss_max) — the reference returns the two
    code strings; ``codes_to_str`` turns them into the same strings."""
    H = np.asarray(H, dtype=np.complex128)
    ant_tx, ant_rx = H.shape
    if vh_fn is None:
        vh_fn = lambda a: np.linalg.svd(a)[2]  # noqa: E731
    wr_quant = quantise_vh(vh_fn(H))            # :59, :61, :64
    wt_quant = quantise_vh(vh_fn(np.transpose(H)))  # :60, :62, :65
    # :67-73 — |wt[:,i]^T (H wr[:,j])|^2 over all (i, j), i-major; argmax = first max.
    sig = np.abs(wt_quant.T @ (H @ wr_quant)) ** 2
    with np.errstate(divide="ignore"):
        rss = 10 * np.log10(sig * 1000)
    idx = int(np.argmax(rss.reshape(-1)))
    tx_idx, rx_idx = divmod(idx, ant_rx)
    wr = quant_codes(wr_quant[:, rx_idx], offset)
    wt = quant_codes(wt_quant[:, tx_idx], offset)
    return wr, wt, tx_idx, rx_idx, float(rss.reshape(-1)[idx])


def codes_to_str(c):
    return "".join(str(int(b)) for b in c)


def codebook_beams(H_est, H_directional, tx, rx, compensation=None):
    """Compute part of codebook_generator (codebook_library.py:192-213): one
    (wr, wt) code pair per recovered row; row 0 of H_est gets the compensation."""
    wr, wt = [], []
    for i in range(len(H_est)):
        H = np.reshape(H_est[i, :], [tx, rx])
        off = None if (i != 0 or compensation is None) else np.asarray(compensation) * (np.pi / 2)
        a, b, *_ = svd_beamformer(H, off)
        wr.append(codes_to_str(a))
        wt.append(codes_to_str(b))
    for i in range(len(H_directional)):
        H = np.reshape(H_directional[i, :], [tx, rx])
        a, b, *_ = svd_beamformer(H)
        wr.append(codes_to_str(a))
        wt.append(codes_to_str(b))
    return wr, wt


# ------------------------------------------------------- LAPACK restatement (zgesdd)
def dlartg(f, g):
    """Reference-LAPACK 3.10+ dlartg (la_xlartg): c >= 0, r = sign(f) * hypot."""
    if g == 0.0:
        return 1.0, 0.0, f
    if f == 0.0:
        return 0.0, math.copysign(1.0, g), abs(g)
    f1, g1 = abs(f), abs(g)
    if RTMIN < f1 < RTMAX and RTMIN < g1 < RTMAX:
        d = math.sqrt(f * f + g * g)
        c = f1 / d
        r = math.copysign(d, f)
        return c, g / r, r
    u = min(SAFMAX, max(SAFMIN, f1, g1))
    fs, gs = f / u, g / u
    d = math.sqrt(fs * fs + gs * gs)
    c = abs(fs) / d
    r = math.copysign(d, f)
    return c, gs / r, r * u


def dlas2(f, g, h):
    """Singular values of [[f, g], [0, h]] (LAPACK dlas2)."""
    fa, ga, ha = abs(f), abs(g), abs(h)
    fhmn, fhmx = min(fa, ha), max(fa, ha)
    if fhmn == 0.0:
        if fhmx == 0.0:
            return 0.0, ga
        mx, mn = max(fhmx, ga), min(fhmx, ga)
        return 0.0, mx * math.sqrt(1.0 + (mn / mx) ** 2)
    if ga < fhmx:
        as_ = 1.0 + fhmn / fhmx
        at = (fhmx - fhmn) / fhmx
        au = (ga / fhmx) ** 2
        c = 2.0 / (math.sqrt(as_ * as_ + au) + math.sqrt(at * at + au))
        return fhmn * c, fhmx / c
    au = fhmx / ga
    if au == 0.0:
        return (fhmn * fhmx) / ga, ga
    as_ = 1.0 + fhmn / fhmx
    at = (fhmx - fhmn) / fhmx
    c = 1.0 / (math.sqrt(1.0 + (as_ * au) ** 2) + math.sqrt(1.0 + (at * au) ** 2))
    ssmin = (fhmn * c) * au
    return ssmin + ssmin, ga / (c + c)


def _sign(a, b):
    return math.copysign(abs(a), b)


def dlasv2(f, g, h):
    """SVD of [[f, g], [0, h]] (LAPACK dlasv2): returns ssmin, ssmax, snr, csr, snl, csl."""
    ft, fa, ht, ha = f, abs(f), h, abs(h)
    pmax = 1
    swap = ha > fa
    if swap:
        pmax = 3
        ft, ht = ht, ft
        fa, ha = ha, fa
    gt, ga = g, abs(g)
    if ga == 0.0:
        ssmin, ssmax = ha, fa
        clt, crt, slt, srt = 1.0, 1.0, 0.0, 0.0
    else:
        gasmal = True
        if ga > fa:
            pmax = 2
            if fa / ga < EPS:
                gasmal = False
                ssmax = ga
                ssmin = fa / (ga / ha) if ha > 1.0 else (fa / ga) * ha
                clt, slt, srt, crt = 1.0, ht / gt, 1.0, ft / gt
        if gasmal:
            d = fa - ha
            l = 1.0 if d == fa else d / fa
            m = gt / ft
            t = 2.0 - l
            mm, tt = m * m, t * t
            s = math.sqrt(tt + mm)
            r = abs(m) if l == 0.0 else math.sqrt(l * l + mm)
            a = 0.5 * (s + r)
            ssmin, ssmax = ha / a, fa * a
            if mm == 0.0:
                if l == 0.0:
                    t = _sign(2.0, ft) * _sign(1.0, gt)
                else:
                    t = gt / _sign(d, ft) + m / t
            else:
                t = (m / (s + t) + m / (r + l)) * (1.0 + a)
            l = math.sqrt(t * t + 4.0)
            crt = 2.0 / l
            srt = t / l
            clt = (crt + srt * m) / a
            slt = (ht / ft) * srt / a
    if swap:
        csl, snl, csr, snr = srt, crt, slt, clt
    else:
        csl, snl, csr, snr = clt, slt, crt, srt
    if pmax == 1:
        tsign = _sign(1.0, csr) * _sign(1.0, csl) * _sign(1.0, f)
    elif pmax == 2:
        tsign = _sign(1.0, snr) * _sign(1.0, csl) * _sign(1.0, g)
    else:
        tsign = _sign(1.0, snr) * _sign(1.0, snl) * _sign(1.0, h)
    ssmax = _sign(ssmax, tsign)
    ssmin = _sign(ssmin, tsign * _sign(1.0, f) * _sign(1.0, h))
    return ssmin, ssmax, snr, csr, snl, csl


def _rot_rows(vt, i, j, c, s):
    """drot on rows i, j: x' = c x + s y, y' = c y - s x."""
    x, y = vt[i].copy(), vt[j].copy()
    vt[i] = c * x + s * y
    vt[j] = c * y - s * x


def dbdsqr_vt(d, e, stats=None):
    """Right singular vectors of the real upper bidiagonal (d, e) by LAPACK dbdsqr
    (relative accuracy, ROTATE path), VT accumulated from the identity.  Returns
    (s, VT) with s descending."""
    d = [float(x) for x in d]
    e = [float(x) for x in e] + [0.0]
    n = len(d)
    vt = np.eye(n)
    if n > 1:
        smax = max(max(abs(x) for x in d), max(abs(x) for x in e[:n - 1]))
        sminoa = abs(d[0])
        if sminoa != 0.0:
            mu = sminoa
            for i in range(1, n):
                mu = abs(d[i]) * (mu / (mu + abs(e[i - 1])))
                sminoa = min(sminoa, mu)
                if sminoa == 0.0:
                    break
        sminoa = sminoa / math.sqrt(n)
        thresh = max(TOL * sminoa, MAXITR * (n * (n * SAFMIN)))
        maxitdivn = MAXITR * n
        iterdivn, it = 0, -1
        oldll, oldm, idir = -1, -1, 0
        m = n  # 1-based index of the last unconverged element
        sminl = 0.0
        sweeps = 0
        while m > 1:
            if it >= n:
                it -= n
                iterdivn += 1
                if iterdivn >= maxitdivn:
                    raise RuntimeError("dbdsqr: no convergence")
            # find the diagonal block (1-based ll..m)
            smax = abs(d[m - 1])
            ll = 0
            split = False
            for lll in range(1, m):
                ll = m - lll
                abss, abse = abs(d[ll - 1]), abs(e[ll - 1])
                if abse <= thresh:
                    split = True
                    break
                smax = max(smax, abss, abse)
            if split:
                e[ll - 1] = 0.0
                if ll == m - 1:
                    m -= 1
                    continue
            else:
                ll = 0
            ll += 1
            if ll == m - 1:
                ssmin, ssmax, sinr, cosr, sinl, cosl = dlasv2(d[m - 2], e[m - 2], d[m - 1])
                d[m - 2], e[m - 2], d[m - 1] = ssmax, 0.0, ssmin
                _rot_rows(vt, m - 2, m - 1, cosr, sinr)
                m -= 2
                continue
            if ll > oldm or m < oldll:
                idir = 1 if abs(d[ll - 1]) >= abs(d[m - 1]) else 2
            if idir == 1:
                if abs(e[m - 2]) <= abs(TOL) * abs(d[m - 1]):
                    e[m - 2] = 0.0
                    continue
                mu = abs(d[ll - 1])
                sminl = mu
                conv = False
                for lll in range(ll, m):
                    if abs(e[lll - 1]) <= TOL * mu:
                        e[lll - 1] = 0.0
                        conv = True
                        break
                    mu = abs(d[lll]) * (mu / (mu + abs(e[lll - 1])))
                    sminl = min(sminl, mu)
                if conv:
                    continue
            else:
                if abs(e[ll - 1]) <= abs(TOL) * abs(d[ll - 1]):
                    e[ll - 1] = 0.0
                    continue
                mu = abs(d[m - 1])
                sminl = mu
                conv = False
                for lll in range(m - 1, ll - 1, -1):
                    if abs(e[lll - 1]) <= TOL * mu:
                        e[lll - 1] = 0.0
                        conv = True
                        break
                    mu = abs(d[lll - 1]) * (mu / (mu + abs(e[lll - 1])))
                    sminl = min(sminl, mu)
                if conv:
                    continue
            oldll, oldm = ll, m
            if n * TOL * (sminl / smax) <= max(EPS, 0.01 * TOL):
                shift = 0.0
            else:
                if idir == 1:
                    sll = abs(d[ll - 1])
                    shift, _ = dlas2(d[m - 2], e[m - 2], d[m - 1])
                else:
                    sll = abs(d[m - 1])
                    shift, _ = dlas2(d[ll - 1], e[ll - 1], d[ll])
                if sll > 0.0 and (shift / sll) ** 2 < EPS:
                    shift = 0.0
            it += m - ll
            sweeps += 1
            rots = []  # (row pair (i, i+1) 0-based, c, s) in application order
            if shift == 0.0:
                if idir == 1:
                    cs, oldcs, oldsn = 1.0, 1.0, 0.0
                    for i in range(ll, m):
                        cs, sn, r = dlartg(d[i - 1] * cs, e[i - 1])
                        if i > ll:
                            e[i - 2] = oldsn * r
                        oldcs, oldsn, d[i - 1] = dlartg(oldcs * r, d[i] * sn)
                        rots.append((i - 1, cs, sn))
                    h = d[m - 1] * cs
                    d[m - 1] = h * oldcs
                    e[m - 2] = h * oldsn
                    for (i, c, s) in rots:           # dlasr('L','V','F')
                        _rot_rows(vt, i, i + 1, c, s)
                    if abs(e[m - 2]) <= thresh:
                        e[m - 2] = 0.0
                else:
                    cs, oldcs, oldsn = 1.0, 1.0, 0.0
                    for i in range(m, ll, -1):
                        cs, sn, r = dlartg(d[i - 1] * cs, e[i - 2])
                        if i < m:
                            e[i - 1] = oldsn * r
                        oldcs, oldsn, d[i - 1] = dlartg(oldcs * r, d[i - 2] * sn)
                        rots.append((i - 2, oldcs, -oldsn))
                    h = d[ll - 1] * cs
                    d[ll - 1] = h * oldcs
                    e[ll - 1] = h * oldsn
                    for (i, c, s) in rots:           # dlasr('L','V','B'): j = m-1 .. 1
                        _rot_rows(vt, i, i + 1, c, s)
                    if abs(e[ll - 1]) <= thresh:
                        e[ll - 1] = 0.0
            else:
                if idir == 1:
                    f = (abs(d[ll - 1]) - shift) * (_sign(1.0, d[ll - 1]) + shift / d[ll - 1])
                    g = e[ll - 1]
                    for i in range(ll, m):
                        cosr, sinr, r = dlartg(f, g)
                        if i > ll:
                            e[i - 2] = r
                        f = cosr * d[i - 1] + sinr * e[i - 1]
                        e[i - 1] = cosr * e[i - 1] - sinr * d[i - 1]
                        g = sinr * d[i]
                        d[i] = cosr * d[i]
                        cosl, sinl, r = dlartg(f, g)
                        d[i - 1] = r
                        f = cosl * e[i - 1] + sinl * d[i]
                        d[i] = cosl * d[i] - sinl * e[i - 1]
                        if i < m - 1:
                            g = sinl * e[i]
                            e[i] = cosl * e[i]
                        rots.append((i - 1, cosr, sinr))
                    e[m - 2] = f
                    for (i, c, s) in rots:
                        _rot_rows(vt, i, i + 1, c, s)
                    if abs(e[m - 2]) <= thresh:
                        e[m - 2] = 0.0
                else:
                    f = (abs(d[m - 1]) - shift) * (_sign(1.0, d[m - 1]) + shift / d[m - 1])
                    g = e[m - 2]
                    for i in range(m, ll, -1):
                        cosr, sinr, r = dlartg(f, g)
                        if i < m:
                            e[i - 1] = r
                        f = cosr * d[i - 1] + sinr * e[i - 2]
                        e[i - 2] = cosr * e[i - 2] - sinr * d[i - 1]
                        g = sinr * d[i - 2]
                        d[i - 2] = cosr * d[i - 2]
                        cosl, sinl, r = dlartg(f, g)
                        d[i - 1] = r
                        f = cosl * e[i - 2] + sinl * d[i - 2]
                        d[i - 2] = cosl * d[i - 2] - sinl * e[i - 2]
                        if i > ll + 1:
                            g = sinl * e[i - 3]
                            e[i - 3] = cosl * e[i - 3]
                        rots.append((i - 2, cosl, -sinl))
                    e[ll - 1] = f
                    if abs(e[ll - 1]) <= thresh:
                        e[ll - 1] = 0.0
                    for (i, c, s) in rots:
                        _rot_rows(vt, i, i + 1, c, s)
        if stats is not None:
            stats["sweeps"] = sweeps
    # make singular values positive, then selection-sort descending (dbdsqr :160-190)
    for i in range(n):
        if d[i] < 0.0:
            d[i] = -d[i]
            vt[i] = -vt[i]
    for i in range(1, n):
        isub, smin = 1, d[0]
        for j in range(2, n + 2 - i):
            if d[j - 1] <= smin:
                isub, smin = j, d[j - 1]
        last = n + 1 - i
        if isub != last:
            d[isub - 1] = d[last - 1]
            d[last - 1] = smin
            vt[[isub - 1, last - 1]] = vt[[last - 1, isub - 1]]
    return np.array(d), vt


def dlapy3(x, y, z):
    """LAPACK dlapy3: sqrt(x^2 + y^2 + z^2) scaled by the largest magnitude."""
    xa, ya, za = abs(x), abs(y), abs(z)
    w = max(xa, ya, za)
    if w == 0.0 or w > 1.79e308:
        return xa + ya + za
    return w * math.sqrt((xa / w) ** 2 + (ya / w) ** 2 + (za / w) ** 2)


def zlarfg(alpha, x):
    """LAPACK zlarfg: returns (beta, tau, v_tail) with H^H [alpha; x] = [beta; 0],
    H = I - tau [1; v] [1; v]^H."""
    xnorm = float(np.linalg.norm(x)) if x.size else 0.0
    ar, ai = alpha.real, alpha.imag
    if xnorm == 0.0 and ai == 0.0:
        return alpha, 0.0 + 0.0j, np.zeros_like(x)
    beta = -math.copysign(dlapy3(ar, ai, xnorm), ar)
    tau = complex((beta - ar) / beta, -ai / beta)
    scal = 1.0 / (alpha - beta)
    return complex(beta, 0.0), tau, x * scal


def zgebd2_upper(A):
    """LAPACK zgebd2 for m >= n: A = Q B P^H, B real upper bidiagonal.  Returns
    (d, e, [(v_i, taup_i)]) with P = G(1)...G(n-1), G(i) = I - taup v v^H acting on
    columns i+1..n."""
    A = np.array(A, dtype=np.complex128)
    m, n = A.shape
    d = np.zeros(n)
    e = np.zeros(max(n - 1, 0))
    refl = []
    for i in range(n):
        beta, tauq, v = zlarfg(A[i, i], A[i + 1:, i])
        d[i] = beta.real
        vq = np.concatenate([[1.0 + 0j], v])
        if i < n - 1:
            C = A[i:, i + 1:]
            w = vq.conj() @ C                      # v^H C
            A[i:, i + 1:] = C - np.conj(tauq) * np.outer(vq, w)
            row = np.conj(A[i, i + 1:])           # zlacgv
            beta2, taup, vp = zlarfg(row[0], row[1:])
            e[i] = beta2.real
            vv = np.concatenate([[1.0 + 0j], vp])
            C2 = A[i + 1:, i + 1:]
            w2 = C2 @ vv
            A[i + 1:, i + 1:] = C2 - taup * np.outer(w2, vv.conj())
            refl.append((i + 1, vv, taup))
    return d, e, refl


SMLSIZ = 25   # ilaenv(9, 'DBDSDC'): dbdsdc's divide-and-conquer threshold


def dc_merge_signs(d, e, vtb):
    """zgesdd's divide-and-conquer sign convention for 26 <= n <= 32, applied to dbdsqr's VT.

    dbdsdc('U', 'I') with n > SMLSIZ calls dlasd0, whose dlasdt tree for n <= 2 (SMLSIZ + 1)
    is one root at row mid = n // 2 (0-based) over the leaves [0, mid) (dlasdq, sqre = 1) and
    (mid, n) (dlasdq, sqre = 0).  dlasd1 merges them: dlasd2 puts the merge row's unit vector
    first in the deflated basis and dlasd3 sets every non-deflated secular vector's first
    component to -1 before normalising (``U(1, I) = NEGONE``), so the merged left vector u_i
    has u_i(mid) < 0.  The singular vectors themselves equal dbdsqr's up to sign (distinct
    singular values), hence: flip VT row i where u_i(mid) = (d_mid v_i(mid) + e_mid
    v_i(mid + 1)) / s_i > 0.  A vector dlasd2 deflated (|z_j| <= 64 eps * scale) keeps its
    leaf's dbdsqr sign instead, which this does not model (only the null space of a rank-
    deficient matrix was seen to deflate; test_beamformer_oracle measures it)."""
    n = len(d)
    mid = n // 2
    um = d[mid] * vtb[:, mid] + e[mid] * vtb[:, mid + 1]
    return vtb * np.where(um > 0.0, -1.0, 1.0)[:, None]


def gesdd_vh(A, stats=None):
    """Vh of zgesdd(JOBZ='A') for a square A with n <= 32 (see module docstring; n > 25 takes
    the divide-and-conquer sign convention of ``dc_merge_signs``)."""
    A = np.asarray(A, dtype=np.complex128)
    n = A.shape[0]
    d, e, refl = zgebd2_upper(A)
    if n == 1:                               # dbdsdc n == 1: VT = 1, the sign goes to U
        return np.ones((1, 1), np.complex128)
    _, vtb = dbdsqr_vt(d.copy(), e.copy(), stats)
    if n > SMLSIZ:
        vtb = dc_merge_signs(d, e, vtb)
    X = vtb.astype(np.complex128)
    for (c0, vv, taup) in reversed(refl):   # X := X G(i)^H, i = n-1 .. 1
        sub = X[:, c0:]
        w = sub @ vv
        X[:, c0:] = sub - np.conj(taup) * np.outer(w, vv.conj())
    return X


# ------------------------------------------- rectangular arrays (tx != rx): zgesdd's paths
def gesdd_paths(m, n):
    """zgesdd's path choice for an m x n input (zgesdd.f: MNTHR1 = INT(MINMN * 17 / 9),
    MNTHR2 = INT(MINMN * 5 / 3)): 'qr' (paths 1-4, M >= MNTHR1: QR first), 'lq' (paths 1t-4t,
    N >= MNTHR1: LQ first) or 'direct' (paths 5/6 and 5t/6t: zgebrd on the input itself;
    5 and 6 differ only in how P^H is formed, not in the result)."""
    minmn = min(m, n)
    mnthr1 = int(minmn * 17.0 / 9.0)
    if m >= n and m >= mnthr1 and m > n:
        return "qr"
    if n > m and n >= mnthr1:
        return "lq"
    return "direct"


def zgeqr2_r(A):
    """R of LAPACK zgeqr2 (Householder QR, zlarfg conventions) of an m x n, m >= n input."""
    A = np.array(A, dtype=np.complex128)
    m, n = A.shape
    for i in range(n):
        beta, tau, v = zlarfg(A[i, i], A[i + 1:, i])
        A[i, i] = beta
        A[i + 1:, i] = 0.0
        if i < n - 1:
            vq = np.concatenate([[1.0 + 0j], v])
            C = A[i:, i + 1:]
            A[i:, i + 1:] = C - np.conj(tau) * np.outer(vq, vq.conj() @ C)   # H(i)^H C
    return np.triu(A[:n, :n])


def zgelq2_lq(A):
    """LAPACK zgelq2 of an m x n, m < n input: (L [m][m] lower, Q [n][n]) with A = L Q[:m],
    Q = H(m)^H ... H(1)^H (zunglq with k = m reflectors, all n rows)."""
    A = np.array(A, dtype=np.complex128)
    m, n = A.shape
    Qh = np.eye(n, dtype=np.complex128)           # H(1) H(2) ... H(m)
    for i in range(m):
        row = np.conj(A[i, i:])                    # zlacgv
        beta, tau, v = zlarfg(row[0], row[1:])
        vv = np.concatenate([[1.0 + 0j], v])
        if i < m - 1:
            C = A[i + 1:, i:]
            A[i + 1:, i:] = C - tau * np.outer(C @ vv, vv.conj())             # C H(i)
        A[i, i] = beta
        A[i, i + 1:] = 0.0
        sub = Qh[:, i:]
        Qh[:, i:] = sub - tau * np.outer(sub @ vv, vv.conj())
    return np.tril(A[:, :m]), Qh.conj().T


def zgebd2_lower(A):
    """LAPACK zgebd2 for m < n: A = Q B P^H, B real lower bidiagonal (d [m], e [m - 1]).
    Returns (d, e, [(c0, v, taup)]) with G(i) = I - taup v v^H acting on columns c0 = i .. n."""
    A = np.array(A, dtype=np.complex128)
    m, n = A.shape
    d = np.zeros(m)
    e = np.zeros(max(m - 1, 0))
    refl = []
    for i in range(m):
        row = np.conj(A[i, i:])                    # zlacgv
        beta, taup, vp = zlarfg(row[0], row[1:])
        d[i] = beta.real
        vv = np.concatenate([[1.0 + 0j], vp])
        refl.append((i, vv, taup))
        if i < m - 1:
            C = A[i + 1:, i:]
            A[i + 1:, i:] = C - taup * np.outer(C @ vv, vv.conj())           # C G(i)
            beta2, tauq, vq = zlarfg(A[i + 1, i], A[i + 2:, i])
            e[i] = beta2.real
            vc = np.concatenate([[1.0 + 0j], vq])
            C2 = A[i + 1:, i + 1:]
            A[i + 1:, i + 1:] = C2 - np.conj(tauq) * np.outer(vc, vc.conj() @ C2)   # H(i)^H C
    return d, e, refl


def lower_to_upper(d, e):
    """dbdsdc('L'): Givens rotations on the left turn the lower bidiagonal into an upper one with
    the same right singular vectors (dbdsdc.f, IUPLO = 2: DLARTG, E(I) = SN D(I+1), D(I+1) = CS D(I+1))."""
    d = [float(x) for x in d]
    e = [float(x) for x in e]
    for i in range(len(d) - 1):
        cs, sn, r = dlartg(d[i], e[i])
        d[i] = r
        e[i] = sn * d[i + 1]
        d[i + 1] = cs * d[i + 1]
    return np.array(d), np.array(e)


def gesdd_vh_rect(A, stats=None):
    """Vh [n][n] of zgesdd(JOBZ='A') for any m x n input with m, n <= 32 (square: gesdd_vh)."""
    A = np.asarray(A, dtype=np.complex128)
    m, n = A.shape
    if m == n:
        return gesdd_vh(A, stats)
    if n == 1:                                   # dbdsdc n == 1: VT = 1
        return np.ones((1, 1), np.complex128)
    path = gesdd_paths(m, n)
    if path == "qr":                             # zgeqrf, zgebrd on R (n x n)
        return gesdd_vh(zgeqr2_r(A), stats)
    if path == "lq":                             # zgelqf, zgebrd on L (m x m), VT = [Vh_L Q[:m]; Q[m:]]
        L, Q = zgelq2_lq(A)
        X = np.empty((n, n), np.complex128)
        X[:m] = (np.ones((1, 1)) if m == 1 else gesdd_vh(L, stats)) @ Q[:m]
        X[m:] = Q[m:]
        return X
    if m > n:                                    # direct, tall: upper bidiagonal n x n
        d, e, refl = zgebd2_upper(A)
        _, vtb = dbdsqr_vt(d.copy(), e.copy(), stats)
        if n > SMLSIZ:
            vtb = dc_merge_signs(d, e, vtb)
        X = vtb.astype(np.complex128)
    else:                                        # direct, wide: lower bidiagonal m x m, VT = [VT_b 0; 0 I] P^H
        d, e, refl = zgebd2_lower(A)
        if m == 1:
            vtb = np.ones((1, 1))
        else:
            du, eu = lower_to_upper(d, e)
            _, vtb = dbdsqr_vt(du.copy(), eu.copy(), stats)
            if m > SMLSIZ:
                vtb = dc_merge_signs(du, eu, vtb)
        X = np.eye(n, dtype=np.complex128)
        X[:m, :m] = vtb
    for (c0, vv, taup) in reversed(refl):        # X := X G(i)^H, last reflector first
        sub = X[:, c0:]
        w = sub @ vv
        X[:, c0:] = sub - np.conj(taup) * np.outer(w, vv.conj())
    return X
