"""Numpy model of the prox eigensolver's two-stage Hermitian reduction (development tool, r06).

Stage 1 (he2hb, LAPACK zhetrd_he2hb lower): panels of NB columns; the panel below the band is
QR-factored (zgeqr2: zlarfg + H^H from the left), T = zlarft (forward, columnwise), and the trailing
matrix takes Q^H A22 Q as A22 -= V W^H + W V^H with X = A22 V T, W = X - 1/2 V (T^H V^H X).
Stage 2 (hb2st): bulge chasing on the lower band (bandwidth NB) with Householder reflectors of length
<= NB: sweep i annihilates column i below the subdiagonal, each chase step right-applies the previous
reflector to the block below it, annihilates the first column of the resulting bulge and applies the new
reflector two-sided to the next diagonal block.  T = Q2^H Q1^H A Q1 Q2, eigenvectors Q1 Q2 z.

The kernels (csrc/ace_heev2.hip) follow this model's index conventions; `python tools/proto_heev2.py`
checks it against numpy.linalg.eigh.
"""
import numpy as np


def zlarfg(x):
    """LAPACK zlarfg: H^H x = beta e1 with H = I - tau v v^H, v[0] = 1, beta real."""
    alpha = x[0]
    xn = np.linalg.norm(x[1:]) if len(x) > 1 else 0.0
    v = np.zeros(len(x), complex)
    v[0] = 1.0
    if xn == 0.0 and alpha.imag == 0.0:
        return alpha.real, 0.0 + 0.0j, v
    beta = -np.copysign(np.sqrt(alpha.real ** 2 + alpha.imag ** 2 + xn ** 2), alpha.real)
    tau = complex((beta - alpha.real) / beta, -alpha.imag / beta)
    v[1:] = x[1:] / (alpha - beta)
    return beta, tau, v


def larft(V, tau):
    """zlarft forward columnwise: H_0 ... H_{k-1} = I - V T V^H."""
    k = V.shape[1]
    T = np.zeros((k, k), complex)
    for i in range(k):
        T[i, i] = tau[i]
        if i:
            y = -tau[i] * (V[:, :i].conj().T @ V[:, i])
            T[:i, i] = T[:i, :i] @ y
    return T


def he2hb(A, nb):
    n = A.shape[0]
    A = A.copy()
    blocks = []   # (r0, V [L][nb], T [nb][nb]) for Q1 = prod_p (I - V_p T_p V_p^H) embedded at rows r0..
    for k in range(0, n - nb, nb):
        r0 = k + nb
        L = n - r0
        P = A[r0:, k:k + nb].copy()
        nref = min(nb, L)
        V = np.zeros((L, nb), complex)
        tau = np.zeros(nb, complex)
        for j in range(nref):
            beta, t, v = zlarfg(P[j:, j])
            P[j, j] = beta
            P[j + 1:, j] = 0
            if j + 1 < nb:
                w = v.conj() @ P[j:, j + 1:]
                P[j:, j + 1:] -= np.conj(t) * np.outer(v, w)
            V[j:, j] = v
            tau[j] = t
        T = larft(V, tau)
        A[r0:, k:k + nb] = P
        A[k:k + nb, r0:] = P.conj().T
        A22 = A[r0:, r0:]
        X = A22 @ V @ T
        M = V.conj().T @ X
        W = X - 0.5 * V @ (T.conj().T @ M)
        A22 -= V @ W.conj().T + W @ V.conj().T
        A[r0:, r0:] = A22
        blocks.append((r0, V, T))
    return A, blocks


def hb2st(B, b):
    """Bulge chasing on a Hermitian band matrix (full storage here, only the lower band is read).
    Returns d, e (real) and the reflectors [(row0, v, tau)] in generation order."""
    n = B.shape[0]
    A = np.tril(B.copy())
    A = A + np.tril(A, -1).conj().T
    refl = []

    def two_sided(r0, r1, v, t):
        # A[r0:r1, r0:r1] <- H^H D H
        D = A[r0:r1, r0:r1]
        x = t * (D @ v)
        alpha = -0.5 * t * np.vdot(x, v)
        w = x + alpha * v
        D -= np.outer(v, w.conj()) + np.outer(w, v.conj())
        A[r0:r1, r0:r1] = D

    for i in range(n - 1):   # (the last, length-1 reflector makes e[n-2] real, as zhetd2)
        r0, r1 = i + 1, min(i + 1 + b, n)           # rows of the first reflector
        beta, t, v = zlarfg(A[r0:r1, i].copy())
        A[r0, i] = beta
        A[r0 + 1:r1, i] = 0
        A[i, r0:r1] = A[r0:r1, i].conj()
        refl.append((r0, v, t))
        two_sided(r0, r1, v, t)
        while True:
            s0, s1 = r1, min(r1 + b, n)             # the block below the last reflector's rows
            if s0 >= n:
                break
            Bk = A[s0:s1, r0:r1]
            Bk = Bk - t * np.outer(Bk @ v, v.conj())   # right-apply H
            beta2, t2, v2 = zlarfg(Bk[:, 0].copy())
            Bk[:, 0] = 0
            Bk[0, 0] = beta2
            if Bk.shape[1] > 1:
                w = v2.conj() @ Bk[:, 1:]
                Bk[:, 1:] -= np.conj(t2) * np.outer(v2, w)
            A[s0:s1, r0:r1] = Bk
            A[r0:r1, s0:s1] = Bk.conj().T
            refl.append((s0, v2, t2))
            two_sided(s0, s1, v2, t2)
            r0, r1, v, t = s0, s1, v2, t2
    d = np.real(np.diag(A)).copy()
    e = np.real(np.diag(A, -1)).copy()
    assert np.abs(np.imag(np.diag(A, -1))).max() <= 1e-12 * max(1.0, np.abs(A).max())
    return d, e, refl, A


def apply_q2(refl, Z):
    Z = Z.astype(complex)
    for r0, v, t in reversed(refl):
        seg = Z[r0:r0 + len(v)]
        Z[r0:r0 + len(v)] = seg - t * np.outer(v, v.conj() @ seg)
    return Z


def apply_q1(blocks, Z):
    for r0, V, T in reversed(blocks):
        seg = Z[r0:]
        Z[r0:] = seg - V @ (T @ (V.conj().T @ seg))
    return Z


def heev2(A, nb=16):
    B, blocks = he2hb(A, nb)
    d, e, refl, Tm = hb2st(B, nb)
    n = A.shape[0]
    T = np.diag(d) + np.diag(e, -1) + np.diag(e, 1)
    lam, z = np.linalg.eigh(T)
    U = apply_q1(blocks, apply_q2(refl, z))
    return lam, U, B, (d, e), refl


if __name__ == "__main__":
    rng = np.random.default_rng(1)
    for n in (40, 64, 121, 256):
        X = rng.standard_normal((n, n)) + 1j * rng.standard_normal((n, n))
        A = (X + X.conj().T) / 2
        lam, U, B, (d, e), refl = heev2(A)
        l0 = np.linalg.eigvalsh(A)
        band = np.abs(np.tril(B, -17)).max()
        res = np.linalg.norm(A @ U - U * lam) / np.linalg.norm(A)
        orth = np.linalg.norm(U.conj().T @ U - np.eye(n))
        print(f"n {n}: eig err {np.abs(lam - l0).max():.2e} band leak {band:.1e} residual {res:.2e} "
              f"orth {orth:.2e} reflectors {len(refl)}")
