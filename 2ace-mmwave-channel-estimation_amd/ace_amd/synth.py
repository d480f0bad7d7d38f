"""Host-side synthetic traces, bit-compatible with the device generator
(csrc/ace_synth.hip) for every integer stream.

Semantics follow the reference generators:
  codebook  main/src/generate_sensing_matrix/Generate_Sensing_Matrix.m:85-122
            ('Random_Phase_State': exp(1j*2*pi*k/4)/sqrt(Nt*Nr), k ~ U{0..3})
  channel   main/src/generate_channel/Generate_Channel.m:64-164
            (L paths, AoD/AoA ~ U(-47.5, 47.5) deg, unit-norm CN gains,
             H = sqrt(Nt*Nr) ARx diag(h) ATx', vecH column-major)
  measure   main/src/generate_measurement/Generate_Measurement.m:67-136
            (B = |FW vecH + w|, w ~ CN(0, 10^(-SNR/10)))
  scaling   ``problem`` returns B, X0, vecH divided by ||B|| -- the normalisation
            InferADMM's inputs get (inferLowRankV4_multi.m:32-38)
The RNG is counter based: splitmix64(seed ^ stream*C1 + (ctr+1)*C2).
"""
from __future__ import annotations

import numpy as np

_C1 = np.uint64(0xD1B54A32D192ED03)
_C2 = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)

ST_CODEBOOK, ST_ANGLES, ST_GAINS, ST_NOISE, ST_X0 = 1, 2, 3, 4, 5
LAMBDA = 3e8 / 60.48e9          # channel_recovery_ADMM_v2_simulation_A2only.m:40
ANT_D = 3.055e-3                # :41
SEEDS = [58659179, 42737934, 36326041, 89830260, 90710947, 96474890, 33424536, 67991541, 42149446,
         38961924]              # first entries of the reference seed list (:103)


def stream_id(kind, real):
    return kind if real is None or real < 0 else kind + 16 * (real + 1)


def sm64(seed, stream, ctr):
    ctr = np.asarray(ctr, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = (np.uint64(seed) ^ (np.uint64(stream) * _C1)) + (ctr + np.uint64(1)) * _C2
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        return z ^ (z >> np.uint64(31))


def u01(seed, stream, ctr):
    return (sm64(seed, stream, ctr) >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)


def normal_pairs(seed, stream, count):
    c = np.arange(count, dtype=np.uint64)
    u1 = u01(seed, stream, 2 * c)
    u2 = u01(seed, stream, 2 * c + 1)
    r = np.sqrt(-2.0 * np.log(1.0 - u1))
    return r * np.cos(2.0 * np.pi * u2) + 1j * (r * np.sin(2.0 * np.pi * u2))


def codebook_codes(seed, m, n, real=None):
    """Phase-state indices k in {0..3}, shape (m, n)."""
    w = np.arange(m * n, dtype=np.uint64)
    return (sm64(seed, stream_id(ST_CODEBOOK, real), w) >> np.uint64(62)).astype(np.uint8).reshape(m, n)


def codebook(seed, m, n, real=None):
    """A[m][n] = j^k / sqrt(n) (complex128)."""
    k = codebook_codes(seed, m, n, real)
    return (1j ** k.astype(np.int64)).astype(np.complex128) / np.sqrt(n)


def channel(seed, real, tx, rx, L=3):
    """vecH (n = tx*rx), element r + rx*t = H[r][t] (Generate_Channel.m:140-160)."""
    st = stream_id(ST_ANGLES, real)
    u = u01(seed, st, np.arange(2 * L, dtype=np.uint64))
    aod = (u[:L] - 0.5) * 95.0
    aoa = (u[L:] - 0.5) * 95.0
    sd, sa = np.sin(aod * np.pi / 180.0), np.sin(aoa * np.pi / 180.0)
    g = normal_pairs(seed, stream_id(ST_GAINS, real), L) * np.sqrt(0.5)
    g = g / np.sqrt(np.sum(np.abs(g) ** 2))
    kap = 2.0 * np.pi * (ANT_D / LAMBDA)
    k = np.arange(tx * rx)
    r, t = k % rx, k // rx
    ph = kap * (sd[None, :] * t[:, None] - sa[None, :] * r[:, None])
    return np.sum(g[None, :] * (np.cos(ph) + 1j * np.sin(ph)), axis=1)


def measurements(seed, real, A, vecH, snr_db=30.0):
    m = A.shape[0]
    sigma2 = 10.0 ** (-snr_db / 10.0)
    w = normal_pairs(seed, stream_id(ST_NOISE, real), m) * np.sqrt(sigma2 * 0.5)
    return np.abs(A @ vecH + w)


def initial_iterate(seed, real, vecH, x0_noise=0.5):
    n = vecH.size
    z = normal_pairs(seed, stream_id(ST_X0, real), n)
    return vecH + z * (x0_noise * np.linalg.norm(vecH) / np.sqrt(n) * np.sqrt(0.5))


def problem(seed, first, count, m, tx, rx, *, a_shared=True, L=3, snr_db=30.0, x0_noise=0.5):
    """Host copy of one synthetic batch: A ([1 or count] x m x n), B, X0, vecH."""
    n = tx * rx
    if a_shared:
        A = codebook(seed, m, n)[None]
    else:
        A = np.stack([codebook(seed, m, n, first + c) for c in range(count)])
    H = np.stack([channel(seed, first + c, tx, rx, L) for c in range(count)])
    B = np.stack([measurements(seed, first + c, A[0 if a_shared else c], H[c], snr_db) for c in range(count)])
    X0 = np.stack([initial_iterate(seed, first + c, H[c], x0_noise) for c in range(count)])
    # InferADMM always sees B / ||B|| (inferLowRankV4_multi.m:32-38); A already has ||A||_F = sqrt(m)
    nb = np.sqrt(np.sum(B * B, axis=1))
    return A, B / nb[:, None], X0 / nb[:, None], H / nb[:, None]
