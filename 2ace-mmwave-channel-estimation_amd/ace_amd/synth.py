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


# ---- multiresolution probing codebooks ---------------------------------------------------------
# codebook/generate_tx_codebook_multires_16ant.py:47-120 and generate_rx_codebook_multires_16ant.py
# draw 2-bit phases per antenna GROUP, in three resolution tiers (groups of 4, 2 and 1 antennas;
# grouping :48, separation [32, 96, 160] rounds :59); processsing_codebook_multires.m builds each
# round's 62 probe rows as kron(tx row, the round's rx row) over the active antennas (two 8-element
# blocks of the 32-element array, id = [1..8, 17..24]).  The tiers hold 1984 / 3968 / 3968 rows
# (..._multiresolution.m:111-112) and the driver picks the tier by M (thresh [96, 256], :137-144).
# The 32-antenna analogue (config 5, builder-defined: the reference defines tiers for 16 antennas
# only) uses all four 8-element blocks with the same in-block grouping, 4x the rounds per tier
# (the array has 4x the unknowns) and 4x the thresholds.
ST_MR_TX, ST_MR_RX = 6, 7
MR_SECTORS = 62                          # probe rows per round (sector_per_cb, :62)
MR_ROUNDS = {16: (32, 64, 64), 32: (128, 256, 256)}
MR_THRESH = {16: (96, 256), 32: (384, 1024)}


def multires_tiers(tx):
    """(rows per tier, thresholds) of the multiresolution codebook for tx antennas per side."""
    if tx not in MR_ROUNDS:
        raise ValueError(f"multiresolution codebooks are defined for 16 and 32 antennas (got {tx})")
    return tuple(MR_SECTORS * r for r in MR_ROUNDS[tx]), MR_THRESH[tx]


def multires_tier_of(M, tx):
    """The tier ..._multiresolution.m:137-144 draws M rows from: 0 (M <= thresh[0]), 1, 2."""
    th = MR_THRESH[tx]
    return 0 if M <= th[0] else (1 if M <= th[1] else 2)


def multires_groups(tx, tier):
    """Group index of each antenna in a tier: within every 8-element block, groups
    [0,1,2,3] [4,5,6,7] (tier 0), [0,1] [2,3] [4,6] [5,7] (tier 1, the reference's [5,7],[6,8]
    pairs), single antennas (tier 2)."""
    a = np.arange(tx)
    blk, e = a // 8, a % 8
    if tier == 0:
        return 2 * blk + e // 4
    if tier == 1:
        return 4 * blk + np.array([0, 0, 1, 1, 2, 3, 2, 3])[e]
    return a


def multires_codes(seed, tx, rows):
    """Phase codes k (entry j^k) of the given global rows of the tx x tx multiresolution
    codebook, shape (len(rows), tx*tx), column t*tx + r = kron(tx row, rx row) (the vec(H)
    order of ``channel``).  Row p belongs to round p // 62; the tx phases are drawn per (row,
    group), the round's rx phases per (round, group)."""
    rows = np.asarray(rows, dtype=np.int64)
    lens, _ = multires_tiers(tx)
    bounds = np.cumsum(lens)
    if rows.size and (rows.min() < 0 or rows.max() >= bounds[-1]):
        raise ValueError("row index outside the codebook")
    tiers = np.searchsorted(bounds, rows, side="right")
    out = np.empty((rows.size, tx * tx), np.uint8)
    for t in range(3):
        sel = np.nonzero(tiers == t)[0]
        if sel.size == 0:
            continue
        g = multires_groups(tx, t)
        ng = int(g.max()) + 1
        p = rows[sel].astype(np.uint64)
        rnd = (rows[sel] // MR_SECTORS).astype(np.uint64)
        gg = np.arange(ng, dtype=np.uint64)
        ktx = (sm64(seed, ST_MR_TX, p[:, None] * np.uint64(ng) + gg[None, :]) >> np.uint64(62)).astype(np.uint8)
        krx = (sm64(seed, ST_MR_RX, rnd[:, None] * np.uint64(ng) + gg[None, :]) >> np.uint64(62)).astype(np.uint8)
        out[sel] = ((ktx[:, g][:, :, None] + krx[:, g][:, None, :]) % 4).reshape(sel.size, tx * tx)
    return out


def multires_codebook(seed, tx, rows):
    """A = j^k / sqrt(n) of the given rows (Random_Phase_State normalisation)."""
    k = multires_codes(seed, tx, rows)
    return (1j ** k.astype(np.int64)).astype(np.complex128) / np.sqrt(tx * tx)


def multires_rows(seed, tx, M):
    """The M codebook rows ..._multiresolution.m:137-144 draws for a sweep point: randperm within
    the tier M selects (M_idx = randperm(tier rows, M) + tier offset), from the build's RNG
    (ace_driver_randperm, stream 0x100 of the first sweep point).  Returns (rows, tier)."""
    from .engine import randperm
    lens, _ = multires_tiers(tx)
    tier = multires_tier_of(M, tx)
    return sum(lens[:tier]) + randperm(seed, 0x100, lens[tier], M).astype(np.int64), tier
