"""GPU: the driver-level boundary (ace_recover_driver via ace_amd.engine) against the
same steps composed by hand and against the oracle pipeline.

Reference: main/channel_recovery_ADMM_v2_simulation_A2only.m:120-178 (cb = amp.*exp(j*angle),
rss_train = sqrt(db2pow(rss)/1000)*rss_fct, ADMM_v2 version 4 -> inferLowRankV4_multi,
H = X/rss_fct, NaN -> 0) and ..._multiresolution.m:111-112/:137-144 (row tiers).  The row
draws are the build's RNG (MATLAB's randperm stream is not reproducible), so the
composition re-draws them with the same (seed, stream) through the C-ABI.
"""
import math

import numpy as np
import pytest

import ace_oracle as O

pytestmark = pytest.mark.gpu

SEEDS = [58659179, 42737934, 36326041]
RSS_FCT = 1e5 / 3


def _trace(P, tx, seed=5):
    from ace_amd import synth
    n = tx * tx
    A = synth.codebook(seed, P, n) * math.sqrt(n)            # unit-modulus QPSK rows, like cb
    h = synth.channel(seed, 0, tx, tx)
    y = np.abs(A @ h) * 1e-4                                 # RSS amplitude, ~-60 dBm
    return np.abs(A), np.angle(A), 10 * np.log10(1000 * y ** 2)


def _snap(v):
    """The driver's exp(1j*angle) components (ace_driver.cpp::snap_unit): a rounding residue of a
    phase-code angle (cos(pi/2) = 6.1e-17) snapped to the exact 0 / +-1 it stands for."""
    v = np.where(np.abs(v) < 1e-15, 0.0, v)
    return np.where(np.abs(np.abs(v) - 1.0) <= 4 * np.finfo(float).eps, np.sign(v), v)


def _cb(amp, ang):
    return amp * (_snap(np.cos(ang)) + 1j * _snap(np.sin(ang)))


def _ref_codebook(key):
    """The reference's probing codebook (tests/golden/ref_codebooks_16x16_packed.npz, 2-bit codes
    of codebook/codebook_mat/random_probe_cb_16x16{,_multires}.mat) as main.py hands it to the
    driver: |cb| and angle(cb) (main.py:301-302)."""
    from conftest import ROOT
    p = np.load(ROOT / "tests" / "golden" / "ref_codebooks_16x16_packed.npz")[key]
    k = np.stack([(p >> (2 * i)) & 3 for i in range(4)], axis=-1).reshape(p.shape[0], -1).astype(np.int64)
    cb = np.exp(1j * np.pi / 2 * k)                          # MATLAB exp(1j*pi/2*phase): cos/sin residues
    return k, np.abs(cb), np.angle(cb)


def _compose(amp, ang, rss, tx, seed, points, tier=None):
    """The driver's steps by hand for sweep points [(i, M)], through the pipeline host API."""
    from ace_amd import engine, infer_low_rank_pipeline_host
    out = []
    for i, M in points:
        off, avail = 0, amp.shape[0]
        if tier is not None:
            off, avail = tier(M)
        idx = engine.randperm(seed, 0x100 + 2 * i, avail, M) + off
        A = _cb(amp, ang)[idx]
        # libm pow as the C++ driver (numpy's power may differ by an ulp)
        B = np.array([math.sqrt(math.pow(10.0, x / 10.0) / 1000.0) * RSS_FCT for x in rss[idx]])
        mt = math.floor(0.95 * M)
        tr = np.stack([engine.randperm(seed, 0x101 + 2 * i + 0x10000 * s, M, mt) for s in range(3)])
        res = infer_low_rank_pipeline_host(A, B[None], tx, tx, tr)
        out.append((res.X[0] / RSS_FCT, A, B, tr))
    return out


def test_driver_explicit_sweep(gpu):
    from ace_amd import engine
    tx = 16
    amp, ang, rss = _trace(400, tx)
    Ms = [121, 225]
    Ha, Hp = engine.recover(engine.DRIVER_A2ONLY, tx, tx, amp, ang, rss, 1, M_list=Ms)
    assert Ha.shape == (2, 1, 256)
    H = np.squeeze(Ha * np.exp(1j * Hp))                     # main.py:428-430
    for i, (Xc, A, B, tr) in enumerate(_compose(amp, ang, rss, tx, SEEDS[0], list(enumerate(Ms)))):
        assert O.phase_aligned_rel_err(H[i], Xc) <= 1e-12       # amp/angle round trip only
    # oracle parity where the oracle is stable against itself (M = 121: 1e-15 input
    # perturbations move it by ~1e-9; M = 225 on this noiseless trace is rounding-chaotic)
    Xc, A, B, tr = _compose(amp, ang, rss, tx, SEEDS[0], [(0, Ms[0])])[0]
    ref = O.infer_low_rank_pipeline(A, B, tx, tx, list(tr))
    assert O.phase_aligned_rel_err(H[0], ref.X / RSS_FCT) <= 1e-5


def test_driver_default_sweep_16ant(gpu):
    """The reference sweep (8 points up to M = 1024) through the engine shim; M = 4 is
    ill-posed for the spectral initialisation and comes back 0 (the reference's NaN -> 0)."""
    from ace_amd import engine
    tx = 16
    amp, ang, rss = _trace(1024, tx)
    eng = engine.start_matlab()
    Ha, Hp = eng.channel_recovery_ADMM_v2_simulation_A2only(tx, tx, engine.double(amp), engine.double(ang),
                                                            engine.double(rss[:, None]), eng.double(2), nargout=2)
    assert Ha.shape == (8, 1, 256)
    assert np.all(Ha[0] == 0) and np.all(np.isfinite(Ha)) and np.all(Ha[1:].max(axis=-1) > 0)
    H = np.squeeze(Ha * np.exp(1j * Hp))
    Ms = engine.m_sweep(tx, tx)
    for (Xc, _, _, _), i in zip(_compose(amp, ang, rss, tx, SEEDS[1], [(1, Ms[1]), (2, Ms[2])]), (1, 2)):
        assert O.phase_aligned_rel_err(H[i], Xc) <= 1e-12


def test_driver_multiresolution_tiers(gpu):
    from ace_amd import engine
    tx = 16
    amp, ang, rss = _trace(9920, tx, seed=9)
    Ms = [64, 121, 300]
    Ha, Hp = engine.recover(engine.DRIVER_MULTIRES, tx, tx, amp, ang, rss, 1, M_list=Ms)
    H = np.squeeze(Ha * np.exp(1j * Hp))

    def tier(M):  # thresh [96, 256], res_separation [1984, 3968, 3968]
        return (0, 1984) if M <= 96 else ((1984, 3968) if M <= 256 else (1984 + 3968, 3968))

    for i, (Xc, _, _, _) in enumerate(_compose(amp, ang, rss, tx, SEEDS[0], list(enumerate(Ms)), tier)):
        assert O.phase_aligned_rel_err(H[i], Xc) <= 1e-12


NUCLEAR_SEEDS = [1024, 2048, 4096, 8192]   # ..._A2nuclear.m:103 (the build picks seeds((seed_id - 1) % 4 + 1))


def _compose_nuclear(amp, ang, rss, tx, seed, points, maxiter=500):
    """channel_recovery_ADMM_v2_simulation_A2nuclear's steps by hand (ADMM_v2_nuclear.m:30-32 ->
    inferLowRank_Nuclear: one restart, one partition)."""
    from ace_amd import engine, infer_low_rank_pipeline_host
    out = []
    for i, M in points:
        idx = engine.randperm(seed, 0x100 + 2 * i, amp.shape[0], M)
        A = _cb(amp, ang)[idx]
        B = np.array([math.sqrt(math.pow(10.0, x / 10.0) / 1000.0) * RSS_FCT for x in rss[idx]])
        tr = engine.randperm(seed, 0x101 + 2 * i, M, math.floor(0.95 * M))[None]
        res = infer_low_rank_pipeline_host(A, B[None], tx, tx, tr, variant="A2nuclear", maxiter=maxiter)
        out.append((res.X[0] / RSS_FCT, A, B, tr))
    return out


def test_driver_nuclear_matches_composition_and_oracle(gpu):
    """channel_recovery_ADMM_v2_simulation_A2nuclear (:104 rows, :158 ADMM_v2_nuclear): equal to the hand
    composition through the pipeline host API at the reference's 500 iterations (two sweep points, run
    concurrently by the driver), and to the oracle's nuclear pipeline where the oracle is stable against
    its own rounding: 25 iterations per stage (a 1e-15 relative change of B moves the oracle's X by
    2e-11 at M = 121 and 3e-9 at M = 225 there, 7e-5 / 0.93 at 60: the nuclear refinement is
    rounding-chaotic)."""
    from ace_amd import engine
    tx = 16
    amp, ang, rss = _trace(400, tx)
    Ms = [121, 225]
    seed = NUCLEAR_SEEDS[(3 - 1) % 4]
    Ha, Hp = engine.recover(engine.DRIVER_A2NUCLEAR, tx, tx, amp, ang, rss, 3, M_list=Ms)
    assert Ha.shape == (2, 1, 256) and np.all(np.isfinite(Ha)) and np.all(Ha.max(axis=-1) > 0)
    H = np.squeeze(Ha * np.exp(1j * Hp))
    for i, (Xc, _, _, _) in enumerate(_compose_nuclear(amp, ang, rss, tx, seed, list(enumerate(Ms)))):
        assert O.phase_aligned_rel_err(H[i], Xc) <= 1e-12, i
    Ha, Hp = engine.recover(engine.DRIVER_A2NUCLEAR, tx, tx, amp, ang, rss, 3, M_list=Ms, maxiter=25)
    H = np.squeeze(Ha * np.exp(1j * Hp))
    for i, (Xc, A, B, tr) in enumerate(_compose_nuclear(amp, ang, rss, tx, seed, list(enumerate(Ms)), maxiter=25)):
        assert O.phase_aligned_rel_err(H[i], Xc) <= 1e-12, i
        ref = O.infer_low_rank_pipeline(A, B, tx, tx, list(tr), variant=O.VARIANT_NUCLEAR, maxiter=25)
        e = O.phase_aligned_rel_err(H[i], ref.X / RSS_FCT)
        assert e <= 1e-6, (Ms[i], e)


def test_driver_phaselift(gpu):
    """channel_recovery_ADMM_v2_simulation_phaselift: rng(4096) rows, MyPhaseLift per sweep point
    with Recover_Channel.m:34's scaling; equals the composition through phaselift_host."""
    from ace_amd import engine, phaselift_host
    tx = 8
    amp, ang, rss = _trace(200, tx)
    Ha, Hp = engine.recover(engine.DRIVER_PHASELIFT, tx, tx, amp, ang, rss, 5, M_list=[36])
    H = np.squeeze(Ha * np.exp(1j * Hp))
    idx = engine.randperm(4096, 0x100, 200, 36)
    A = _cb(amp, ang)[idx]
    B = np.array([math.sqrt(math.pow(10.0, x / 10.0) / 1000.0) * RSS_FCT for x in rss[idx]])
    sig = phaselift_host(A, ((B / 2e5) ** 2 * 1e10)[None]).sig[0] / math.sqrt(1e10) * 2e5
    assert O.phase_aligned_rel_err(H, sig / RSS_FCT) <= 1e-12


def test_driver_reference_probe_codebook_int8_path(gpu):
    """main.py's input path on the reference's own probing codebook (random_probe_cb_16x16.mat,
    3968 x 256, handed over as |cb| / angle(cb)): the reference sweep through the engine shim.
    The refinement solves run on the exact int8 phase-code applies (the snapped |cb| / angle(cb)
    is the exact phase code again), and the M = 121 point matches the oracle pipeline on the same rows (1e-5)."""
    from ace_amd import engine, path_counts
    tx = 16
    k, amp, ang = _ref_codebook("random")
    cb = (1j ** k).astype(complex)
    assert np.abs(np.cos(ang)).min() > 0 and np.abs(np.cos(ang)).min() < 1e-15   # MATLAB-style residues
    h = __import__("ace_amd").synth.channel(17, 0, tx, tx)
    rss = 10 * np.log10(1000 * (np.abs(cb @ h) * 1e-4) ** 2)
    path_counts(reset=True)
    eng = engine.start_matlab()
    Ha, Hp = eng.channel_recovery_ADMM_v2_simulation_A2only(tx, tx, engine.double(amp), engine.double(ang),
                                                            engine.double(rss[:, None]), eng.double(3), nargout=2)
    pc = path_counts(reset=True)
    assert Ha.shape == (8, 1, 256) and np.all(np.isfinite(Ha)) and np.all(Ha[1:].max(axis=-1) > 0)
    # one refinement per well-posed point on the int8 applies: M = 36 ... 529 (M = 4 is ill-posed and
    # skipped; M = 784, 1024 exceed the int8 A^H kernel's LDS-resident K, i8ah_lds_bytes, and run f64)
    assert pc["int8_shared"] == 5 and pc["f64_private"] == 0, pc
    H = np.squeeze(Ha * np.exp(1j * Hp))
    Ms = engine.m_sweep(tx, tx)
    Xc, A, B, tr = _compose(amp, ang, rss, tx, SEEDS[2], [(2, Ms[2])])[0]
    assert np.array_equal(A, cb[engine.randperm(SEEDS[2], 0x100 + 4, 3968, Ms[2])])   # snapped: exact j^k
    assert O.phase_aligned_rel_err(H[2], Xc) <= 1e-12
    ref = O.infer_low_rank_pipeline(A, B, tx, tx, list(tr))
    assert O.phase_aligned_rel_err(H[2], ref.X / RSS_FCT) <= 1e-5


def test_driver_reference_multires_codebook(gpu):
    """channel_recovery_ADMM_v2_simulation_multiresolution on the reference's multiresolution
    codebook (random_probe_cb_16x16_multires.mat, 9920 x 256 in tiers of 1984 / 3968 / 3968 rows):
    one sweep point per tier, each equal to the hand composition with the tiered rows."""
    from ace_amd import engine
    tx = 16
    k, amp, ang = _ref_codebook("multires")
    cb = (1j ** k).astype(complex)
    h = __import__("ace_amd").synth.channel(19, 0, tx, tx)
    rss = 10 * np.log10(1000 * (np.abs(cb @ h) * 1e-4) ** 2)
    Ms = [64, 121, 300]
    Ha, Hp = engine.recover(engine.DRIVER_MULTIRES, tx, tx, amp, ang, rss, 1, M_list=Ms)
    H = np.squeeze(Ha * np.exp(1j * Hp))

    def tier(M):
        return (0, 1984) if M <= 96 else ((1984, 3968) if M <= 256 else (1984 + 3968, 3968))

    for i, (Xc, _, _, _) in enumerate(_compose(amp, ang, rss, tx, SEEDS[0], list(enumerate(Ms)), tier)):
        assert np.all(np.isfinite(Xc))
        assert O.phase_aligned_rel_err(H[i], Xc) <= 1e-12, i
