"""CPU tests of the beamformer oracle against the reference's own
outputs (tests/golden/beamformer_ref.npz, made by importing main/codebook_library.py —
tests/golden/make_beam_golden.py) and of the LAPACK restatement against numpy itself.

The restatement (oracle/beamformer_oracle.py: zgebd2 -> dbdsqr [-> the divide-and-conquer
merge's signs for n > 25] -> zunmbr) is what the HIP kernel implements; pinning it to
numpy.linalg.svd pins the phase/sign convention the 2-bit codes depend on."""
import pathlib

import numpy as np
import pytest

import beamformer_oracle as BO

GOLD = pathlib.Path(__file__).resolve().parent / "golden" / "beamformer_ref.npz"


def _groups():
    z = np.load(GOLD)
    for name in z["names"]:
        name = str(name)
        off = z[f"{name}__offset"] if f"{name}__offset" in z.files else None
        yield name, z[f"{name}__H"], off, z[f"{name}__wr"], z[f"{name}__wt"]


@pytest.mark.parametrize("name", [g[0] for g in _groups()])
def test_oracle_matches_reference_codes(name):
    """numpy-backed oracle == reference svd_beamformer(_compensation) strings, every case."""
    for gname, H, off, wr, wt in _groups():
        if gname != name:
            continue
        for k in range(len(H)):
            a, b, *_ = BO.svd_beamformer(H[k], None if off is None else off[k])
            assert (a == wr[k]).all() and (b == wt[k]).all(), (name, k)


def test_restated_gesdd_reproduces_reference_codes():
    """The LAPACK restatement reproduces the reference's codes exactly, n = 32 (numpy's
    divide-and-conquer path: the dlasd1 merge's sign convention) included."""
    for name, H, off, wr, wt in _groups():
        for k in range(len(H)):
            a, b, *_ = BO.svd_beamformer(H[k], None if off is None else off[k], vh_fn=BO.gesdd_vh)
            assert (a == wr[k]).all() and (b == wt[k]).all(), (name, k)


@pytest.mark.parametrize("n", [1, 2, 5, 16, 24, 25, 26, 29, 31, 32])
def test_restated_vh_equals_numpy(n):
    rng = np.random.default_rng(100 + n)
    for _ in range(20 if n <= 25 else 8):
        A = rng.standard_normal((n, n)) + 1j * rng.standard_normal((n, n))
        np.testing.assert_allclose(BO.gesdd_vh(A), np.linalg.svd(A)[2], atol=1e-11)


@pytest.mark.parametrize("n", [26, 32])
def test_divide_and_conquer_signs_on_structured_inputs(n):
    """n > 25: the merge's sign rule on real, low-rank-plus-noise and exactly rank-one inputs.  Every
    vector matches numpy where the merge deflates nothing; an exactly rank-one H deflates its null
    space (which is degenerate: any basis is a valid SVD, and LAPACK's is not reproduced), yet the
    beam codes -- the top pair -- still match."""
    rng = np.random.default_rng(200 + n)
    for kind in ("real", "rank1noise", "rank1"):
        for _ in range(4):
            if kind == "real":
                H = rng.standard_normal((n, n)) + 0j
            else:
                u = rng.standard_normal((n, 1)) + 1j * rng.standard_normal((n, 1))
                v = rng.standard_normal((1, n)) + 1j * rng.standard_normal((1, n))
                H = u @ v + (1e-2 if kind == "rank1noise" else 0.0) * (rng.standard_normal((n, n)) + 1j * rng.standard_normal((n, n)))
            if kind != "rank1":
                np.testing.assert_allclose(BO.gesdd_vh(H), np.linalg.svd(H)[2], atol=1e-10)
            a, b, *_ = BO.svd_beamformer(H, vh_fn=BO.gesdd_vh)
            ra, rb, *_ = BO.svd_beamformer(H)
            assert (a == ra).all() and (b == rb).all(), kind


@pytest.mark.parametrize("m,n", [(16, 4), (4, 16), (12, 8), (8, 12), (32, 16), (16, 32), (20, 32), (32, 26),
                                 (26, 32), (1, 8), (8, 1), (2, 3), (5, 9), (24, 31), (31, 17)])
def test_restated_rectangular_vh_equals_numpy(m, n):
    """tx != rx: zgesdd's QR-first / LQ-first / direct paths (gesdd_vh_rect) against numpy.  A row may
    differ by its sign only where numpy's own choice is rounding-sensitive (it flips under a 1e-15
    relative perturbation of the input): checked, not assumed."""
    rng = np.random.default_rng(300 + 37 * m + n)
    for _ in range(6):
        A = rng.standard_normal((m, n)) + 1j * rng.standard_normal((m, n))
        got, ref = BO.gesdd_vh_rect(A), np.linalg.svd(A)[2]
        bad = np.abs(got - ref).max(axis=1) > 1e-9
        if bad.any():
            assert np.abs(got[bad] + ref[bad]).max() < 1e-9
            per = np.linalg.svd(A * (1 + 1e-15))[2]
            assert (np.abs(per[bad] - ref[bad]).max(axis=1) > 1e-9).all()


def test_dlartg_and_dlasv2_identities():
    c, s, r = BO.dlartg(-3.0, 4.0)           # 3.10+ convention: c >= 0, r has the sign of f
    assert c > 0 and r == -5.0 and abs(c * -3.0 + s * 4.0 - r) < 1e-15
    rng = np.random.default_rng(5)
    for _ in range(200):
        f, g, h = rng.standard_normal(3) * 10.0 ** rng.integers(-3, 3, 3)
        ssmin, ssmax, snr, csr, snl, csl = BO.dlasv2(f, g, h)
        B = np.array([[f, g], [0.0, h]])
        L = np.array([[csl, snl], [-snl, csl]])
        R = np.array([[csr, snr], [-snr, csr]])
        np.testing.assert_allclose(L @ B @ R.T, np.diag([ssmax, ssmin]), atol=1e-12 * abs(B).max())


def test_codebook_beams_structure():
    rng = np.random.default_rng(9)
    H_est = rng.standard_normal((3, 16)) + 1j * rng.standard_normal((3, 16))
    wr, wt = BO.codebook_beams(H_est, H_est[:1], 4, 4, compensation=np.array([0, 1, 2, 3]))
    assert len(wr) == len(wt) == 4 and all(len(s) == 4 and set(s) <= set("0123") for s in wr + wt)
    a, b, *_ = BO.svd_beamformer(H_est[1].reshape(4, 4))
    assert wr[1] == BO.codes_to_str(a) and wt[1] == BO.codes_to_str(b)
