"""CPU tests of the beamformer oracle against the reference's own
outputs (tests/golden/beamformer_ref.npz, made by importing main/codebook_library.py —
tests/golden/make_beam_golden.py) and of the LAPACK restatement against numpy itself.

The restatement (oracle/beamformer_oracle.py: zgebd2 -> dbdsqr -> zunmbr) is what the HIP
kernel implements; pinning it to numpy.linalg.svd pins the phase/sign convention the 2-bit
codes depend on."""
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
    """The LAPACK restatement reproduces the reference's codes for n <= 25 exactly; for
    n = 32 (numpy switches to divide and conquer) up to a per-beam code offset of 0 or 2."""
    for name, H, off, wr, wt in _groups():
        for k in range(len(H)):
            a, b, *_ = BO.svd_beamformer(H[k], None if off is None else off[k], vh_fn=BO.gesdd_vh)
            if H.shape[1] <= 25:
                assert (a == wr[k]).all() and (b == wt[k]).all(), (name, k)
            else:
                for got, exp in ((a, wr[k]), (b, wt[k])):
                    d = (got.astype(int) - exp.astype(int)) % 4
                    assert np.all(d == d[0]) and d[0] in (0, 2), (name, k)


@pytest.mark.parametrize("n", [1, 2, 5, 16, 24])
def test_restated_vh_equals_numpy(n):
    rng = np.random.default_rng(100 + n)
    for _ in range(20):
        A = rng.standard_normal((n, n)) + 1j * rng.standard_normal((n, n))
        np.testing.assert_allclose(BO.gesdd_vh(A), np.linalg.svd(A)[2], atol=1e-11)


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
