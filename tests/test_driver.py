"""Driver-level boundary (ace_recover_driver / ace_amd.engine) -- host logic on CPU.

Reference: main/channel_recovery_ADMM_v2_simulation_A2only.m:106-118 (M sweep, error
:117), :137 (randperm), multiresolution tiers ..._multiresolution.m:111-112/:137-144,
and the MATLAB Engine call shape of main/main.py:427-437.  These checks run before any
GPU work, so they need no device.
"""
import numpy as np
import pytest

from ace_amd import engine, AceError


def test_m_sweep_matches_reference_formula():
    # round(linspace(2, sqrt(4*tx*rx), 8)).^2
    assert engine.m_sweep(32, 32).tolist() == [4, 121, 400, 841, 1369, 2116, 3025, 4096]
    assert engine.m_sweep(16, 16).tolist() == [4, 36, 121, 225, 361, 529, 784, 1024]
    for a in (4, 8, 16, 32, 36):
        ref = np.round(np.linspace(2, np.sqrt(4 * a * a), 8)) ** 2
        assert engine.m_sweep(a, a).tolist() == ref.astype(int).tolist()


def test_m_sweep_rejects_other_arrays():
    with pytest.raises(engine.MatlabExecutionError, match="4/8/16/32"):
        engine.m_sweep(5, 5)


def test_randperm_is_a_permutation_prefix():
    a = engine.randperm(58659179, 7, 100, 100)
    assert sorted(a.tolist()) == list(range(100))
    b = engine.randperm(58659179, 7, 1000, 60)
    assert len(set(b.tolist())) == 60 and b.min() >= 0 and b.max() < 1000
    assert np.array_equal(b, engine.randperm(58659179, 7, 1000, 60))           # deterministic
    assert not np.array_equal(b, engine.randperm(58659179, 8, 1000, 60))       # stream-dependent
    # uniformity: every index equally likely at position 0 (chi-square, loose bound)
    first = np.array([engine.randperm(1, s, 8, 1)[0] for s in range(4000)])
    cnt = np.bincount(first, minlength=8)
    assert ((cnt - 500) ** 2 / 500).sum() < 40


def _trace(P, n, seed=0):
    rng = np.random.default_rng(seed)
    amp = np.ones((P, n))
    ang = rng.integers(0, 4, (P, n)) * (np.pi / 2)
    rss = rng.uniform(-70, -40, P)
    return amp, ang, rss


def test_driver_argument_errors_need_no_gpu():
    eng = engine.start_matlab()
    amp, ang, rss = _trace(64, 256)
    with pytest.raises(engine.MatlabExecutionError, match="seed_id"):
        eng.channel_recovery_ADMM_v2_simulation_A2only(16, 16, amp, ang, rss, 0, nargout=2)
    with pytest.raises(engine.MatlabExecutionError, match="4/8/16/32"):
        eng.channel_recovery_ADMM_v2_simulation_A2only(5, 5, amp[:, :25], ang[:, :25], rss, 1, nargout=2)
    with pytest.raises(engine.MatlabExecutionError, match="M = "):
        eng.channel_recovery_ADMM_v2_simulation_A2only(16, 16, amp, ang, rss, 1, nargout=2)   # M up to 1024 > P
    with pytest.raises(engine.MatlabExecutionError, match="multiresolution codebook needs"):
        eng.channel_recovery_ADMM_v2_simulation_multiresolution(16, 16, amp, ang, rss, 1, nargout=2)
    with pytest.raises(engine.MatlabExecutionError, match="shapes"):
        eng.channel_recovery_ADMM_v2_simulation_A2only(16, 16, amp[:, :10], ang, rss, 1, nargout=2)
    with pytest.raises(engine.MatlabExecutionError, match="M = "):
        eng.channel_recovery_ADMM_v2_simulation_phaselift(16, 16, amp, ang, rss, 1, nargout=2)
    with pytest.raises(AceError, match="unknown driver"):
        engine.recover(7, 16, 16, amp, ang, rss, 1)
    with pytest.raises(engine.MatlabExecutionError, match="nargout"):
        eng.channel_recovery_ADMM_v2_simulation_A2only(16, 16, amp, ang, rss, 1, nargout=1)


def test_engine_double_shim():
    eng = engine.start_matlab()
    assert eng.double(3) == 3.0 and isinstance(eng.double(3), float)
    assert engine.double([[1, 2]]).dtype == np.float64
