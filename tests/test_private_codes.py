"""Host-side checks of the private phase-code arithmetic (ace_private.hip, no GPU):

* pc_k_kernel's 2-bit SWAR difference count: for phase codes a_ik = c j^(k_ik),
  K_il = sum_k a_ik conj(a_lk) = c^2 sum_k j^((k_ik - k_lk) mod 4) = c^2 ((n0 - n2) + j (n1 - n3)),
  with n_d counted 16 codes per dword via  lo = (a ^ b) & L,  hi = (((a ^ b) >> 1) ^ (~a & b)) & L;
* the v_perm code lookups (LUT_P / LUT_Q / LUT_NQ) give the 2x2 real expansion of A and A^H.
"""
import numpy as np

L55 = 0x55555555


def _pack(codes):
    w = 0
    for u, c in enumerate(codes):
        w |= int(c) << (2 * u)
    return w


def _swar_counts(a, b):
    xo = a ^ b
    lo = xo & L55
    hi = ((xo >> 1) ^ (~a & b & 0xFFFFFFFF)) & L55
    pc = lambda v: bin(v & 0xFFFFFFFF).count("1")
    return pc(lo & ~hi), pc(hi & ~lo), pc(lo & hi)


def test_swar_difference_counts():
    rng = np.random.default_rng(0)
    for _ in range(2000):
        ka, kb = rng.integers(0, 4, 16), rng.integers(0, 4, 16)
        n1, n2, n3 = _swar_counts(_pack(ka), _pack(kb))
        d = (ka - kb) % 4
        assert (n1, n2, n3) == ((d == 1).sum(), (d == 2).sum(), (d == 3).sum())


def test_k_from_codes_equals_product():
    rng = np.random.default_rng(1)
    m, n = 12, 48
    k = rng.integers(0, 4, (m, n))
    A = (1j ** k) / np.sqrt(n)
    K = A @ A.conj().T
    words = [[_pack(k[i, 16 * w:16 * w + 16]) for w in range(n // 16)] for i in range(m)]
    Kc = np.zeros((m, m), complex)
    for i in range(m):
        for l in range(m):
            c = np.array([_swar_counts(words[i][w], words[l][w]) for w in range(n // 16)]).sum(axis=0)
            n0 = n - c.sum()
            Kc[i, l] = ((n0 - c[1]) + 1j * (c[0] - c[2])) / n
    assert np.abs(Kc - K).max() < 1e-14


def _lut(v, code):
    return np.int8(np.uint8((v >> (8 * code)) & 0xFF))


def test_code_lookups_are_the_real_expansion():
    LUT_P, LUT_Q, LUT_NQ = 0x00FF0001, 0xFF000100, 0x0100FF00
    for code in range(4):
        a = 1j ** code
        p, q = a.real, a.imag
        assert (_lut(LUT_P, code), _lut(LUT_Q, code), _lut(LUT_NQ, code)) == (round(p), round(q), round(-q))
        # A^H lanes: Re conj(a) g = p x + q y, Im conj(a) g = -q x + p y
        g = 0.3 - 1.7j
        assert np.isclose(_lut(LUT_P, code) * g.real + _lut(LUT_Q, code) * g.imag, (np.conj(a) * g).real)
        assert np.isclose(_lut(LUT_NQ, code) * g.real + _lut(LUT_P, code) * g.imag, (np.conj(a) * g).imag)
        # A lanes: Re a v = p x - q y, Im a v = q x + p y
        assert np.isclose(_lut(LUT_P, code) * g.real + _lut(LUT_NQ, code) * g.imag, (a * g).real)
        assert np.isclose(_lut(LUT_Q, code) * g.real + _lut(LUT_P, code) * g.imag, (a * g).imag)
