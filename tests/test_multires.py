"""The multiresolution probing codebooks (ace_amd.synth.multires_*): the reference's 16-antenna
layout, pinned by the reference's own codebook, and the 32-antenna analogue configs[4] uses.

Reference: codebook/generate_tx_codebook_multires_16ant.py:47-120 (and the rx twin) draw 2-bit
phases per antenna group in three tiers; processsing_codebook_multires.m builds each round's 62
probe rows as kron(tx row, the round's rx row) over the 16 active antennas;
main/channel_recovery_ADMM_v2_simulation_multiresolution.m:111-112,137-144 picks the tier by M.
The fixture is codebook/codebook_mat/random_probe_cb_16x16_multires.mat as 2-bit codes
(tests/golden/ref_codebooks_16x16_packed.npz)."""
import numpy as np
import pytest

from ace_amd import synth
from conftest import ROOT


def _unpack(p):
    return np.stack([(p >> (2 * i)) & 3 for i in range(4)], axis=-1).reshape(p.shape[0], -1).astype(np.int64)


def _check_structure(codes, tx, first_row=0):
    """Every row is kron(tx phases, rx phases) with the phases constant on the tier's antenna groups,
    and the 62 rows of a round share the rx phases."""
    lens, _ = synth.multires_tiers(tx)
    bounds = np.cumsum(lens)
    rx_of_round = {}
    for i, code in enumerate(codes):
        row = first_row + i
        t = int(np.searchsorted(bounds, row, side="right"))
        C = code.reshape(tx, tx)                     # C[t_ant, r_ant] (column t*tx + r)
        a, b = (C[:, 0] - C[0, 0]) % 4, C[0, :] % 4
        assert np.array_equal((a[:, None] + b[None, :]) % 4, C), row
        g = synth.multires_groups(tx, t)
        for gg in range(g.max() + 1):
            assert len(set(a[g == gg])) == 1 and len(set(b[g == gg])) == 1, (row, gg)
        rnd = row // synth.MR_SECTORS
        rb = (b - b[0]) % 4
        assert np.array_equal(rx_of_round.setdefault(rnd, rb), rb), row


def test_reference_multires_codebook_has_the_generator_layout():
    g = np.load(ROOT / "tests" / "golden" / "ref_codebooks_16x16_packed.npz")
    codes = _unpack(g["multires"])
    lens, th = synth.multires_tiers(16)
    assert codes.shape == (sum(lens), 256) and lens == (1984, 3968, 3968) and th == (96, 256)
    _check_structure(codes, 16)


@pytest.mark.parametrize("tx", [16, 32])
def test_generator_layout(tx):
    lens, _ = synth.multires_tiers(tx)
    rows = np.concatenate([np.arange(130), lens[0] + np.arange(130), lens[0] + lens[1] + np.arange(130)])
    codes = synth.multires_codes(11, tx, rows)
    for k, start in enumerate((0, lens[0], lens[0] + lens[1])):
        _check_structure(codes[130 * k: 130 * (k + 1)], tx, start)
    # row-addressable: any subset of rows reproduces the same codes
    sub = rows[::7]
    assert np.array_equal(synth.multires_codes(11, tx, sub), codes[::7])
    # uniform 2-bit phases
    cnt = np.bincount(codes.ravel(), minlength=4) / codes.size
    assert np.all(np.abs(cnt - 0.25) < 0.03)


def test_tiers_and_rows():
    assert synth.multires_tiers(32) == ((7936, 15872, 15872), (384, 1024))
    assert [synth.multires_tier_of(M, 16) for M in (96, 97, 256, 257)] == [0, 1, 1, 2]
    assert [synth.multires_tier_of(M, 32) for M in (256, 384, 385, 1024, 4096)] == [0, 0, 1, 1, 2]
    rows, tier = synth.multires_rows(5, 32, 256)
    assert tier == 0 and len(set(rows.tolist())) == 256 and rows.min() >= 0 and rows.max() < 7936
    rows2, tier2 = synth.multires_rows(5, 32, 2116)
    assert tier2 == 2 and rows2.min() >= 7936 + 15872
    A = synth.multires_codebook(5, 32, rows)
    assert np.allclose(np.abs(A), 1 / 32) and A.shape == (256, 1024)
    with pytest.raises(ValueError):
        synth.multires_tiers(8)
