"""The roofline accounting of bench.py: algorithmic bytes / ops per realisation and
iteration of the unit path, and the bench contract's metric name.  Host-only."""
import importlib.util
import pathlib

ROOT = pathlib.Path(__file__).resolve().parent.parent


def _bench():
    spec = importlib.util.spec_from_file_location("bench_under_test", ROOT / "bench.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_unit_bytes_match_design():
    b = _bench()
    m, n, tx = 256, 1024, 32
    ub = b.unit_bytes(m, n, tx, tx)
    # Z-step steady state: certificate and control from RealState only (the data pass is fused
    # into apply_AH)
    assert ub["zstep"] == 0
    # gyk: read Y, M, AX, B (f64); write g, AX, M, Y_new (no K Y / dual terms: lazy dual residual)
    assert ub["apply_G"] == 16 * 7 * m + 8 * m == 30 * 1024
    # fused apply_AH: read g and Z, write Z' (W stays on chip)
    assert ub["apply_AH"] == 16 * (m + 2 * n)


def test_gyf_bytes():
    b = _bench()
    m, n = 256, 1024
    # gyk + fused apply_AH in one launch: read Y, M, AX, B, Z; write AX, M, Y, Z' (g stays on chip)
    assert b.gyf_bytes(m, n) == 16 * 6 * m + 8 * m + 32 * n == 58 * 1024


def test_msp_bytes():
    b = _bench()
    # m-space form: read Y, M, AX, S, B; write AX, M, Y, S' (no Z, no apply_AH pass)
    assert b.msp_bytes(256) == 16 * 8 * 256 + 8 * 256 == 34 * 1024


def test_int8_ops_and_flops():
    b = _bench()
    io = b.unit_i8_ops(256, 1024)
    assert io["apply_AH"] == 2 * 8 * 2048 * 512 == io["apply_A"]
    assert io["apply_G"] == 0                           # no K Y in the steady state (lazy dual residual)
    uf = b.unit_flops(256, 1024, 32, 32)
    assert uf["apply_G"] == 8 * 256 * 256              # g = G T, 8 flops per complex MAC


def test_private_bytes_and_ops():
    b = _bench()
    m, n = 256, 1024
    # G_b lower triangle (c128) + A^H codes (2 bits) + Y, M, AX (c128) and B (f64) in, AX, M, Y out + W out
    assert b.private_bytes(m, n) == 16 * m * (m + 1) // 2 + m * n // 4 + 16 * 6 * m + 8 * m + 16 * n
    po = b.private_ops(m, n)
    assert po["int8"] == 2 * 3 * 8 * (2 * n) * (2 * m)   # three digit-plane right-hand sides (g, Y, Y - Y0)
    assert po["f64"] == 8 * m * m


def test_metric_is_baselines():
    import json
    b = _bench()
    base = json.loads((ROOT / "BASELINE.json").read_text())
    assert b.METRIC == base["metric"]
