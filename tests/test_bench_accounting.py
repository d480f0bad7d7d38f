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


def test_nuclear_bytes():
    b = _bench()
    m, n = 256, 1024
    nb = b.nuclear_bytes(m, n)
    # gyk: Y, M, AX, B in, g, AX, M, Y out, plus Z and N for the digit planes of V = Z - N/mu
    assert nb["apply_G"] == 16 * 7 * m + 8 * m + 32 * n
    assert nb["apply_AH"] == 16 * (m + n)          # g in, W out
    assert nb["zstep"] == 16 * 5 * n               # W, Z, N in; Z', N' out
    r = b.unit_resources("apply_G", m, n, variant="A2nuclear", pc=False, gyf=False, gyk=True, i8=True, msp_frac=0.0)
    assert r == {"f64": 8 * m * m, "int8": 2 * 8 * 2 * m * 2 * n, "hbm": nb["apply_G"]}


def test_roofline_picks_bound_and_serial_frac():
    b = _bench()
    r = b.roofline_from("k", 1e-4, {"f64": 78.6e12 * 2e-5, "hbm": 8e12 * 5e-5})
    assert r["resource"] == "hbm" and abs(r["frac"] - 0.5) < 1e-9
    assert abs(r["serial_frac"] - 0.7) < 1e-9 and r["other_resources"]["f64"]["frac"] == 0.2


def test_pmc_traffic_is_keyed_by_workload(tmp_path, monkeypatch):
    import json
    b = _bench()
    prof = tmp_path / "profiles"
    prof.mkdir()
    meta = {"_meta": {"batch": 4096}}
    (prof / "r02_v9_pmc_hbm.json").write_text(json.dumps({"gyk_kernel": {"hbm_bytes": 1.0}, **meta}))
    (prof / "r03_v1_nuclear_pmc_hbm.json").write_text(json.dumps({"gyk_kernel": {"hbm_bytes": 2.0}, **meta}))
    (prof / "r03_v2_config5_pmc_hbm.json").write_text(json.dumps({"gyk_kernel": {"hbm_bytes": 3.0}, **meta}))
    monkeypatch.setattr(b, "ROOT", tmp_path)
    assert b._pmc_traffic("gyk_kernel", "unit") == (1, "profiles/r02_v9_pmc_hbm.json")
    assert b._pmc_traffic("gyk_kernel", "nuclear") == (2, "profiles/r03_v1_nuclear_pmc_hbm.json")
    assert b._pmc_traffic("gyk_kernel", "config5") == (3, "profiles/r03_v2_config5_pmc_hbm.json")
    assert b._pmc_traffic("gyk_kernel", "private") is None


def test_pmc_traffic_rescaled_to_the_lines_batch(tmp_path, monkeypatch):
    """A PMC profile of another batch size is rescaled per realisation (config 5's
    traffic was divided by four times the realisations the profile's launches carried); a profile
    without its batch recorded is not used."""
    import json
    b = _bench()
    prof = tmp_path / "profiles"
    prof.mkdir()
    (prof / "r04_v1_config5_pmc_hbm.json").write_text(json.dumps({"nms_kernel<false>": {"hbm_bytes": 800.0},
                                                                   "_meta": {"batch": 16384}}))
    (prof / "r04_v2_pipeline_pmc_hbm.json").write_text(json.dumps({"zstep_kernel<0>": {"hbm_bytes": 8.0}}))
    monkeypatch.setattr(b, "ROOT", tmp_path)
    v, src = b._pmc_traffic("nms_kernel", "config5", 65536)
    assert v == 3200 and "batch 16384" in src
    assert b._pmc_traffic("zstep_kernel", "pipeline", 4096) is None


def test_nms_bytes():
    b = _bench()
    m = 256
    # read Y, M, e, A E (c128) and B (f64); write Y, M, e, A E
    assert b.nms_bytes(m) == 16 * 8 * m + 8 * m
    r = b.unit_resources("apply_G", m, 1024, variant="A2nuclear", pc=False, gyf=False, gyk=True, i8=True,
                         msp_frac=0.0, nms=True)
    assert r == {"f64": 8 * m * m, "hbm": b.nms_bytes(m)}
    assert b.unit_resources("zstep", m, 1024, variant="A2nuclear", pc=False, gyf=False, gyk=True, i8=True,
                            msp_frac=0.0, nms=True) == {}


def test_work_roofline_attaches_class_kernel_traffic(tmp_path, monkeypatch):
    import json
    b = _bench()
    prof = tmp_path / "profiles"
    prof.mkdir()
    (prof / "r03_v9_phaselift_pmc_hbm.json").write_text(json.dumps({"he2hb_kernel": {"hbm_bytes": 5.0},
                                                                     "_meta": {"batch": 512}}))
    monkeypatch.setattr(b, "ROOT", tmp_path)
    kt = [0.0] * 10
    kn = [0] * 10
    kw, kb, ko = [0.0] * 10, [0.0] * 10, [0.0] * 10
    kt[8], kn[8], kw[8] = 100.0, 10, 1e12        # zstep class: the prox eig
    r, shares = b.work_roofline(kt, kn, kw, kb, ko, "note", tag="phaselift", batch=512)
    assert r["kernel"] == "zstep" and r["traffic"] == 5 and r["traffic_kernel"] == "he2hb_kernel"
    r, _ = b.work_roofline(kt, kn, kw, kb, ko, "note", tag="pipeline", batch=512)
    assert r["traffic"] is None


def test_work_roofline_dominant_by_device_time():
    """The dominant class is the one with the most device time whatever work it carries (VERDICT r03:
    the pipeline's r-column Z-step, 37 % of its device time, had no flop count and was never
    picked); its bound is the resource with the largest time at peak among flops, bytes, int8 ops."""
    b = _bench()
    kt, kn = [0.0] * 10, [0] * 10
    kw, kb, ko = [0.0] * 10, [0.0] * 10, [0.0] * 10
    kt[4], kn[4], kw[4] = 10.0, 10, 1e12            # apply_G: f64 GEMM, little device time
    kt[8], kn[8], kw[8], kb[8] = 37.0, 10, 1e11, 8e10   # zstep: HBM-bound by time at peak
    kt[3], kn[3], kb[3], ko[3] = 20.0, 10, 1e10, 5e13   # apply_A: int8 ops
    r, shares = b.work_roofline(kt, kn, kw, kb, ko, "note")
    assert r["kernel"] == "zstep" and r["resource"] == "hbm" and r["bound"] == "hbm"
    assert abs(r["frac"] - 8e9 / 3.7e-3 / 8e12) < 1e-4 and "f64" in r["other_resources"]
    assert shares["zstep"] == round(37 / 67, 4)
    kt[8], kb[8], kw[8] = 37.0, 0.0, 0.0            # no work count: reported, marked latency
    r, _ = b.work_roofline(kt, kn, kw, kb, ko, "note")
    assert r["kernel"] == "zstep" and r["bound"] == "latency"
