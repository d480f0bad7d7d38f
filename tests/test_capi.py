"""CPU tests of the C-ABI library: it loads, exports every symbol include/ace.h
declares, and its argument validation (which runs before any HIP call) behaves.
No compute calls -- there is no GPU here."""
import ctypes as C
import pathlib
import re

import numpy as np
import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]


def _declared_functions():
    text = (ROOT / "include" / "ace.h").read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(ace_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    from ace_amd._lib import LIB_PATH
    lib = C.CDLL(str(LIB_PATH))
    names = _declared_functions()
    assert "ace_admm_solve_batch" in names and len(names) >= 10
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing


def test_library_is_gfx950():
    from ace_amd._lib import LIB_PATH
    blob = LIB_PATH.read_bytes()
    assert b"gfx950" in blob


def test_cfg_defaults_match_reference():
    """inferLowRankV4_multi.m:6-14 defaults."""
    import ace_amd
    c = ace_amd.default_cfg()
    assert (c.maxiter, c.mu0, c.rho, c.tol_rel, c.tol_abs) == (500, 1e-3, 1.03, 1e-4, 1e-8)
    assert c.variant == ace_amd.ACE_VARIANT_A2ONLY and c.scale_by_row == 1 and c.a_shared == 1
    assert c.r == 1 and not c.rank_one     # the refinement stage, one flag for the batch
    with pytest.raises(TypeError):
        ace_amd.default_cfg(no_such_field=1)


def test_workspace_size():
    import ace_amd
    lib = ace_amd.LIB
    c = ace_amd.default_cfg()
    w = lib.ace_admm_workspace_size(C.byref(c), 4096, 256, 1024)
    # 6 n-vectors (X Z N V optX Q) + 9 m-vectors + K, G, A^H, per-realisation state
    assert 4096 * (6 * 1024 + 9 * 256) * 16 < w < 2 * 4096 * (6 * 1024 + 9 * 256) * 16
    assert lib.ace_admm_workspace_size(C.byref(c), 0, 256, 1024) == 0
    c20 = ace_amd.default_cfg(r=20)          # the r-column stages carry r columns of state
    assert lib.ace_admm_workspace_size(C.byref(c20), 64, 256, 1024) > 64 * 20 * 6 * 1024 * 16
    cp = ace_amd.default_cfg(a_shared=0)
    assert lib.ace_admm_workspace_size(C.byref(cp), 8, 256, 1024) > 8 * 2 * 256 * 256 * 16


@pytest.mark.parametrize("kw,tx,rx,msg", [
    ({}, 4, 5, "tx*rx"),
    ({}, 33, 1, "tx in [1,32]"),   # (odd tx <= 31 is padded to tx + 1 rows; 33 would need 34)
    ({"variant": 7}, 4, 4, "unknown variant"),
    ({"maxiter": 0}, 4, 4, "maxiter"),
    ({"mu0": 0.0}, 4, 4, "mu0"),
    ({"r": 33}, 4, 4, "r must be in"),
    ({"r": 2, "a_shared": 0}, 4, 4, "shared A"),
])
def test_validation_errors(kw, tx, rx, msg):
    """Validation runs before any HIP call; NULL buffers make a missed check fail safely."""
    import ace_amd
    c = ace_amd.default_cfg(**kw)
    n = 16 if msg == "tx*rx" else tx * rx
    rc = ace_amd.LIB.ace_admm_solve_batch(C.byref(c), 1, 4, n, tx, rx, None, None, None, None, None, None, None,
                                          None, None, 0, None)
    assert rc in (ace_amd._lib.ACE_ERR_ARG, ace_amd._lib.ACE_ERR_UNSUPPORTED)
    assert msg in ace_amd.LIB.ace_last_error().decode()


def test_null_buffers_rejected():
    import ace_amd
    c = ace_amd.default_cfg()
    rc = ace_amd.LIB.ace_admm_solve_batch(C.byref(c), 1, 4, 16, 4, 4, None, None, None, None, None, None, None,
                                          None, None, 0, None)
    assert rc == ace_amd._lib.ACE_ERR_ARG
    assert b"NULL" in ace_amd.LIB.ace_last_error()


def test_host_api_shape_checks():
    import ace_amd
    with pytest.raises(ValueError):
        ace_amd.infer_admm_host(np.zeros((2, 4, 16), complex), np.ones((3, 4)), np.ones((3, 16), complex), 4, 4)
    with pytest.raises(NotImplementedError):   # r <= 32 columns (the reference's stages use r = 20)
        ace_amd.InferADMM(np.zeros((4, 16), complex), np.ones(4), np.ones((16, 33), complex), True, False, 4, 4)
    with pytest.raises(ValueError):            # one use_rank_one flag per realisation
        ace_amd.infer_admm_host(np.zeros((1, 4, 16), complex), np.ones((3, 4)), np.ones((3, 16), complex), 4, 4,
                                use_rank_one=np.ones(2, bool))
    with pytest.raises(NotImplementedError):
        ace_amd.InferADMM(np.zeros((4, 16), complex), np.ones(4), np.ones(16, complex), True, False, 4, 4,
                          lambda_=0.1)
