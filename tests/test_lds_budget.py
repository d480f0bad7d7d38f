"""LDS budgets of the kernels that take more than the 64 KiB default of dynamic LDS (CPU test).

Round 4 lost the K Y apply (i8ah_kernel<KY>) for every m with more than 64 KiB of digit planes: a
commit grew the kernel's static LDS from 448 to 592 B while its launcher raised the dynamic limit
to a hard-coded 160 KiB - 512 B, so hipFuncSetAttribute failed and the launch was refused
(ace_admm.cpp reported it 200 iterations later).  The launchers now derive each budget from the
code object's static LDS at run time (csrc/ace_api.cpp lds_dyn_budget), and this test pins the
other half on the CPU: it compiles the sources with the compiler's resource report and checks
that static + the dynamic LDS the launcher requests (ace_lds_request, host arithmetic in
libace.so) fits the CU's 160 KiB at every shape the reference's paths take:

* the 16-antenna driver sweep M = 121 .. 529 on the int8 path
  (main/channel_recovery_ADMM_v2_simulation_A2only.m:106-118),
* the 32-antenna r-column stages at m_t = 243 (inferLowRankV4_multi.m:258,270),
* the unit at m = 256 (fused apply_AH, gyk / gyf, the m-space run, the A2nuclear m-space kernel),
* PhaseLift's prox eigendecomposition (prox_trace.m:88-92) at the reduced order d = m = 256 for both
  reductions, and the spectral initialisation's hetrd up to order 1024.
"""
import concurrent.futures as cf
import pathlib
import re
import subprocess

import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]
CSRC = ROOT / "2ace-mmwave-channel-estimation_amd" / "csrc"
HIPCC = "/opt/rocm/bin/hipcc"
LDS_CU = 160 * 1024

# (ace_lds_request name, source, mangled-name pattern of the kernel(s) it launches, sizes that must fit)
CASES = [
    ("i8ah", "ace_i8gemm.hip", [r"i8ah_kernelILb0ELb0E"], [64, 121, 225, 243, 256, 361, 529]),
    ("i8ah_ky", "ace_i8gemm.hip", [r"i8ah_kernelILb1ELb0E"], [64, 121, 225, 243, 256, 361, 529]),
    ("i8ah_fuse", "ace_i8gemm.hip", [r"i8ah_kernelILb0ELb1E"], [64, 121, 225, 256]),
    ("gyk", "ace_i8gemm.hip", [r"10gyk_kernel"], [64, 121, 225, 256]),
    ("gyf", "ace_i8gemm.hip", [r"10gyf_kernel"], [64, 121, 225, 256]),
    ("msr", "ace_i8gemm.hip", [r"msr_kernelILi2E", r"msr_kernelILi4E"], [256]),
    ("nms", "ace_nucmsp.hip", [r"nms_kernelILb0E", r"nms_kernelILb1E"], [64, 256]),
    ("hetrd", "ace_spectral.hip", [r"12hetrd_kernel"], [256, 1024]),
    ("hetrd_blk", "ace_spectral.hip", [r"16hetrd_blk_kernelILi4E", r"16hetrd_blk_kernelILi2E"],
     [128, 243, 256]),   # (the prox order d = m, §4; the spectral order m_t = 243; panels of 4 / 2)
    # the two-stage prox eigensolver (r06): every order it takes (32 <= d <= 256)
    ("he2hb", "ace_heev2.hip", [r"12he2hb_kernel"], [32, 40, 121, 200, 256]),
    ("hb2st", "ace_heev2.hip", [r"12hb2st_kernel"], [32, 40, 121, 200, 256]),
    ("bt2", "ace_heev2.hip", [r"12bt2q2_kernel", r"12bt2q1_kernel"], [32, 40, 121, 200, 256]),
]

_REMARK = re.compile(r"remark: Function Name: (\S+)|remark:\s+LDS Size \[bytes/block\]: (\d+)")


def _static_lds(src: str) -> dict:
    """Static LDS per kernel (mangled name) from the gfx950 resource report of one source."""
    cmd = [HIPCC, "--offload-arch=gfx950", "--offload-device-only", "-O3", "-std=c++17",
           "-mllvm", "-amdgpu-mfma-vgpr-form=1", f"-I{ROOT / 'include'}", "-c", str(CSRC / src),
           "-o", "/dev/null", "-Rpass-analysis=kernel-resource-usage"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-2000:]
    res, name = {}, None
    for m in _REMARK.finditer(out.stderr):
        if m.group(1):
            name = m.group(1)
        elif name is not None:
            res[name] = int(m.group(2))
            name = None
    return res


@pytest.fixture(scope="module")
def static_lds():
    if not pathlib.Path(HIPCC).exists():
        pytest.skip("hipcc not available")
    srcs = sorted({c[1] for c in CASES})
    with cf.ThreadPoolExecutor(max_workers=len(srcs)) as ex:
        return dict(zip(srcs, ex.map(_static_lds, srcs)))


@pytest.mark.parametrize("name,src,pats,sizes", CASES, ids=[c[0] for c in CASES])
def test_static_plus_dynamic_fits_the_cu(static_lds, name, src, pats, sizes):
    from ace_amd import _lib
    kernels = static_lds[src]
    for pat in pats:
        hits = {k: v for k, v in kernels.items() if re.search(pat, k)}
        assert len(hits) == 1, f"{pat}: {sorted(hits) or 'no kernel'} in {src}"
        (kname, static), = hits.items()
        for m in sizes:
            dyn = _lib.lds_request(name, m)
            assert static + dyn <= LDS_CU, (
                f"{kname}: static {static} B + dynamic {dyn} B at m = {m} exceeds the CU's {LDS_CU} B")


def test_no_hard_coded_budgets():
    """Every dynamic-LDS limit goes through lds_dyn_budget: no launcher raises a literal limit."""
    for p in CSRC.glob("*.hip"):
        text = p.read_text()
        assert "hipFuncSetAttribute" not in text, f"{p.name} raises an LDS limit outside lds_dyn_budget"
        assert not re.search(r"160\s*\*\s*1024\s*-", text), f"{p.name} hard-codes a 160 KiB headroom"


def test_unknown_kernel_is_an_error():
    from ace_amd import _lib
    with pytest.raises(_lib.AceError):
        _lib.lds_request("nope", 256)


def test_prox_reduction_has_a_fitting_path_at_every_order(static_lds):
    """the prox's blocked reduction does not fit the CU above d of about 470; the launcher
    then takes hetrd_kernel (a choice of path, not a refusal).  At every order the PhaseLift host accepts
    up to the reference's 32-antenna sweep (d = 841, 1024) one of the two must fit."""
    from ace_amd import _lib
    kernels = static_lds["ace_spectral.hip"]
    st_blk = max(v for k, v in kernels.items() if re.search(r"16hetrd_blk_kernelILi4E", k))
    st_unb = max(v for k, v in kernels.items() if re.search(r"12hetrd_kernel", k))
    for d in (243, 256, 470, 512, 560, 841, 1024):
        blk_fits = st_blk + _lib.lds_request("hetrd_blk", d) <= LDS_CU
        unb_fits = st_unb + _lib.lds_request("hetrd", d) <= LDS_CU
        assert blk_fits or unb_fits, d
    assert st_blk + _lib.lds_request("hetrd_blk", 512) > LDS_CU   # (so the fallback is what d = 512 exercises)
