"""The host-ASan/UBSan build of the C-ABI library (`make -C csrc sanitize`: host side of every
translation unit instrumented, device code not) driving small solves through every *_host
wrapper, the driver (A2only, PhaseLift) and the beamformer on the GPU
(`tests/native/capi_sanitize.cpp gpu`).  Leak detection is off: the HIP runtime keeps its
allocations to process exit."""
import os
import pathlib
import subprocess

import pytest

pytestmark = pytest.mark.gpu

EXE = pathlib.Path(__file__).resolve().parent / "native" / "ace_capi_sanitize"


def test_capi_gpu_asan_ubsan():
    if not EXE.exists():   # a test tool, built by __graft_entry__.build() when the sanitizer runtime links
        pytest.skip("no sanitizer build (make -C 2ace-mmwave-channel-estimation_amd/csrc sanitize)")
    env = dict(os.environ)
    env["ASAN_OPTIONS"] = "detect_leaks=0:halt_on_error=1"
    env["UBSAN_OPTIONS"] = "halt_on_error=1:print_stacktrace=1"
    p = subprocess.run([str(EXE), "gpu"], capture_output=True, text=True, timeout=240, env=env)
    assert p.returncode == 0 and p.stdout.strip().endswith("OK"), (p.returncode, p.stdout[-2000:], p.stderr[-4000:])
    assert "runtime error" not in p.stderr, p.stderr[-4000:]
