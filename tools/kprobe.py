"""Diagnostic: per-kernel-class device time of one batch solve (event timing)."""
import ctypes as C, sys, os, json, pathlib
ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "2ace-mmwave-channel-estimation_amd"))
import torch
import ace_amd
from ace_amd._lib import LIB, KERNEL_CLASSES, check

def run(batch=4096, m=256, tx=32, iters=200, variant="A2only", private=False, **kw):
    A, B, X0, H = ace_amd.synth_problem(58659179, 0, batch, m, tx, tx, a_shared=not private)
    ws = ace_amd.solver.Workspace()
    out = ace_amd.infer_admm_batch(A, B, X0, tx, tx, variant=variant, maxiter=iters, fixed_iters=True, workspace=ws, **kw)
    torch.cuda.synchronize()
    check(LIB.ace_prof_start(iters * 8 + 32))
    out = ace_amd.infer_admm_batch(A, B, X0, tx, tx, variant=variant, maxiter=iters, fixed_iters=True, workspace=ws, out=out, **kw)
    kt = (C.c_double * 10)(); kn = (C.c_int32 * 10)()
    check(LIB.ace_prof_stop(kt, kn))
    res = {KERNEL_CLASSES[i]: round(kt[i] / kn[i], 4) for i in range(10) if kn[i]}
    res["total_ms"] = round(sum(kt), 2)
    return res

if __name__ == "__main__":
    cfgs = json.loads(sys.argv[1]) if len(sys.argv) > 1 else [{}]
    for c in cfgs:
        print(json.dumps(c), json.dumps(run(**c)), flush=True)
