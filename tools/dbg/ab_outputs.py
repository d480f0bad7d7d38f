"""A/B bit-identity of solver outputs between two builds of libace.so (ACE_LIB): run in two
processes, `ab_outputs.py save <out.npz>` with each library, then `ab_outputs.py cmp a.npz b.npz`.
Diagnostic only."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "2ace-mmwave-channel-estimation_amd"))

if sys.argv[1] == "save":
    import torch
    from ace_amd import infer_admm_batch, synth_problem
    out = {}
    for name, (batch, m, tx, fixed, it) in {"u32": (1024, 256, 32, True, 60), "u32c": (512, 256, 32, False, 200),
                                             "u16": (256, 64, 16, True, 60), "u16c": (256, 121, 16, False, 300)}.items():
        A, B, X0, _ = synth_problem(91, 0, batch, m, tx, tx)
        r = infer_admm_batch(A, B, X0, tx, tx, maxiter=it, fixed_iters=fixed)
        torch.cuda.synchronize()
        out[name + "_X"] = r.X.cpu().numpy()
        out[name + "_Y"] = r.Y.cpu().numpy()
        out[name + "_it"] = r.iters.cpu().numpy()
    np.savez(sys.argv[2], **out)
else:
    a, b = np.load(sys.argv[2]), np.load(sys.argv[3])
    for k in a.files:
        d = np.abs(a[k] - b[k]).max() if a[k].dtype != np.int32 else int((a[k] != b[k]).sum())
        print(f"{k}: {'identical' if np.array_equal(a[k], b[k]) else 'DIFFERS'} (max diff {d})")
