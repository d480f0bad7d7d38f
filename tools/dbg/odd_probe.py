"""Probe: A2only Y/X parity against the C oracle at tiny geometries (odd tx via padding, even tx direct)."""
import sys
import numpy as np
sys.path[:0] = ["oracle", "tests", "2ace-mmwave-channel-estimation_amd"]
import ace_oracle as O
import ace_oracle_c as OC
from ace_amd import infer_admm_host, synth

for tx, rx, m, sh in [(1, 8, 32, False), (2, 8, 32, False), (2, 4, 32, False), (3, 3, 32, False), (2, 4, 64, True),
                      (2, 8, 64, True), (1, 8, 64, True)]:
    A, B, X0, _ = synth.problem(31 + tx, 0, 4, m, tx, rx, a_shared=sh)
    U = np.stack([OC.make_U(a) for a in A])
    try:
        res = infer_admm_host(A, B, X0, tx, rx, variant="A2only")
    except Exception as e:
        print(tx, rx, m, sh, "error", e, flush=True)
        continue
    Xo, Yo, ito, cvo, _ = OC.infer_admm_r1_batch(A, U, B, X0, tx, rx, variant=0)
    ex = [O.unit_phase_aligned_rel_err(res.X[b], Xo[b]) for b in range(4)]
    ey = [O.unit_phase_aligned_rel_err(res.Y[b], Yo[b]) for b in range(4)]
    print(tx, rx, m, sh, "iters", res.iters.tolist(), ito.tolist(), "ex %.1e ey %.1e" % (max(ex), max(ey)), flush=True)
