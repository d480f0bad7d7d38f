"""Probe: the order that raised the Newton-Schulz failure once (r06), then the same case repeated."""
import sys
import numpy as np
sys.path[:0] = ["oracle", "tests", "2ace-mmwave-channel-estimation_amd"]
from ace_amd import infer_admm_host, synth

cases = [(1, 8, 32), (2, 8, 32), (2, 4, 32), (1, 8, 64), (1, 8, 64), (2, 4, 64), (1, 8, 64)]
for tx, rx, m in cases:
    A, B, X0, _ = synth.problem(31 + tx, 0, 4, m, tx, rx, a_shared=True)
    try:
        res = infer_admm_host(A, B, X0, tx, rx, variant="A2only")
        print(tx, rx, m, "ok", res.iters.tolist(), flush=True)
    except Exception as e:
        print(tx, rx, m, "error", e, flush=True)
