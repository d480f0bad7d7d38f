"""Count exact / sign-equivalent / other beam-code agreement of the GPU beamformer vs the
oracle (numpy zgesdd, the reference's dependency) on large random sweeps."""
import json, sys, numpy as np
sys.path.insert(0, "2ace-mmwave-channel-estimation_amd"); sys.path.insert(0, "oracle")
import beamformer_oracle as BO
from ace_amd import svd_beamformer_host
out = {}
for name, n, count, kind in (("gauss16", 16, 20000, "g"), ("rank1noise16", 16, 10000, "r"), ("gauss8", 8, 10000, "g"),
                             ("gauss32", 32, 2000, "g")):
    rng = np.random.default_rng(77 + n)
    H = rng.standard_normal((count, n, n)) + 1j * rng.standard_normal((count, n, n))
    if kind == "r":
        u = rng.standard_normal((count, n, 1)) + 1j * rng.standard_normal((count, n, 1))
        v = rng.standard_normal((count, 1, n)) + 1j * rng.standard_normal((count, 1, n))
        H = u @ v + 1e-2 * H
    res = svd_beamformer_host(H)
    exact = sign = other = idx_bad = 0
    for k in range(count):
        a, b, ti, ri, _ = BO.svd_beamformer(H[k])
        idx_bad += int(not (res.beam_idx[k] == (ti, ri)).all())
        if (res.wr_code[k] == a).all() and (res.wt_code[k] == b).all():
            exact += 1
            continue
        ok = True
        for g, e in ((res.wr_code[k], a), (res.wt_code[k], b)):
            d = (g.astype(int) - e.astype(int)) % 4
            ok &= bool(np.all(d == d[0]) and d[0] in (0, 2))
        sign += ok
        other += not ok
    out[name] = dict(count=count, exact=exact, sign_only=sign, other=other, beam_idx_mismatch=idx_bad)
    print(name, out[name], flush=True)
json.dump(out, open("gpurun_out/r18/bf_parity_count.json", "w"), indent=1)
