#!/usr/bin/env python3
"""Generate tests/golden/beamformer_ref.npz from the reference's own Python.

The downstream beamformer is plain numpy in the reference
(main/codebook_library.py:57-138), so its golden vectors come from importing that module
and calling ``svd_beamformer`` / ``svd_beamformer_compensation`` on seeded inputs.  Only
inputs and the returned code strings (as 0..3 integer arrays) are stored; nothing of the
reference's source travels.  Run in the build container (the GPU box has no
/root/reference):

    python tests/golden/make_beam_golden.py
"""
import pathlib
import sys

import numpy as np

HERE = pathlib.Path(__file__).resolve().parent
REF_MAIN = pathlib.Path("/root/reference/main")
CALIB = np.array([0, 2, 3, 0, 0, 3, 0, 3, 1, 0, 0, 3, 0, 3, 0, 0])   # main.py:367 calibration_bit


def cn(rng, *shape):
    return rng.standard_normal(shape) + 1j * rng.standard_normal(shape)


def cases(rng):
    """(name, H [k][n][n], offset [k][n] or None)."""
    out = []
    out.append(("generic16", cn(rng, 32, 16, 16), None))
    u, v = cn(rng, 32, 16, 1), cn(rng, 32, 1, 16)
    out.append(("rank1noise16", u @ v + 1e-3 * cn(rng, 32, 16, 16), None))
    u, v = cn(rng, 16, 16, 1), cn(rng, 16, 1, 16)
    out.append(("rank1_16", 1e-3 * (u @ v), None))             # the r = 1 pipeline output shape
    out.append(("comp16", cn(rng, 16, 16, 16), np.tile(CALIB * (np.pi / 2), (16, 1))))
    u, v = cn(rng, 16, 16, 1), cn(rng, 16, 1, 16)
    out.append(("comp_rank1noise16", u @ v + 1e-2 * cn(rng, 16, 16, 16),
                np.tile(CALIB * (np.pi / 2), (16, 1))))
    for n in (1, 2, 3, 4, 8, 12):
        out.append((f"small{n}", cn(rng, 8, n, n), None))
    out.append(("real16", rng.standard_normal((8, 16, 16)) + 0j, None))
    out.append(("zero16", np.zeros((1, 16, 16), np.complex128), None))
    out.append(("generic32", cn(rng, 6, 32, 32), None))          # zgesdd divide-and-conquer regime
    return out


def main():
    sys.path.insert(0, str(REF_MAIN))
    import codebook_library as ref  # the reference module (numpy/scipy only)

    rng = np.random.default_rng(20231102)
    blob = {}
    for name, H, off in cases(rng):
        wr, wt = [], []
        for k in range(len(H)):
            if off is None:
                a, b = ref.svd_beamformer(H[k])
            else:
                a, b = ref.svd_beamformer_compensation(H[k], off[k])
            wr.append([int(c) for c in a])
            wt.append([int(c) for c in b])
        blob[f"{name}__H"] = H
        if off is not None:
            blob[f"{name}__offset"] = off
        blob[f"{name}__wr"] = np.array(wr, np.uint8)
        blob[f"{name}__wt"] = np.array(wt, np.uint8)
    blob["names"] = np.array([c[0] for c in cases(np.random.default_rng(0))])
    np.savez_compressed(HERE / "beamformer_ref.npz", **blob)
    print("wrote", HERE / "beamformer_ref.npz", len(blob["names"]), "groups")


if __name__ == "__main__":
    main()
