#!/usr/bin/env python3
"""Golden vectors for the input format, produced by RUNNING the reference's own classes.

Test infrastructure only; same import recipe as gen_golden.py.  Exercised (reference file:line):
  * ModuloPadding.apply (every numpy / torch pad mode, all alignments)   src/models/input.py:79-138
  * Input.__getitem__ clip + range map                                     src/models/input.py:208-226
  * TorchAdapter.__getitem__ NCHW permute, flow nan_to_num / clip           src/models/input.py:245-313
Usage:  python tests/golden/gen_golden_input.py        (writes tests/golden/input_*.npz)
"""

import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gen_golden import OUT, _import_reference  # noqa: E402

CASES = [  # (name, mode, size [w_mod, h_mod], align_hz, align_vt, clip, range)
    ("zeros_lt", "zeros", (8, 8), "left", "top", (0.0, 1.0), (-1.0, 1.0)),
    ("zeros_cc64", "zeros", (64, 64), "center", "center", (0.0, 1.0), (-1.0, 1.0)),
    ("ones_rb", "ones", (16, 8), "right", "bottom", (0.1, 0.9), (0.0, 255.0)),
    ("edge_cc", "edge", (16, 16), "center", "center", (0.0, 1.0), (-1.0, 1.0)),
    ("reflect_lt", "reflect", (8, 16), "left", "top", (0.0, 1.0), (-1.0, 1.0)),
    ("symmetric_rb", "symmetric", (16, 16), "right", "bottom", (0.0, 1.0), (-1.0, 1.0)),
    ("wrap_cc", "wrap", (32, 32), "center", "center", (0.0, 1.0), (-1.0, 1.0)),
    ("trep_lt", "torch.replicate", (8, 8), "left", "top", (0.0, 1.0), (-1.0, 1.0)),
    ("trefl_cc", "torch.reflect", (16, 8), "center", "center", (0.0, 1.0), (-1.0, 1.0)),
    ("tcirc_rb", "torch.circular", (8, 16), "right", "bottom", (0.0, 1.0), (-1.0, 1.0)),
]


def main():
    _import_reference()
    from src.models import input as ref_input
    rng = np.random.default_rng(97531)
    b, h, w = 2, 13, 21
    for name, mode, size, ahz, avt, clip, rg in CASES:
        img1 = rng.uniform(-0.2, 1.2, (b, h, w, 3)).astype(np.float32)     # outside [0, 1]: exercises the clip
        img2 = rng.uniform(-0.2, 1.2, (b, h, w, 3)).astype(np.float32)
        flow = (5.0 * rng.standard_normal((b, h, w, 2))).astype(np.float32)
        flow[0, 0, 0] = (np.nan, np.inf)
        flow[1, 2, 3] = (-np.inf, 3e10)
        valid = rng.uniform(size=(b, h, w)) > 0.2
        valid[0, 0, 0] = True
        meta = [type("M", (), {"original_extents": ((0, h), (0, w))})() for _ in range(b)]
        pad = ref_input.ModuloPadding(mode, list(size), align_hz=ahz, align_vt=avt)
        src = [(img1, img2, flow, valid, meta)]
        inp = ref_input.Input(src, clip, rg, pad)
        adapter = ref_input.TorchAdapter(inp, flow=True, validate=False)
        o1, o2, of, ov, om = adapter[0]
        path = os.path.join(OUT, f"input_{name}.npz")
        np.savez_compressed(path, img1=img1, img2=img2, flow=flow, valid=valid, mode=mode, size=np.asarray(size),
                            align_hz=ahz, align_vt=avt, clip=np.asarray(clip, np.float64),
                            range=np.asarray(rg, np.float64), out1=o1.numpy(), out2=o2.numpy(), out_flow=of.numpy(),
                            out_valid=ov.numpy(), extents=np.asarray(om[0].original_extents))
        print(f"input_{name}.npz  {os.path.getsize(path) / 1e3:.1f} kB  out {tuple(o1.shape)}")


if __name__ == "__main__":
    main()
