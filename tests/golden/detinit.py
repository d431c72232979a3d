"""Deterministic, name-keyed parameter initialisation shared by the fixture generator and tests.

Test infrastructure only.  Every floating-point entry of a module's state_dict is filled from
``numpy.random.default_rng(crc32(key))`` so that a reference module (in the build container)
and the drop-in module under test (anywhere) hold bit-identical weights without committing them.
"""

import zlib

import numpy as np


def det_init(module, scale=0.1):
    import torch
    with torch.no_grad():
        for key, val in module.state_dict().items():
            if not torch.is_floating_point(val):
                continue
            rng = np.random.default_rng(zlib.crc32(key.encode()))
            a = rng.standard_normal(tuple(val.shape)).astype(np.float32)
            if key.endswith("running_var"):
                a = 1.0 + 0.5 * np.abs(a)
            elif key.endswith(".weight") and val.dim() == 1:        # norm affine scale
                a = 1.0 + scale * a
            else:
                a = scale * a
            val.copy_(torch.from_numpy(a))
    return module


def det_init_fanin(module, head_gain=0.1):
    """Name-keyed, seeded like det_init, but He-scaled (std sqrt(2 / fan_in)) so a deep network
    (the end-to-end RAFT fixture) keeps O(1) activations; flow-producing output convs
    (`*flow.conv2.weight`) get `head_gain` so 12 GRU updates stay within a few pixels."""
    import torch
    with torch.no_grad():
        for key, val in module.state_dict().items():
            if not torch.is_floating_point(val):
                continue
            rng = np.random.default_rng(zlib.crc32(key.encode()))
            a = rng.standard_normal(tuple(val.shape)).astype(np.float64)
            if key.endswith("running_var"):
                a = 1.0 + 0.5 * np.abs(a)
            elif key.endswith("running_mean"):
                a = 0.1 * a
            elif key.endswith(".weight") and val.dim() == 1:
                a = 1.0 + 0.1 * a
            elif key.endswith(".weight"):
                a = a * np.sqrt(2.0 / float(np.prod(val.shape[1:])))
                if key.endswith("flow.conv2.weight"):
                    a = a * head_gain
            else:
                a = 0.01 * a
            val.copy_(torch.from_numpy(a.astype(np.float32)))
    return module
