"""Input format (frame pair + flow target) — TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Restates src/models/input.py in float32 numpy:
* ``Input.__getitem__`` clip and range map (input.py:215-221),
* ``ModuloPadding.apply`` extents, alignment and numpy pad modes (input.py:79-138; the torch.* modes
  replicate / reflect / circular equal numpy edge / reflect / wrap for the pads used here),
* ``TorchAdapter.__getitem__`` NCHW permute, ``nan_to_num`` and clip of the flow (input.py:280-313).
"""

import numpy as np

_NP_MODE = {"edge": "edge", "torch.replicate": "edge", "reflect": "reflect", "torch.reflect": "reflect",
            "symmetric": "symmetric", "wrap": "wrap", "torch.circular": "wrap"}


def pad_extents(h, w, size, align_hz="left", align_vt="top"):
    """input.py:93-118 -> (ph1, ph2), (pw1, pw2)."""
    new_h = (h + size[1] - 1) // size[1] * size[1]
    new_w = (w + size[0] - 1) // size[0] * size[0]
    ph, pw = new_h - h, new_w - w
    ph1 = {"top": 0, "bottom": ph, "center": ph // 2}[align_vt]
    pw1 = {"left": 0, "right": pw, "center": pw // 2}[align_hz]
    return (ph1, ph - ph1), (pw1, pw - pw1)


def input_images(img, clip=(0.0, 1.0), rng=(-1.0, 1.0), mode="zeros", size=None, align_hz="left", align_vt="top"):
    """(B,H,W,C) float32 -> (B,C,H',W') float32, input.py:220-221 then :120-127 then :280."""
    img = np.asarray(img, dtype=np.float32)
    x = (rng[1] - rng[0]) * np.clip(img, clip[0], clip[1]) + rng[0]        # float32 (weak python scalars)
    if size is not None:
        (ph1, ph2), (pw1, pw2) = pad_extents(img.shape[1], img.shape[2], size, align_hz, align_vt)
        pad = ((0, 0), (ph1, ph2), (pw1, pw2), (0, 0))
        if mode in ("zeros", "ones"):
            x = np.pad(x, pad, mode="constant", constant_values=0.0 if mode == "zeros" else 1.0)
        else:
            x = np.pad(x, pad, mode=_NP_MODE[mode])
    return np.ascontiguousarray(x.transpose(0, 3, 1, 2)).astype(np.float32)


def input_flow(flow, valid, size=None, align_hz="left", align_vt="top", flow_inf=1e10):
    """(B,H,W,2), (B,H,W) -> (B,2,H',W') float32, (B,H',W') bool: input.py:120-122 and :305-313."""
    flow = np.asarray(flow, dtype=np.float32)
    valid = np.asarray(valid, dtype=bool)
    if size is not None:
        (ph1, ph2), (pw1, pw2) = pad_extents(flow.shape[1], flow.shape[2], size, align_hz, align_vt)
        flow = np.pad(flow, ((0, 0), (ph1, ph2), (pw1, pw2), (0, 0)), mode="constant", constant_values=0)
        valid = np.pad(valid, ((0, 0), (ph1, ph2), (pw1, pw2)), mode="constant", constant_values=False)
    flow = np.nan_to_num(flow, nan=0.0, posinf=flow_inf, neginf=-flow_inf)
    flow = np.clip(flow, -flow_inf, flow_inf)
    return np.ascontiguousarray(flow.transpose(0, 3, 1, 2)).astype(np.float32), valid
