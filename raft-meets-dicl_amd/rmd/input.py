"""Drop-in for the input format of src/models/input.py on the GPU.

The reference prepares every batch on the host (numpy clip + range map, np.pad / F.pad modulo
padding, then a permute to NCHW in TorchAdapter) and copies it to the GPU.  Here the raw frames go
to HBM once and one rmd_input_images launch per image produces the padded (B, C, H', W') network
input; rmd_input_flow pads the flow target and its validity mask the same way.

  ModuloPadding   <- input.py:32-138 (same config keys, validation and error messages)
  InputSpec       <- input.py:153-190; InputSpec.prepare() = Input.__getitem__ (input.py:208-226)
                     followed by TorchAdapter.__getitem__ (input.py:245-313) on the GPU

prepare(device='cpu') runs the reference's own host path (numpy clip / range map / np.pad, NCHW
permute) and returns CPU tensors, so the module works on either device as the reference's does.

Differences: on the GPU the statistic pad modes (maximum, mean, median, minimum) raise
NotImplementedError (no config uses them; every cfg pads with zeros; the host path supports them);
the non-finite-input warnings of TorchAdapter (which only mark metadata) are left to the caller.
"""

import numpy as np
import torch

from . import _lib
from .ops import _ptr, _stream

FLOW_INF = 1e10            # TorchAdapter.flow_inf (input.py:241-243)

_MODES = {"zeros": 0, "ones": 1, "edge": 2, "torch.replicate": 2, "reflect": 3, "torch.reflect": 3,
          "symmetric": 4, "wrap": 5, "torch.circular": 5}
_STAT_MODES = ("maximum", "mean", "median", "minimum")


class ModuloPadding:
    """input.py:32-138: pad (H, W) up to multiples of size = [w_mod, h_mod]."""
    type = "modulo"

    @classmethod
    def _typecheck(cls, cfg):
        if cfg["type"] != cls.type:
            raise ValueError(f"invalid padding type '{cfg['type']}', expected '{cls.type}'")

    @classmethod
    def from_config(cls, cfg):
        cls._typecheck(cfg)
        size = [int(x) for x in list(cfg["size"])]
        if len(size) != 2:
            raise ValueError("expected list/tuple of 2 integers for attribute 'size'")
        return cls(cfg["mode"], size, align_hz=cfg.get("align-horizontal", "left"),
                   align_vt=cfg.get("align-vertical", "top"))

    def __init__(self, mode, size, align_hz="left", align_vt="top"):
        if align_hz not in ("left", "center", "right"):
            raise ValueError(f"invalid horizontal alignment for padding: {align_hz}")
        if align_vt not in ("bottom", "center", "top"):
            raise ValueError(f"invalid vertical alignment for padding: {align_vt}")
        if mode not in _MODES and mode not in _STAT_MODES:
            raise ValueError(f"invalid padding mode: {mode}")
        self.mode, self.size, self.align_hz, self.align_vt = mode, size, align_hz, align_vt

    def get_config(self):
        return {"type": self.type, "mode": self.mode, "size": self.size,
                "align-horizontal": self.align_hz, "align-vertical": self.align_vt}

    def extents(self, h, w):
        """(new_h, new_w, (ph1, ph2), (pw1, pw2)) as input.py:93-118."""
        new_h = (h + self.size[1] - 1) // self.size[1] * self.size[1]
        new_w = (w + self.size[0] - 1) // self.size[0] * self.size[0]
        ph, pw = new_h - h, new_w - w
        ph1 = {"top": 0, "bottom": ph, "center": ph // 2}[self.align_vt]
        pw1 = {"left": 0, "right": pw, "center": pw // 2}[self.align_hz]
        return new_h, new_w, (ph1, ph - ph1), (pw1, pw - pw1)

    def mode_id(self):
        if self.mode in _STAT_MODES:
            raise NotImplementedError(f"rmd: padding mode '{self.mode}' is not provided on the GPU")
        return _MODES[self.mode]


def _build_padding(cfg):
    if cfg is None:
        return None
    return {ModuloPadding.type: ModuloPadding}[cfg["type"]].from_config(cfg)


def _to_gpu(a, dtype, device):
    t = torch.as_tensor(np.ascontiguousarray(a)) if isinstance(a, np.ndarray) else a
    return t.to(device=device, dtype=dtype, non_blocking=True).contiguous()


class InputSpec:
    """input.py:153-190 with a GPU prepare()."""

    @classmethod
    def from_config(cls, cfg):
        cfg = cfg if cfg is not None else {}
        clip = [float(x) for x in cfg.get("clip", (0, 1))]
        if len(clip) != 2:
            raise ValueError("invalid value for 'clip', expected list/tuple of two floats")
        rng = cfg.get("range", (-1, 1))
        if len(rng) != 2:
            raise ValueError("invalid value for 'range', expected list/tuple of two floats")
        return cls(clip, rng, _build_padding(cfg.get("padding")))

    def __init__(self, clip=(0.0, 1.0), range=(-1.0, 1.0), padding=None):
        self.clip = clip
        self.range = range
        self.padding = padding

    def get_config(self):
        return {"clip": self.clip, "range": self.range,
                "padding": self.padding.get_config() if self.padding is not None else None}

    def prepare(self, img1, img2, flow=None, valid=None, device="cuda"):
        """(B,H,W,C) frames (+ (B,H,W,2) flow, (B,H,W) valid), numpy or torch, host or GPU ->
        img1, img2 (B,C,H',W') float32, flow (B,2,H',W') float32, valid (B,H',W') bool, extents
        ((h1, h2), (w1, w2)) per input.py:133-135, all on the GPU."""
        device = torch.device(device)
        if device.type == "cpu":
            return self._prepare_host(img1, img2, flow, valid)
        if device.type != "cuda":
            raise RuntimeError(f"rmd: prepare() runs on 'cuda' (HIP kernels) or 'cpu', got '{device.type}'")
        i1, i2 = _to_gpu(img1, torch.float32, device), _to_gpu(img2, torch.float32, device)
        if i1.dim() != 4 or i1.shape != i2.shape:
            raise ValueError(f"img1/img2 must be equal (B,H,W,C) shapes, got {tuple(i1.shape)} / {tuple(i2.shape)}")
        b, h, w, c = i1.shape
        if self.padding is not None:
            hp, wp, (ph1, ph2), (pw1, pw2) = self.padding.extents(h, w)
            mode = self.padding.mode_id()
        else:
            hp, wp, ph1, ph2, pw1, pw2, mode = h, w, 0, 0, 0, 0, 0
        outs = []
        with torch.cuda.device(device):
            for im in (i1, i2):
                o = torch.empty((b, c, hp, wp), dtype=torch.float32, device=device)
                _lib.check(_lib.lib().rmd_input_images(
                    _ptr(im), b, h, w, c, float(self.clip[0]), float(self.clip[1]), float(self.range[0]),
                    float(self.range[1]), hp, wp, ph1, pw1, mode, _ptr(o), _stream(o)), "rmd_input_images")
                outs.append(o)
            fo = vo = None
            if flow is not None:
                fl = _to_gpu(flow, torch.float32, device)
                va = _to_gpu(valid, torch.uint8, device)
                if tuple(fl.shape) != (b, h, w, 2) or tuple(va.shape) != (b, h, w):
                    raise ValueError(f"flow/valid must be (B,H,W,2)/(B,H,W), got {tuple(fl.shape)} / {tuple(va.shape)}")
                fo = torch.empty((b, 2, hp, wp), dtype=torch.float32, device=device)
                vo = torch.empty((b, hp, wp), dtype=torch.uint8, device=device)
                _lib.check(_lib.lib().rmd_input_flow(_ptr(fl), _ptr(va), b, h, w, hp, wp, ph1, pw1, float(FLOW_INF),
                                                     _ptr(fo), _ptr(vo), _stream(fo)), "rmd_input_flow")
                vo = vo.bool()
        # input.py:133-135 adds (ph1, ph2) / (pw1, pw2) to the original ((0, h), (0, w)) extents
        extents = ((ph1, h + ph2), (pw1, w + pw2))
        return outs[0], outs[1], fo, vo, extents

    def _prepare_host(self, img1, img2, flow, valid):
        """device='cpu': the reference's own host path — np.clip + range map (input.py:215-221), np.pad
        in the padding mode (input.py:79-138; the statistic modes too), NHWC -> NCHW and the flow's
        nan_to_num / clip to +-FLOW_INF (TorchAdapter, input.py:245-313) — as CPU tensors."""
        def host(a, dtype):
            a = a.detach().cpu().numpy() if isinstance(a, torch.Tensor) else np.asarray(a)
            return np.ascontiguousarray(a, dtype=dtype)
        i1, i2 = host(img1, np.float32), host(img2, np.float32)
        if i1.ndim != 4 or i1.shape != i2.shape:
            raise ValueError(f"img1/img2 must be equal (B,H,W,C) shapes, got {tuple(i1.shape)} / {tuple(i2.shape)}")
        b, h, w, c = i1.shape
        if self.padding is not None:
            hp, wp, (ph1, ph2), (pw1, pw2) = self.padding.extents(h, w)
        else:
            hp, wp, ph1, ph2, pw1, pw2 = h, w, 0, 0, 0, 0
        widths = ((0, 0), (ph1, ph2), (pw1, pw2), (0, 0))

        def pad(a):
            if self.padding is None or (ph1, ph2, pw1, pw2) == (0, 0, 0, 0):
                return a
            mode = self.padding.mode
            if mode in ("zeros", "ones"):
                return np.pad(a, widths, mode="constant", constant_values=0.0 if mode == "zeros" else 1.0)
            np_mode = {"torch.replicate": "edge", "torch.reflect": "reflect", "torch.circular": "wrap"}.get(mode, mode)
            return np.pad(a, widths, mode=np_mode)

        outs = []
        for im in (i1, i2):
            im = (self.range[1] - self.range[0]) * np.clip(im, self.clip[0], self.clip[1]) + self.range[0]
            outs.append(torch.from_numpy(np.ascontiguousarray(pad(im.astype(np.float32)).transpose(0, 3, 1, 2))))
        fo = vo = None
        if flow is not None:
            fl, va = host(flow, np.float32), host(valid, np.bool_)
            if fl.shape != (b, h, w, 2) or va.shape != (b, h, w):
                raise ValueError(f"flow/valid must be (B,H,W,2)/(B,H,W), got {fl.shape} / {va.shape}")
            fl = np.clip(np.nan_to_num(fl, nan=0.0, posinf=FLOW_INF, neginf=-FLOW_INF), -FLOW_INF, FLOW_INF)
            fl = np.pad(fl.astype(np.float32), widths, mode="constant")
            va = np.pad(va, widths[:3], mode="constant")
            fo = torch.from_numpy(np.ascontiguousarray(fl.transpose(0, 3, 1, 2)))
            vo = torch.from_numpy(np.ascontiguousarray(va))
        return outs[0], outs[1], fo, vo, ((ph1, h + ph2), (pw1, w + pw2))
