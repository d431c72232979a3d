"""Op selection from the model configuration — the drop-in's answer to SURVEY.md §5 "Config / flags".

The reference builds every model from a cfg/model/*.yaml whose ``model.parameters`` section goes to
``Model.from_config`` (e.g. src/models/impls/raft_fs.py:175-197 reads 'corr-levels', 'corr-radius',
'mixed-precision', ... with ``param_cfg.get(key, default)``) and comes back out of ``get_config()``.
The correlation blocks it then constructs take only ``(fmap1, fmap2, num_levels, radius)``
(raft.py:384, raft_fs.py:132).  The drop-in reads three more keys from that same ``parameters``
section; all are optional and their defaults reproduce the reference:

  corr-precision      fp32 (default: split-bf16 MFMA, 24-bit pyramid (fp32 rounded to 16 significant
                      bits), ~1e-5 of the reference) | fp32-f32 (same GEMM, fp32 pyramid) | fp32-s24 (= fp32) |
                      fp32-exact | bf16 (bf16 MFMA, fp16 pyramid: the bench mode) | bf16-f32 | fp32-f16
  corr-method         auto (default) | volume | otf — all-pairs pyramid + lookup, or the on-the-fly
                      lookup with no O(N^2) buffer (both differentiable); auto takes the volume unless
                      its bytes (pyramid, plus the dense fp32 gradient when training) pass the budget
  corr-memory-budget  bytes the volume may take before auto switches to otf (int, or a string with a
                      KiB / MiB / GiB suffix; default 16 GiB)

A maintainer passes them where the reference reads its other parameters — either per block:
    CorrBlock(fmap1, fmap2, num_levels=..., radius=..., **rmd.config.corr_options(param_cfg).kwargs())
or once per process, from ``Model.from_config``:  ``rmd.config.configure(cfg['parameters'])``
(INTEGRATION.md §2).  Blocks constructed with ``precision=None`` / ``method=None`` use the process
values.
"""

import re
from collections import namedtuple

PRECISIONS = ("fp32", "fp32-f32", "fp32-s24", "fp32-exact", "bf16", "bf16-f32", "fp32-f16")
METHODS = ("auto", "volume", "otf")
KEYS = ("corr-precision", "corr-method", "corr-memory-budget")
DEFAULTS = {"corr-precision": "fp32", "corr-method": "auto", "corr-memory-budget": 16 << 30}

_STORAGE_BYTES = {"fp32": 3, "fp32-f32": 4, "fp32-s24": 3, "fp32-exact": 4, "bf16": 2, "bf16-f32": 4, "fp32-f16": 2}


class CorrOptions(namedtuple("CorrOptions", ["precision", "method", "memory_budget"])):
    """Validated correlation options (constructor keyword arguments of the drop-in blocks)."""

    def kwargs(self):
        return {"precision": self.precision, "method": self.method, "memory_budget": self.memory_budget}

    def parameters(self):
        """The ``parameters`` entries that reproduce these options (for ``Model.get_config``)."""
        return {"corr-precision": self.precision, "corr-method": self.method,
                "corr-memory-budget": self.memory_budget}


def _bytes(v):
    if isinstance(v, (int, float)) and not isinstance(v, bool):
        if v <= 0:
            raise ValueError(f"corr-memory-budget must be positive, got {v}")
        return int(v)
    m = re.fullmatch(r"\s*([0-9]+(?:\.[0-9]*)?)\s*([KMGT]i?B?|B)?\s*", str(v), re.IGNORECASE)
    if not m:
        raise ValueError(f"corr-memory-budget: cannot parse {v!r} (bytes, or a number with KiB/MiB/GiB)")
    unit = (m.group(2) or "B").upper().rstrip("B").rstrip("I")
    mult = {"": 1, "K": 1 << 10, "M": 1 << 20, "G": 1 << 30, "T": 1 << 40}[unit]
    return _bytes(float(m.group(1)) * mult)


def corr_options(parameters=None, **overrides):
    """CorrOptions from a cfg/model ``parameters`` mapping (missing keys: the process values), with
    keyword overrides ``precision`` / ``method`` / ``memory_budget``.  Unknown values raise ValueError,
    as the reference's from_config does for bad types."""
    base = _current
    p = dict(parameters or {})
    def pick(key, pkey, default):
        # an explicit override wins even when falsy (0, ''): it then reaches the validation below
        v = overrides.get(key)
        return v if v is not None else p.get(pkey, default)

    precision = pick("precision", "corr-precision", base.precision)
    method = pick("method", "corr-method", base.method)
    budget = pick("memory_budget", "corr-memory-budget", base.memory_budget)
    if precision not in PRECISIONS:
        raise ValueError(f"unknown corr-precision '{precision}', expected one of {list(PRECISIONS)}")
    if method not in METHODS:
        raise ValueError(f"unknown corr-method '{method}', expected one of {list(METHODS)}")
    return CorrOptions(precision, method, _bytes(budget))


_current = CorrOptions(DEFAULTS["corr-precision"], DEFAULTS["corr-method"], DEFAULTS["corr-memory-budget"])


def configure(parameters=None, **overrides):
    """Set the process-wide options from a cfg/model ``parameters`` mapping (what ``Model.from_config``
    would call); returns the previous options (pass them back to ``restore``)."""
    global _current
    prev = _current
    _current = corr_options(parameters, **overrides)
    return prev


def restore(opts):
    global _current
    _current = opts


def current():
    return _current


_ELEMENT_BYTES = {0: 4, 1: 2, 4: 3}     # RMD_F32, RMD_F16, RMD_S24 (include/rmd.h)


def pyramid_bytes(batch, height, width, levels, precision, channels=None, gpu=True):
    """HBM bytes of the pyramid a block of this precision writes, in the storage and layout the call
    resolves (rmd_pyramid_describe_for): the 24-bit S24 storage of 'fp32' / 'fp32-s24' exists only where
    the split-bf16 x3 GEMM runs (a GPU block, C <= 256, every S24 level slab < 2 GiB) — elsewhere the
    pyramid is F32, a third larger; the bf16 GEMM's tiles layout pads odd heights.  Without
    the channel count the S24 modes are charged F32 bytes (the larger of the two)."""
    from . import _lib, ops                  # lazy: no import-time dependency on the library
    compute, storage = ops.PRECISIONS[precision]
    if storage == _lib.RMD_S24 and (not gpu or channels is None):
        storage = _lib.RMD_F32                # CPU kernels store F32; unknown C: the larger storage
    if gpu and channels is not None:
        d = _lib.describe_for(batch, height, width, levels, storage, channels, compute)
    else:
        d = _lib.describe(batch, height, width, levels, storage)
    return d.total_elements * _ELEMENT_BYTES[d.storage]


def volume_bytes(batch, height, width, levels, precision, training, channels=None, gpu=True):
    """HBM bytes of the all-pairs path for a (batch, height, width) query grid: the pooled pyramid in the
    storage the call resolves (pyramid_bytes), plus the dense fp32 pyramid gradient when training.  A
    training block also keeps each lookup's fp32 gradient until the pyramid backward, up to
    rmd.ops.GRAD_PENDING_BYTES (1 GiB) before they are folded into G — at most that much more."""
    n = height * width
    t = sum((height >> l) * (width >> l) for l in range(levels))
    b = pyramid_bytes(batch, height, width, levels, precision, channels, gpu)
    if training:
        b += batch * n * (t + 8 * levels * height) * 4          # G over the 8-padded target rows
    return b


OTF_BACKWARD_MAX_CHANNELS = 256       # rmd_corr_otf_backward's limit (include/rmd.h)


def choose_method(method, batch, height, width, levels, precision, training, budget, channels=None, gpu=True):
    """'volume' or 'otf' for a block: explicit methods pass through; 'auto' takes the volume while it
    fits the budget (volume_bytes, with the storage resolved for `channels` on a GPU block).  A GPU
    training block with more than 256 channels has no on-the-fly backward: 'auto' keeps the volume for
    it and an explicit 'otf' raises here, at construction, instead of in backward (the CPU kernels
    train any channel count)."""
    otf_trainable = not training or not gpu or channels is None or channels <= OTF_BACKWARD_MAX_CHANNELS
    if method == "otf" and not otf_trainable:
        raise ValueError(f"corr-method 'otf' cannot train a block with {channels} channels "
                         f"(the on-the-fly backward supports C <= {OTF_BACKWARD_MAX_CHANNELS}); use 'volume'")
    if method != "auto":
        return method
    if not otf_trainable:
        return "volume"
    vb = volume_bytes(batch, height, width, levels, precision, training, channels, gpu)
    return "otf" if vb > budget else "volume"
