#!/usr/bin/env python3
"""Locate wrong outputs of rmd_dap against torch fp32: counts of bad entries per image, 32-row tile,
wave (32-pixel tile mod 8) and workgroup block, for a few shapes.  usage: dap_diag.py [lib ...]"""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "raft-meets-dicl_amd"))
from rmd import _lib  # noqa: E402

for path in (sys.argv[1:] or [None]):
  lib = _lib.lib() if path is None else ctypes.CDLL(os.path.abspath(path))
  print(json.dumps({"lib": path or "librmd.so"}))
  lib.rmd_dap.argtypes = [ctypes.c_void_p] * 2 + [ctypes.c_int] * 4 + [ctypes.c_void_p] * 2
  dev = torch.device("cuda:0")
  st = torch.cuda.current_stream()
  g = torch.Generator().manual_seed(0)
  for b, d, h, w in [(1, 324, 12, 16), (1, 324, 16, 32), (1, 324, 16, 64), (1, 324, 48, 160), (8, 324, 12, 16),
                     (8, 324, 48, 160), (2, 132, 48, 160)]:
      n = h * w
      x = torch.randn(b, d, n, generator=g).to(dev)
      wt = (torch.randn(d, d, generator=g) * 0.05).to(dev)
      out = torch.full_like(x, float("nan"))
      assert lib.rmd_dap(x.data_ptr(), wt.data_ptr(), b, d, n, 0, out.data_ptr(), ctypes.c_void_p(st.cuda_stream)) == 0
      torch.cuda.synchronize()
      ref = wt @ x
      bad = ~((out - ref).abs() <= 1e-3 * ref.abs().max())
      res = {"shape": [b, d, h, w], "bad": int(bad.sum()), "of": bad.numel()}
      if res["bad"]:
          nz = bad.nonzero()
          bi, ro, px = nz[:, 0], nz[:, 1], nz[:, 2]
          res["per_image"] = torch.bincount(bi, minlength=b).tolist()
          res["per_rowtile"] = torch.bincount(ro // 32).tolist()
          res["per_wave"] = torch.bincount((px // 32) % 8, minlength=8).tolist()
          res["per_wgblock"] = torch.bincount(px // 256).tolist()[:40]
          res["per_pixel_in_tile"] = torch.bincount(px % 32, minlength=32).tolist()
          res["per_row_in_tile"] = torch.bincount(ro % 32, minlength=32).tolist()
          res["nan"] = int(out.isnan().sum())
      if hasattr(lib, "rmd_dap_debug_read"):
          cnt = (ctypes.c_uint * 4)()
          lib.rmd_dap_debug_read(cnt)
          res["debug_x_w0_w1"] = list(cnt)[:3]
      print(json.dumps(res), flush=True)
