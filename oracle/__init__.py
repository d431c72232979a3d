"""CPU restatement of qzed/raft-meets-dicl's cost-volume hot path — TEST INFRASTRUCTURE ONLY.

This package is the parity oracle.  It restates the reference algorithm directly (numpy) and is pinned against golden vectors produced
by running the reference itself (``tests/golden/gen_golden.py``; checked by
``tests/test_oracle_golden.py``).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import,
call or link anything under ``oracle/``, and only as the checker / the timed CPU baseline.  The
product path (``raft-meets-dicl_amd/``) never imports it and has no CPU fallback.
"""

from .corr import (corr_volume, corr_pyramid, corr_lookup, corr_lookup_fs, corr_lookup_backward,
                   corr_lookup_fs_backward, pyramid_level_shapes)
from .dicl import (dicl_stack, dicl_stack_at, dicl_stack_backward, dicl_stack_int, dicl_stack_int_at,
                   dicl_stack_int_backward, dap, dap_backward,
                   warp_backwards, warp_backwards_backward)
from .heads import up8, up8_backward, softargmax, softargmax_backward
from .input import input_images, input_flow, pad_extents

__all__ = ["corr_volume", "corr_pyramid", "corr_lookup", "corr_lookup_fs", "corr_lookup_backward",
           "corr_lookup_fs_backward",
           "pyramid_level_shapes", "dicl_stack", "dicl_stack_at", "dicl_stack_backward", "dicl_stack_int",
           "dicl_stack_int_at",
           "dicl_stack_int_backward", "dap", "dap_backward", "up8", "up8_backward", "softargmax",
           "softargmax_backward", "warp_backwards", "warp_backwards_backward", "input_images", "input_flow",
           "pad_extents"]
