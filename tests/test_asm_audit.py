"""Static audit of the hand-pipelined correlation GEMM (corr_pyramid_stationary) in its gfx950 .s.

The kernel issues its B-fragment loads in inline asm and retires them with ONE hand-placed
`s_waitcnt vmcnt(23)`; that is only correct if, between each block of 16 asm loads and its wait,
the wave issues exactly 23 other vector-memory ops (the epilogue stores), the 16 destination
registers are not touched, and nothing spills to scratch.  Compiled here with hipcc -save-temps.
"""

import os
import re
import shutil
import subprocess
import tempfile

import pytest

from conftest import ROOT

HIPCC = "/opt/rocm/bin/hipcc"
SRC = os.path.join(ROOT, "raft-meets-dicl_amd", "csrc", "corr_pyramid.hip")
STORES_PER_TILE = {1: 12, 2: 23}      # STraits<TH>::kStores


def _regs(line):
    out = set()
    for m in re.finditer(r"\bv\[(\d+):(\d+)\]", line):
        out |= set(range(int(m.group(1)), int(m.group(2)) + 1))
    for m in re.finditer(r"\bv(\d+)\b", line):
        out.add(int(m.group(1)))
    return out


@pytest.fixture(scope="module")
def module_asm():
    if not os.path.exists(HIPCC):
        pytest.skip("hipcc not available")
    tmp = tempfile.mkdtemp()
    try:
        subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", f"-I{ROOT}/include",
                        f"-I{os.path.dirname(SRC)}", "-save-temps", "-c", SRC, "-o", os.path.join(tmp, "x.o")],
                       cwd=tmp, check=True, capture_output=True, timeout=600)
        s = [f for f in os.listdir(tmp) if f.endswith(".s") and "gfx950" in f][0]
        txt = open(os.path.join(tmp, s)).read()
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    return txt


@pytest.fixture(params=[1, 2], ids=["8waves", "4waves"])
def kernel_asm(request, module_asm):
    th = request.param
    m = re.search(rf"^(_ZN3rmd\w*corr_pyramid_stationaryILi{th}ELi0E\w*):[^\n]*\n(.*?)\.end_amdhsa_kernel",
                  module_asm, re.S | re.M)
    assert m, f"stationary<{th}, 0> kernel not found"
    return th, m.group(2).split("\n")


def test_no_scratch(kernel_asm):
    assert not any("scratch_" in ln for ln in kernel_asm[1])


def _asm_flags(lines):
    """Per line: True if it lies inside an inline-asm region (;;#ASMSTART .. ;;#ASMEND)."""
    inside, flags = False, []
    for ln in lines:
        if "ASMSTART" in ln:
            inside = True
        elif "ASMEND" in ln:
            inside = False
        flags.append(inside)
    return flags


def test_every_asm_load_window_is_exact(kernel_asm):
    th, lines = kernel_asm
    asm = _asm_flags(lines)
    loads = [i for i, ln in enumerate(lines) if asm[i] and "global_load_dwordx4" in ln]
    assert len(loads) % 16 == 0 and loads, "asm B-fragment loads come in blocks of 16"
    windows = 0
    for k in range(0, len(loads), 16):
        blk = loads[k:k + 16]
        dests = set()
        for i in blk:
            dests |= _regs(lines[i].split(",")[0])
        stores = 0
        j = blk[0] + 1
        while j < len(lines) and not (asm[j] and "s_waitcnt vmcnt" in lines[j]):
            ln = lines[j]
            if j in blk:
                pass
            elif "global_store" in ln or "buffer_store" in ln:
                stores += 1
            elif "global_load" in ln or "buffer_load" in ln or "flat_" in ln or "scratch_" in ln:
                raise AssertionError(f"unexpected vector-memory op in a load window: {ln.strip()}")
            elif j > blk[-1] and not ln.strip().startswith(";") and (_regs(ln) & dests):
                raise AssertionError(f"in-flight load register touched before its wait: {ln.strip()}")
            j += 1
        n = int(re.search(r"vmcnt\((\d+)\)", lines[j]).group(1))
        if n == 0:
            assert stores == 0          # prologue load: drained outright
        else:
            assert n == STORES_PER_TILE[th] and stores == STORES_PER_TILE[th], (n, stores)
            windows += 1
    assert windows >= 1, "expected the pipelined load window of the loop"
