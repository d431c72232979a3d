"""Static audit of the correlation GEMM kernels in their gfx950 .s.

corr_pyramid_w8 (the default bf16 path): no scratch, accumulators in VGPRs (no v_accvgpr_read
round trips), exactly 128 MFMAs and 23 buffer stores per 32-query tile, every store range-checked
(buffer_store ... offen), the B-fragment loads coalesced global_load_dwordx4.

corr_pyramid_stationary<2, 0> (the product path for maps whose 32-bit store offsets would overflow,
e.g. 4K frames; GPU test: test_gpu_corr.py::test_stationary_path_4k_sampled_vs_oracle):

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
HIPFLAGS = ["-fno-slp-vectorize"]      # as raft-meets-dicl_amd/csrc/Makefile
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
                        f"-I{os.path.dirname(SRC)}", "-save-temps", *HIPFLAGS, "-c", SRC, "-o", os.path.join(tmp, "x.o")],
                       cwd=tmp, check=True, capture_output=True, timeout=600)
        s = [f for f in os.listdir(tmp) if f.endswith(".s") and "gfx950" in f][0]
        txt = open(os.path.join(tmp, s)).read()
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    return txt


@pytest.fixture(params=[2], ids=["4waves"])
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


@pytest.fixture
def w8_asm(module_asm):
    m = re.search(r"^(_ZN3rmd\w*corr_pyramid_w8ILi2E\w*):[^\n]*\n(.*?)\.end_amdhsa_kernel", module_asm, re.S | re.M)
    assert m, "corr_pyramid_w8<2> not found"
    return m.group(2).split("\n")


def test_w8_no_scratch_no_agpr_round_trips(w8_asm):
    body = [ln.strip() for ln in w8_asm]
    assert not any(ln.startswith("scratch_") for ln in body)
    assert not any(ln.startswith("v_accvgpr_read") for ln in body)


def test_w8_one_tile_per_loop_iteration(w8_asm):
    """The tile loop holds 128 MFMAs (16 k-steps x 8 target tiles), 16 B-fragment loads and the 23
    range-checked epilogue stores (16 + 4 + 2 + 1 over levels 0-3)."""
    body = [ln.strip() for ln in w8_asm]
    heads = [i for i, ln in enumerate(body) if "Loop Header" in ln]
    assert heads, "no loop found"
    start = heads[-1]
    end = max(i for i, ln in enumerate(body) if ln.startswith("s_cbranch") and i > start)
    loop = body[start:end]
    assert sum(ln.startswith("v_mfma_f32_32x32x16_bf16") for ln in loop) == 128
    assert sum(ln.startswith("global_load_dwordx4") for ln in loop) == 16
    stores = [ln for ln in loop if ln.startswith("buffer_store")]
    assert len(stores) == 23 and all(" offen" in ln for ln in stores)


def test_dicl_backward_has_no_flat_atomics():
    """The DICL backward kernels accumulate tap gradients into an LDS window with ds_add_f32;
    a pointer selected between the window and global memory would be generic and turn every
    add into a flat atomic (measured 0.96 vs 0.27 ms at cfg4).  Audit the whole dicl.hip module."""
    if not os.path.exists(HIPCC):
        pytest.skip("hipcc not available")
    src = os.path.join(ROOT, "raft-meets-dicl_amd", "csrc", "dicl.hip")
    tmp = tempfile.mkdtemp()
    try:
        out = os.path.join(tmp, "dicl.s")
        subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", f"-I{ROOT}/include",
                        f"-I{os.path.dirname(src)}", *HIPFLAGS, "--cuda-device-only", "-S", src, "-o", out],
                       check=True, capture_output=True, timeout=600)
        txt = open(out).read()
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    assert "flat_atomic" not in txt
    assert txt.count("ds_add_f32") > 0


def test_product_library_reads_no_environment():
    """A/B knobs and ablations live in the diagnostic build only (`make diag` -> librmd_diag.so):
    the product library imports no getenv and names no RMD_* variable."""
    lib = os.path.join(ROOT, "raft-meets-dicl_amd", "rmd", "librmd.so")
    if not os.path.exists(lib):
        pytest.skip("librmd.so not built")
    syms = subprocess.run(["nm", "-D", "--undefined-only", lib], capture_output=True, text=True, check=True).stdout
    assert "getenv" not in syms
    data = open(lib, "rb").read()
    for name in (b"RMD_ABLATE", b"RMD_LOOKUP_SPLIT", b"RMD_LOOKUP_NT", b"RMD_GEMM_KERNEL", b"RMD_STORE_AUX",
                 b"RMD_OTF_ABLATE", b"RMD_DICL_BWD_ABL"):
        assert name not in data, name
