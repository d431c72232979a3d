"""HIP-graph capture of the rmd operators (include/rmd.h ABI rule: launchers never allocate, free or
synchronise, and launch on the caller's stream — torch's current stream — so torch.cuda.graph
captures them).  Each captured sequence replays bitwise equal to the eager result, also after the
inputs were overwritten in place (the graph reads the live buffers)."""

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _capture(fn):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):                      # warm-up outside the capture (allocator, hipFuncSetAttribute)
            fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = fn()
    return g, out


def _flow(b, h, w, g, scale):
    ys, xs = torch.meshgrid(torch.arange(h, dtype=torch.float32), torch.arange(w, dtype=torch.float32), indexing="ij")
    return (torch.stack([xs, ys])[None] + scale * torch.randn(b, 2, h, w, generator=g)).to(DEV)


@pytest.mark.parametrize("precision", ["bf16", "fp32"])
def test_corr_block_step_graph_replay(precision):
    from rmd import ops
    g = torch.Generator().manual_seed(0)
    b, c, h, w = 2, 256, 23, 40
    f1 = torch.randn(b, c, h, w, generator=g).to(DEV)
    f2 = torch.randn(b, c, h, w, generator=g).to(DEV)
    co = [_flow(b, h, w, g, 3.0) for _ in range(3)]

    def step():
        pyr = ops.corr_pyramid(f1, f2, 4, precision)
        return torch.stack([ops.corr_lookup(pyr, co[i], 4) for i in range(3)])

    graph, gout = _capture(step)
    graph.replay()
    torch.cuda.synchronize()
    assert torch.equal(gout, step())
    f1.copy_(torch.randn(b, c, h, w, generator=g).to(DEV))          # new inputs, same buffers
    co[1].add_(0.75)
    graph.replay()
    torch.cuda.synchronize()
    assert torch.equal(gout, step())


def test_dicl_dap_otf_graph_replay():
    from rmd import ops
    g = torch.Generator().manual_seed(1)
    b, c, h, w = 2, 32, 24, 40
    f1 = torch.randn(b, c, h, w, generator=g).to(DEV)
    f2 = torch.randn(b, c, h, w, generator=g).to(DEV)
    co = _flow(b, h, w, g, 2.0)
    wt = (torch.eye(81) + 0.05 * torch.randn(81, 81, generator=g)).to(DEV)[:, :, None, None]
    st = ops.otf_prepare(f1, f2, 2, "bf16")

    def step():
        stack = ops.dicl_stack(f1, f2, co, 4)                       # (B, 9, 9, 2C, h, w)
        cost = stack[:, :, :, :1].reshape(b, 81, h, w).contiguous()
        return ops.dap(cost, wt), ops.dicl_stack_int(f1, f2, 3, 3), ops.otf_lookup(st, co, 4)

    graph, gouts = _capture(step)
    graph.replay()
    torch.cuda.synchronize()
    for a, e in zip(gouts, step()):
        assert torch.equal(a, e)
