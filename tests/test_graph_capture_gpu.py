"""The C-ABI is stream-ordered and never allocates or synchronises, so whole
rounds capture into a hipGraph (torch.cuda.CUDAGraph on ROCm) and replay with
one launch per graph instead of a tracing compiler: a FedADMM round (fused
ADMM-SGD + dual step, ordered mean) and a ring mix, replayed, are
bit-identical to the eager calls."""
import numpy as np
import pytest
import torch

from oracle import bits_equal
from dolhip import ops

pytestmark = pytest.mark.gpu


def test_captured_round_replays_bit_identically(gpu):
    n, P = 12, 4096 + 8
    g = torch.Generator(device=gpu).manual_seed(3)
    bufs = {k: torch.randn(n, P, generator=g, device=gpu) for k in ("w", "g", "mom", "alpha", "y")}
    theta = torch.randn(P, generator=g, device=gpu)
    wp, wn = torch.rand(n, generator=g, device=gpu), torch.rand(n, generator=g, device=gpu)
    order = torch.tensor([3, 0, 7, 11], dtype=torch.int32, device=gpu)
    mean = torch.empty(P, device=gpu)
    init = {k: v.clone() for k, v in bufs.items()}

    def round_():
        ops.admm_step_dual(bufs["w"], bufs["g"], theta, bufs["alpha"], buf=bufs["mom"], rho=0.1, lr=0.05,
                           momentum=0.5, first_step=False, write_grad=False)
        ops.ordered_mean(bufs["w"], order, out=mean)
        ops.mix_ring(bufs["w"], bufs["y"], wp, wn)

    round_()  # eager reference
    torch.cuda.synchronize()
    want = {k: v.clone() for k, v in bufs.items()}
    want_mean = mean.clone()
    for k in bufs:
        bufs[k].copy_(init[k])
    s = torch.cuda.Stream(device=gpu)
    s.wait_stream(torch.cuda.current_stream(gpu))
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(graph, stream=s):
            round_()
    torch.cuda.current_stream(gpu).wait_stream(s)
    for k in bufs:  # capture does not execute; reset anyway and replay
        bufs[k].copy_(init[k])
    graph.replay()
    torch.cuda.synchronize()
    for k in bufs:
        assert bits_equal(bufs[k].cpu().numpy(), want[k].cpu().numpy()), k
    assert bits_equal(mean.cpu().numpy(), want_mean.cpu().numpy())
