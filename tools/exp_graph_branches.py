#!/usr/bin/env python
"""Do the parallel branches of a captured HIP graph run concurrently on this ROCm?  Two independent spin kernels
(torch.cuda._sleep, ~1 ms each) captured on a forked stream pair (event fork / join inside the capture) vs the same
two in one stream; replay wall per graph.  Concurrent branches -> ~1x, serialised -> ~2x."""
import time

import torch


def timed(g, n=20):
    g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        g.replay()
    torch.cuda.synchronize()
    return 1e3 * (time.perf_counter() - t0) / n


def main():
    cyc = 2_000_000
    s_cap = torch.cuda.Stream()
    s_side = torch.cuda.Stream()
    # warm
    torch.cuda._sleep(cyc)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    torch.cuda._sleep(cyc)
    torch.cuda.synchronize()
    one = 1e3 * (time.perf_counter() - t0)
    g1 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g1, stream=s_cap):
        torch.cuda._sleep(cyc)
        torch.cuda._sleep(cyc)
    g2 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g2, stream=s_cap):
        s_side.wait_stream(s_cap)
        torch.cuda._sleep(cyc)
        with torch.cuda.stream(s_side):
            torch.cuda._sleep(cyc)
        s_cap.wait_stream(s_side)
    print({"one_kernel_ms": round(one, 3), "serial_graph_ms": round(timed(g1), 3),
           "forked_graph_ms": round(timed(g2), 3)})


if __name__ == "__main__":
    main()
