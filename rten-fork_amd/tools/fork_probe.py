"""Probe: do forked branches of a captured hipGraph run concurrently on
MI355X, and what does a fork/join cost?  torch.cuda._sleep spins one
workgroup for a cycle count."""
import time
import torch

def timeit(fn, n=200):
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e6

cyc = 20000  # ~ 10 us at ~2.1 GHz?
main = torch.cuda.Stream()
side = torch.cuda.Stream()

def serial():
    for _ in range(4):
        torch.cuda._sleep(cyc)

def forked():
    cur = torch.cuda.current_stream()
    for _ in range(2):
        side.wait_stream(cur)
        torch.cuda._sleep(cyc)
        with torch.cuda.stream(side):
            torch.cuda._sleep(cyc)
        cur.wait_stream(side)

def chain_only(k):
    def f():
        for _ in range(k):
            torch.cuda._sleep(cyc)
    return f

with torch.cuda.stream(main):
    print(f"eager 1 sleep: {timeit(chain_only(1)):.1f} us, 4 serial: {timeit(serial):.1f} us, 2x(fork 2): {timeit(forked):.1f} us")
    for name, fn in (("serial4", serial), ("fork2x2", forked), ("one", chain_only(1)), ("two", chain_only(2))):
        g = torch.cuda.CUDAGraph()
        fn()
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=main):
            fn()
        def rep():
            g.replay()
        print(f"graph {name}: {timeit(rep):.1f} us/replay")
