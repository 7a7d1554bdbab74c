"""Does one cross-stream fork/join make a whole hipGraph slower?  Replays a graph of N tiny kernels
captured on one stream (linear), and the same graph with a side-stream branch of one kernel forked in
the middle and joined before the end (the DDP bucket all-reduce shape).  Reports us per replay and
the per-kernel difference.  python tools/graph_fork_probe.py"""
import json

import torch


def build(n, forks):
    x = torch.zeros(1024, device="cuda")
    y = torch.zeros(1024, device="cuda")
    side = torch.cuda.Stream()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s), torch.cuda.graph(g, stream=s):
        for i in range(n):
            x.add_(1.0)
            if forks and i in forks:
                side.wait_stream(s)
                with torch.cuda.stream(side):
                    y.add_(1.0)
                s.wait_stream(side) if forks[i] == "join_now" else None
        if forks:
            s.wait_stream(side)
    torch.cuda.synchronize()
    return g


def timeit(g, iters=50):
    for _ in range(5):
        g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        g.replay()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / iters * 1000.0


def main():
    for n in (50, 200):
        lin = timeit(build(n, None))
        one = timeit(build(n, {n // 2: "late_join"}))
        three = timeit(build(n, {n // 4: "late_join", n // 2: "late_join", 3 * n // 4: "late_join"}))
        print(json.dumps({"kernels": n, "linear_us": round(lin, 1), "one_fork_us": round(one, 1),
                          "three_forks_us": round(three, 1),
                          "extra_per_kernel_us": round((one - lin) / n, 3)}), flush=True)


if __name__ == "__main__":
    main()
