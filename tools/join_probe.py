"""Cost of a side-stream join inside a captured HIP graph: a chain of 40 small kernels on the main
stream (GPU-side: every replay is enqueued behind a long sleep kernel), with (a) nothing else, (b) one kernel forked onto a side stream at the start and joined
after kernel 20, (c) the same fork joined at the end only.  Prints the replay time of each (best of
5 x 200 replays)."""
import torch


def main():
    dev = torch.device("cuda")
    x = torch.zeros(1 << 16, device=dev)
    y = torch.zeros(1 << 16, device=dev)
    s, side = torch.cuda.Stream(), torch.cuda.Stream()

    def body(mode):
        if mode != "none":
            side.wait_stream(s)
            with torch.cuda.stream(side):
                y.add_(1.0)
        for i in range(40):
            if mode == "mid" and i == 20:
                s.wait_stream(side)
            x.add_(1.0)
        if mode != "none":
            s.wait_stream(side)

    res = {}
    for mode in ("none", "mid", "end"):
        g = torch.cuda.CUDAGraph()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            body(mode)
            torch.cuda.synchronize()
            with torch.cuda.graph(g, stream=s):
                body(mode)
        best = None
        for _ in range(5):
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            with torch.cuda.stream(s):
                torch.cuda._sleep(200_000_000)   # (the host enqueues every replay while the GPU sleeps)
            e0.record(s)
            with torch.cuda.stream(s):
                for _ in range(200):
                    g.replay()
            e1.record(s)
            e1.synchronize()
            t = e0.elapsed_time(e1) / 200 * 1e3
            best = t if best is None else min(best, t)
        res[mode] = best
        print(f"{mode:5s} {best:8.2f} us per replay", flush=True)
    print(f"join mid-chain costs {res['mid'] - res['end']:.2f} us; fork+join at the end {res['end'] - res['none']:.2f} us")
    # (d) the same work as three single-stream graphs: head / tail on the main stream, the side kernel
    # on the side stream, joined by a stream-level event between head and tail
    gh, gt, gs = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(gh, stream=s):
            for _ in range(20):
                x.add_(1.0)
        with torch.cuda.graph(gt, stream=s):
            for _ in range(20):
                x.add_(1.0)
    with torch.cuda.stream(side):
        with torch.cuda.graph(gs, stream=side):
            y.add_(1.0)
    torch.cuda.synchronize()
    for join in (False, True):
        best = None
        for _ in range(5):
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            with torch.cuda.stream(s):
                torch.cuda._sleep(200_000_000)
            e0.record(s)
            for _ in range(200):
                if join:
                    side.wait_stream(s)
                    with torch.cuda.stream(side):
                        gs.replay()
                    ev = torch.cuda.Event()
                    ev.record(side)
                with torch.cuda.stream(s):
                    gh.replay()
                    if join:
                        s.wait_event(ev)
                    gt.replay()
            e1.record(s)
            e1.synchronize()
            t = e0.elapsed_time(e1) / 200 * 1e3
            best = t if best is None else min(best, t)
        print(f"split graphs {'with' if join else 'without'} the side graph + event join: {best:8.2f} us", flush=True)


if __name__ == "__main__":
    main()
