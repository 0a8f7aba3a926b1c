"""Study: what does a cross-stream wait (hipStreamWaitEvent -> an AQL barrier packet) cost on the
waiting queue when the awaited work finished long ago? Two ~20 us copies per iteration on one
stream, optionally with a wait on an event of an idle second stream (recorded once per iteration,
before the first copy) between them; GPU time per iteration from events around 400 iterations.
The fused step's tail has one or two such joins before Adam (profiles/r5/tail_timeline_*_r5.txt).
"""
import torch


def run(n_wait: int, iters: int = 400) -> float:
    dev = torch.device("cuda", 0)
    a = torch.empty(16 << 20, device=dev)
    b = torch.empty_like(a)
    s0, s1 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    evs = [torch.cuda.Event() for _ in range(max(n_wait, 1))]
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def body():
        for e in evs[:n_wait]:
            e.record(s1)
        with torch.cuda.stream(s0):
            b.copy_(a)
            for e in evs[:n_wait]:
                s0.wait_event(e)
            a.copy_(b)

    for _ in range(20):
        body()
    torch.cuda.synchronize()
    t0.record(s0)
    for _ in range(iters):
        body()
    t1.record(s0)
    torch.cuda.synchronize()
    return t0.elapsed_time(t1) * 1e3 / iters


def main():
    res = {}
    for rnd in range(3):
        for n in (0, 1, 2):
            res.setdefault(n, []).append(run(n))
    base = sorted(res[0])[1]
    for n in (0, 1, 2):
        med = sorted(res[n])[1]
        print("waits %d: %.2f us/iteration (median of 3), +%.2f us vs none" % (n, med, med - base))


if __name__ == "__main__":
    main()
