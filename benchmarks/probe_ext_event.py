"""Probe: an external event recorded INSIDE a captured hipGraph (torch.cuda.Event(external=True))
orders work issued outside the graph on another stream after the graph launch -- the mechanism a
one-graph DDP step needs to start collectives mid-graph. Prints ok / FAIL per replay."""
import torch


def main():
    dev = torch.device("cuda", 0)
    s_main = torch.cuda.Stream(device=dev)
    s_comm = torch.cuda.Stream(device=dev)
    ev = torch.cuda.Event(external=True)
    x = torch.zeros(1 << 20, device=dev)
    y = torch.zeros(1 << 20, device=dev)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s_main):
        torch.cuda._sleep(1000)
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=s_main):
            torch.cuda._sleep(2_000_000)  # ~1 ms: the work before the mid-graph event
            x.add_(1.0)
            ev.record()
            torch.cuda._sleep(2_000_000)  # more graph work after the event
            x.add_(100.0)
    ok = True
    for it in range(3):
        with torch.cuda.stream(s_main):
            g.replay()
        s_comm.wait_event(ev)
        with torch.cuda.stream(s_comm):
            y.copy_(x)                    # must see exactly the pre-event value of THIS replay
        torch.cuda.synchronize()
        want = 1.0 + 101.0 * it
        got = float(y[0])
        print("replay %d: outside-graph copy saw %.1f (want %.1f, graph end %.1f): %s" %
              (it, got, want, float(x[0]), "ok" if got == want else "FAIL"))
        ok = ok and got == want
    print("EXTERNAL_EVENT_OK" if ok else "EXTERNAL_EVENT_FAIL")


if __name__ == "__main__":
    main()
