"""Which cross-stream event patterns survive HIP graph capture (torch.cuda.graph) on this stack."""
import sys

import torch


def run(pattern):
    dev = torch.device("cuda", 0)
    main = torch.cuda.Stream(device=dev)
    s1, s2 = torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev)
    x = torch.ones(1024, device=dev)
    g = torch.cuda.CUDAGraph()
    st = {"main": None, "s1": s1, "s2": s2}
    with torch.cuda.stream(main):
        with torch.cuda.graph(g):
            st["main"] = torch.cuda.current_stream()
            ev = {}

            def sig(who, tag):
                e = torch.cuda.Event()
                e.record(st[who])
                ev[tag] = e

            def wait(who, tag):
                st[who].wait_event(ev[tag])

            def work(who):
                with torch.cuda.stream(st[who]):
                    x.add_(1.0)
            sig("main", "fork"); wait("s1", "fork"); wait("s2", "fork")
            work("s1"); work("s2"); work("main")
            if pattern == "side_to_side":
                sig("s1", "a"); wait("s2", "a"); work("s2")
            sig("s1", "j1"); sig("s2", "j2"); wait("main", "j1")
            if pattern != "transitive":
                wait("main", "j2")
            else:
                wait("s1", "j2"); sig("s1", "j3"); wait("main", "j3")
    g.replay()
    torch.cuda.synchronize()
    print(pattern, "ok", float(x[0]), flush=True)


run(sys.argv[1])
