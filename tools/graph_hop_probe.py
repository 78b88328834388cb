"""Cost of a cross-stream dependency in a replayed HIP graph (round 3): a chain of N tiny kernels
captured (a) all on one stream, (b) alternating between the capture stream and a second stream, an event edge per hop,
(c) on one stream but each kernel also waiting on an event recorded by an idle second stream at the
start, (d) two kernels per step on one stream vs (e) the same two forked onto two streams and joined
every step.  Replay time per kernel (per step for d/e).
usage: python tools/graph_hop_probe.py [N] -> one JSON line."""
import json
import sys

import torch

N = int(sys.argv[1]) if len(sys.argv) > 1 else 64
dev = torch.device("cuda")
x = torch.zeros(1024, device=dev)
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()


def chain_single():
    for _ in range(N):
        x.add_(1.0)


def chain_pingpong():
    # alternating between the capture stream and s1 (two non-capture streams ping-ponging crashes torch's
    # capture_end on this stack: DESIGN.md section 4)
    main = torch.cuda.current_stream()
    cur, oth = main, s1
    for _ in range(N):
        with torch.cuda.stream(cur):
            x.add_(1.0)
            ev = torch.cuda.Event()
            ev.record(cur)
        oth.wait_event(ev)
        cur, oth = oth, cur
    main.wait_stream(s1)


def chain_waits():
    main = torch.cuda.current_stream()
    s2.wait_stream(main)                 # fork s2 (idle) off the capture stream
    with torch.cuda.stream(s2):
        ev0 = torch.cuda.Event()
        ev0.record(s2)
    for _ in range(N):
        main.wait_event(ev0)
        x.add_(1.0)
    main.wait_stream(s2)


y = torch.zeros(1024, device=dev)


def chain_single2():
    for _ in range(N):
        x.add_(1.0)
        y.add_(1.0)


def chain_forkjoin():
    # per iteration: fork (x on the capture stream, y on s1 concurrently), then join before the next
    main = torch.cuda.current_stream()
    for _ in range(N):
        s1.wait_stream(main)
        x.add_(1.0)
        with torch.cuda.stream(s1):
            y.add_(1.0)
        main.wait_stream(s1)


def replay_us(body, reps=50):
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        if body is chain_pingpong:
            s1.wait_stream(torch.cuda.current_stream())
        body()
    g.replay()
    torch.cuda.synchronize()
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0.record()
    for _ in range(reps):
        g.replay()
    t1.record()
    torch.cuda.synchronize()
    return t0.elapsed_time(t1) * 1e3 / reps


res = {"kernels": N}
for name, body in (("single_stream", chain_single), ("alternating_streams", chain_pingpong),
                   ("single_with_event_waits", chain_waits), ("single_two_per_step", chain_single2),
                   ("fork_join_two_per_step", chain_forkjoin)):
    us = replay_us(body)
    res[name + "_us"] = round(us, 2)
    res[name + "_us_per_kernel"] = round(us / N, 3)
res["hop_cost_us"] = round(res["alternating_streams_us_per_kernel"] - res["single_stream_us_per_kernel"], 3)
res["fork_join_cost_us_per_step"] = round(res["fork_join_two_per_step_us_per_kernel"] - res["single_two_per_step_us_per_kernel"], 3)
print(json.dumps(res))
