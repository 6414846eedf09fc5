#!/usr/bin/env python3
"""Where the first launch after an idle sync loses time (bench.py's timed
region starts from an idle GPU): host time of one encode_batch_split call in
steady state and right after a sync, and the HIP-event time from a marker
recorded just before the first launch to the end of that launch, against the
same launch queued behind others.  10+4 @ 1 MiB x 256 stripes, as bench.py."""
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import reedsolomon_amd as rs  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    k, m, vec, S = 10, 4, 1 << 20, 256
    r = rs.New(k, m, device=0)
    data = torch.randint(0, 256, (S, k, vec), dtype=torch.uint8, device=dev)
    parity = torch.empty((S, m, vec), dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream(dev)

    def step():
        r.encode_batch_split(data, parity, stream=st)

    for _ in range(400):
        step()
    torch.cuda.synchronize()
    # host enqueue cost per call while the GPU is busy (queue not empty)
    host = []
    for _ in range(40):
        t = time.perf_counter()
        step()
        host.append((time.perf_counter() - t) * 1e6)
    torch.cuda.synchronize()
    print(f"host us per call, queue busy: median {statistics.median(host):.1f} max {max(host):.1f}", flush=True)
    # first launch after an idle sync
    first_host, first_ev, first_wall = [], [], []
    for _ in range(30):
        for _ in range(20):
            step()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record(st)
        step()
        t1 = time.perf_counter()
        e1.record(st)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        first_host.append((t1 - t0) * 1e6)
        first_ev.append(e0.elapsed_time(e1) * 1e3)
        first_wall.append((t2 - t0) * 1e6)
    # the same launch queued behind another (no idle gap)
    queued = []
    for _ in range(30):
        step()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        step()
        e1.record(st)
        torch.cuda.synchronize()
        queued.append(e0.elapsed_time(e1) * 1e3)
    med = statistics.median
    print(f"first launch after sync: host call {med(first_host):.1f} us, event pair {med(first_ev):.1f} us, "
          f"wall to sync {med(first_wall):.1f} us", flush=True)
    print(f"queued launch: event pair {med(queued):.1f} us", flush=True)
    print(f"idle-start cost: {med(first_ev) - med(queued):.1f} us (event pair), "
          f"{med(first_wall) - med(queued):.1f} us (wall)", flush=True)


if __name__ == "__main__":
    main()
