#!/usr/bin/env python3
"""Concurrency stress on one GPU: T threads for S seconds, random operations
on shared and private handles, every result checked against the CPU oracle.

    python tools/gpu_stress.py [threads=8] [seconds=90] [jit=policy|all]

jit=policy keeps the library's default compile policy (machine-code
networks once a matrix's launches would pay for one); jit=all compiles
every matrix on the launching thread at its first launch (rs_tune jit 2),
which with the random erasure sets below passes the 256-matrix cap and
exercises eviction under concurrent launches.

Mix per iteration (one of):
  host  - Go-API calls on pageable numpy vectors (Encode / Reconst / Update /
          Replace; 1 B - 200 KiB; shapes up to 20+8): the resident host-call
          engine, the coalescing and staging paths;
  dev   - device batch Encode + Reconst of 1..p lost (5-8 lost takes the
          run-time compiled kernels once they are ready; compiles start at the
          first sight of a matrix, jit_min_bytes 0);
  multi - multi-pattern Reconst with a different erasure set per stripe;
  wide  - (jit=policy) large device batches of wide rebuilds with a FRESH
          erasure pattern each time, sized so that one launch crosses the
          library's compile threshold (16+16 Reconst of 16 x 48 stripes @ 1 MiB,
          100+28 Reconst of 20 x 80 stripes @ 256 KiB): first-sight machine-code
          compiles from several threads at once under the shipped policy.
Handles are shared between threads for one shape per class, so concurrent
callers hit the same handle (rs.go's *RS is safe for concurrent use).
Prints one JSON line; exits 1 on any mismatch or error.
"""
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import reedsolomon_amd as rs  # noqa: E402
from oracle import oracle as orc  # noqa: E402  (checker only)

SHAPES = [(10, 4), (12, 4), (10, 8), (6, 3), (20, 8), (16, 8), (8, 6), (16, 16), (32, 24)]


def main():
    T = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    SECS = float(sys.argv[2]) if len(sys.argv) > 2 else 90.0
    MODE = sys.argv[3] if len(sys.argv) > 3 else "policy"
    orc.build()
    assert torch.cuda.is_available()
    if MODE == "all":  # compile every matrix on first sight: hammer the compile and eviction paths
        assert rs.lib().rs_tune(b"jit", 2) == 0
    shared = {s: rs.New(*s) for s in SHAPES}
    wide_shapes = [(16, 16, 1 << 20, 16, 48), (100, 28, 256 << 10, 20, 80)]  # d, p, size, lost, stripes
    for d, p, *_ in wide_shapes:
        shared[(d, p)] = rs.New(d, p)
    lock = threading.Lock()
    stats = {"host": 0, "dev": 0, "multi": 0, "wide": 0, "errors": []}
    t_end = time.time() + SECS

    def fail(msg):
        with lock:
            stats["errors"].append(msg)

    def host_op(rng, r, d, p):
        size = int(rng.choice([1, 15, 16, 100, 4096, 8192, 8192 + 5, 65536, 200000]))
        data = [rng.integers(0, 256, size, dtype=np.uint8) for _ in range(d)]
        enc = [x.copy() for x in data] + [np.zeros(size, np.uint8) for _ in range(p)]
        assert orc.encode(d, p, enc) == 0
        op = int(rng.integers(4))
        if op == 0:
            act = [x.copy() for x in data] + [np.full(size, 0xA5, np.uint8) for _ in range(p)]
            r.Encode(act)
            ok = all(np.array_equal(act[d + j], enc[d + j]) for j in range(p))
        elif op == 1:
            lost = sorted(int(v) for v in rng.choice(d + p, int(rng.integers(1, p + 1)), replace=False))
            act = [x.copy() for x in enc]
            for v in lost:
                act[v][:] = 0x3C
            r.Reconst(act, [v for v in range(d + p) if v not in lost], lost)
            ok = all(np.array_equal(act[v], enc[v]) for v in range(d + p))
        elif op == 2:
            row = int(rng.integers(d))
            new = rng.integers(0, 256, size, dtype=np.uint8)
            act = [x.copy() for x in enc]
            r.Update(act[row], new, row, act[d:])
            exp = [x.copy() for x in data] + [np.zeros(size, np.uint8) for _ in range(p)]
            exp[row] = new
            assert orc.encode(d, p, exp) == 0
            ok = all(np.array_equal(act[d + j], exp[d + j]) for j in range(p))
        else:
            rows = [int(v) for v in rng.choice(d, int(rng.integers(1, min(d, 6) + 1)), replace=False)]
            delta = [rng.integers(0, 256, size, dtype=np.uint8) for _ in rows]
            act = [x.copy() for x in enc]
            r.Replace(delta, rows, act[d:])
            exp = [x.copy() for x in data] + [np.zeros(size, np.uint8) for _ in range(p)]
            for k, rr in enumerate(rows):
                exp[rr] = exp[rr] ^ delta[k]
            assert orc.encode(d, p, exp) == 0
            ok = all(np.array_equal(act[d + j], exp[d + j]) for j in range(p))
        if not ok:
            fail(f"host op {op} {d}+{p} size {size}")

    def dev_op(rng, r, d, p, stream):
        S = int(rng.integers(1, 6))
        n = int(rng.choice([16, 4096 + 5, 65536, 262144 + 48]))
        G = orc.gen_matrix(d, p).reshape(p, d)
        host = rng.integers(0, 256, (S, d + p, n), dtype=np.uint8)
        host[:, d:] = orc.encode_numpy(G, host[:, :d])
        with torch.cuda.stream(stream):
            buf = torch.from_numpy(host).to("cuda", non_blocking=False)
            lost = sorted(int(v) for v in rng.choice(d + p, int(rng.integers(1, p + 1)), replace=False))
            buf[:, lost] = 0x77
            r.reconst_batch(buf, [], lost, stream=stream)
            stream.synchronize()
            got = buf.cpu().numpy()
        if not np.array_equal(got, host):
            fail(f"dev reconst {d}+{p} S {S} n {n} lost {lost}")

    def multi_op(rng, r, d, p, stream):
        S, n = int(rng.integers(2, 40)), int(rng.choice([1024, 8192, 65536]))
        G = orc.gen_matrix(d, p).reshape(p, d)
        hd = rng.integers(0, 256, (S, d, n), dtype=np.uint8)
        hp = orc.encode_numpy(G, hd)
        masks = np.zeros(S, np.uint64)
        for s in range(S):
            if rng.integers(5):
                lost = rng.choice(d + p, int(rng.integers(1, p + 1)), replace=False)
                masks[s] = sum(1 << int(v) for v in lost)
        with torch.cuda.stream(stream):
            data = torch.from_numpy(hd.copy()).cuda()
            par = torch.from_numpy(hp.copy()).cuda()
            for s in range(S):
                for v in range(d + p):
                    if (int(masks[s]) >> v) & 1:
                        (data[s, v] if v < d else par[s, v - d]).fill_(0xEE)
            r.reconst_batch_multi(data, par, masks, stream=stream)
            stream.synchronize()
            ok = np.array_equal(data.cpu().numpy(), hd) and np.array_equal(par.cpu().numpy(), hp)
        if not ok:
            fail(f"multi {d}+{p} S {S} n {n}")

    def wide_op(rng, stream):
        d, p, n, nl, S = wide_shapes[int(rng.integers(len(wide_shapes)))]
        r = shared[(d, p)]
        G = orc.gen_matrix(d, p).reshape(p, d)
        one = rng.integers(0, 256, (1, d + p, n), dtype=np.uint8)
        one[:, d:] = orc.encode_numpy(G, one[:, :d])  # the oracle's stripe, tiled S times on the GPU
        lost = sorted(int(v) for v in rng.choice(d + p, nl, replace=False))  # fresh pattern
        with torch.cuda.stream(stream):
            ref = torch.from_numpy(one).cuda().expand(S, d + p, n).contiguous()
            buf = ref.clone()
            buf[:, lost] = 0x5A
            r.reconst_batch(buf, [], lost, stream=stream)
            ok = bool(torch.equal(buf, ref))
            stream.synchronize()
            del buf, ref
        if not ok:
            fail(f"wide reconst {d}+{p} S {S} n {n} lost {lost}")

    def worker(i):
        rng = np.random.default_rng(1000 + i)
        stream = torch.cuda.Stream()
        private = {}
        while time.time() < t_end:
            d, p = SHAPES[int(rng.integers(len(SHAPES)))]
            if rng.integers(2):
                r = shared[(d, p)]
            else:
                r = private.setdefault((d, p), rs.New(d, p))
            kinds = ("host", "host", "dev", "multi") + (("wide",) if MODE == "policy" else ())
            kind = kinds[int(rng.integers(len(kinds)))]
            try:
                if kind == "wide":
                    wide_op(rng, stream)
                elif kind == "host":
                    host_op(rng, r, d, p)
                elif kind == "dev":
                    dev_op(rng, r, d, p, stream)
                else:
                    multi_op(rng, r, d, p, stream)
            except Exception as e:  # noqa: BLE001
                fail(f"{kind} {d}+{p}: {e!r}")
                return
            with lock:
                stats[kind] += 1

    th = [threading.Thread(target=worker, args=(i,)) for i in range(T)]
    for t in th:
        t.start()
    last = time.time()
    while any(t.is_alive() for t in th):
        time.sleep(0.5)
        if time.time() - last > 20:
            last = time.time()
            print(f"progress: {stats['host']} host, {stats['dev']} dev, {stats['multi']} multi, {stats['wide']} wide, "
                  f"{len(stats['errors'])} errors", flush=True)
    for t in th:
        t.join()
    out = {"threads": T, "seconds": SECS, "jit_mode": MODE, "host": stats["host"], "dev": stats["dev"], "multi": stats["multi"], "wide": stats["wide"],
           "errors": stats["errors"][:20], "jit": rs.jit_stats()}
    print(json.dumps(out), flush=True)
    sys.exit(1 if stats["errors"] else 0)


if __name__ == "__main__":
    main()
