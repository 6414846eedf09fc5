"""The resident host-call engine (engine.cpp, gf_engine in kernels.hip):
small synchronous host calls served through a doorbell in host memory.
Every result is compared with the CPU oracle (rs_oracle.c restating rs.go)
and with the same call made with the engine off (one launch per call)."""
import threading
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_dev():
    import torch

    assert torch.cuda.is_available()
    torch.cuda.init()
    return torch


@pytest.fixture
def engine(rslib):
    """Engine on with default settings; restored afterwards."""
    L = rslib.lib()
    assert L.rs_tune(b"host_engine", 1) == 0
    yield L
    L.rs_tune(b"host_engine", 1)
    L.rs_tune(b"host_engine_waves", 8)
    L.rs_tune(b"host_engine_idle_us", 200)
    L.rs_tune(b"host_engine_max_bytes", 128 << 10)


def _rand(rng, n):
    return rng.integers(0, 256, n, dtype=np.uint8)


@pytest.mark.parametrize("waves", [8, 1, 16])
def test_engine_calls_vs_oracle(rslib, orc, torch_dev, engine, waves):
    """Encode / Reconst / Update / Replace host calls of many shapes and sizes
    (tails, 8 KiB, 128 KiB; up to 8 output rows and 32 columns through the
    engine, larger shapes through the launch path) against the oracle."""
    assert engine.rs_tune(b"host_engine_waves", waves) == 0
    rng = np.random.default_rng(50 + waves)
    for d, p in [(10, 4), (12, 4), (6, 3), (8, 8), (20, 4), (32, 8), (3, 1), (40, 10)]:
        r = rslib.New(d, p)
        for size in (1, 17, 255, 1024, 4097, 8192, 131072):
            data = [_rand(rng, size) for _ in range(d)]
            v = [x.copy() for x in data] + [np.full(size, 0xA5, np.uint8) for _ in range(p)]
            r.Encode(v)
            exp = [x.copy() for x in data] + [np.zeros(size, np.uint8) for _ in range(p)]
            assert orc.encode(d, p, exp) == 0
            for j in range(d, d + p):
                assert np.array_equal(v[j], exp[j]), ("encode", d, p, size, j)
            lost = sorted(int(x) for x in rng.choice(d + p, min(p, 4), replace=False))
            w = [x.copy() for x in exp]
            for i in lost:
                w[i][:] = 0x11
            r.Reconst(w, [], lost)
            for i in range(d + p):
                assert np.array_equal(w[i], exp[i]), ("reconst", d, p, size, lost, i)
            row = int(rng.integers(0, d))
            new = _rand(rng, size)
            act = [x.copy() for x in exp]
            r.Update(act[row], new, row, act[d:])
            ref = [x.copy() for x in exp]
            ref[row] = new.copy()
            assert orc.encode(d, p, ref) == 0
            q = orc.update_quirk_range(size)
            for j in range(d, d + p):
                assert np.array_equal(act[j], ref[j]), ("update", d, p, size, j, q)
            rows = sorted(int(x) for x in rng.choice(d, min(d, 3), replace=False))
            delta = [_rand(rng, size) for _ in rows]
            act = [x.copy() for x in exp]
            r.Replace([x.copy() for x in delta], rows, act[d:])
            ref = [x.copy() for x in exp]
            for k, rr in enumerate(rows):
                ref[rr] = np.bitwise_xor(ref[rr], delta[k])
            assert orc.encode(d, p, ref) == 0
            for j in range(d, d + p):
                assert np.array_equal(act[j], ref[j]), ("replace", d, p, size, rows, j)
        calls, launches = r.host_engine_stats()
        if p <= 8 and d <= 32:
            assert calls > 0 and launches >= 1, (d, p, calls, launches)


def test_engine_idle_relaunch(rslib, orc, torch_dev, engine):
    """With a short idle window the engine leaves between spaced calls and a
    new instance serves the next one; bursts share one instance."""
    assert engine.rs_tune(b"host_engine_idle_us", 50) == 0
    d, p, size = 10, 4, 8192
    r = rslib.New(d, p)
    rng = np.random.default_rng(7)
    data = [_rand(rng, size) for _ in range(d)]
    exp = [x.copy() for x in data] + [np.zeros(size, np.uint8) for _ in range(p)]
    assert orc.encode(d, p, exp) == 0
    for k in range(6):
        v = [x.copy() for x in data] + [np.zeros(size, np.uint8) for _ in range(p)]
        r.Encode(v)
        assert all(np.array_equal(v[j], exp[j]) for j in range(d, d + p)), k
        time.sleep(0.005)
    calls, launches = r.host_engine_stats()
    assert calls == 6 and launches == 6, (calls, launches)
    assert engine.rs_tune(b"host_engine_idle_us", 100000) == 0
    for k in range(50):  # a burst: one instance
        v = [x.copy() for x in data] + [np.zeros(size, np.uint8) for _ in range(p)]
        r.Encode(v)
        assert all(np.array_equal(v[j], exp[j]) for j in range(d, d + p)), k
    calls2, launches2 = r.host_engine_stats()
    assert calls2 == 56 and launches2 == launches + 1, (calls2, launches2)
    assert engine.rs_tune(b"host_engine_idle_us", 200) == 0


def test_engine_concurrent_threads_and_torch_sync(rslib, orc, torch_dev, engine):
    """16 threads of mixed host calls on one handle (coalesced batches through
    the engine), every result checked; then a device-wide torch sync right
    after a call returns promptly (the engine leaves within its idle window)."""
    torch = torch_dev
    d, p = 10, 4
    r = rslib.New(d, p)
    errors = []

    def worker(tid):
        rng = np.random.default_rng(1000 + tid)
        try:
            for it in range(40):
                size = int(rng.choice([8192, 8192, 4096 + 3, 65536]))
                data = [_rand(rng, size) for _ in range(d)]
                exp = [x.copy() for x in data] + [np.zeros(size, np.uint8) for _ in range(p)]
                assert orc.encode(d, p, exp) == 0
                v = [x.copy() for x in data] + [np.zeros(size, np.uint8) for _ in range(p)]
                if tid % 2:
                    v = [x.copy() for x in exp]
                    lost = [1, 12]
                    for i in lost:
                        v[i][:] = 0
                    r.Reconst(v, [], lost)
                else:
                    r.Encode(v)
                for j in range(d + p):
                    if not np.array_equal(v[j], exp[j]):
                        errors.append((tid, it, size, j))
                        return
        except Exception as e:  # noqa: BLE001
            errors.append((tid, repr(e)))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(16)]
    for t in th:
        t.start()
    for t in th:
        t.join(120)
    assert not errors, errors[:5]
    calls, _ = r.host_engine_stats()
    assert calls > 0
    v = [np.zeros(8192, np.uint8) for _ in range(d + p)]
    r.Encode(v)
    t0 = time.perf_counter()
    torch.cuda.synchronize()
    assert time.perf_counter() - t0 < 0.5


def test_engine_on_off_identical(rslib, torch_dev, engine):
    """Engine on and off give the same bytes (8 rows, 32 columns, accumulate)."""
    rng = np.random.default_rng(3)
    for d, p, size in [(32, 8, 8192 + 5), (10, 4, 8192), (16, 6, 100000)]:
        r = rslib.New(d, p)
        data = [_rand(rng, size) for _ in range(d)]
        outs = []
        for on in (1, 0):
            assert engine.rs_tune(b"host_engine", on) == 0
            v = [x.copy() for x in data] + [np.zeros(size, np.uint8) for _ in range(p)]
            r.Encode(v)
            par = [x.copy() for x in v[d:]]
            r.Update(v[5], data[0], 5, par)
            outs.append((v[d:], par))
        for a, b in zip(outs[0][0] + outs[0][1], outs[1][0] + outs[1][1]):
            assert np.array_equal(a, b), (d, p, size)
