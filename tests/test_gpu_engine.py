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
    """Engine on with default settings, except that a call after a quiet
    period waits for the relaunch instead of taking the launch path (these
    tests count engine calls; test_engine_idle_relaunch and
    test_engine_cold_launch_concurrent cover that path); restored afterwards."""
    L = rslib.lib()
    assert L.rs_tune(b"host_engine", 1) == 0
    assert L.rs_tune(b"host_engine_cold_launch", 0) == 0
    yield L
    L.rs_tune(b"host_engine", 1)
    L.rs_tune(b"host_engine_waves", 8)
    L.rs_tune(b"host_engine_group_waves", 8)
    L.rs_tune(b"host_engine_idle_us", 2000)
    L.rs_tune(b"host_engine_life_us", 4000)
    L.rs_tune(b"host_engine_max_bytes", 1 << 20)
    L.rs_tune(b"host_engine_wg_units", 0)
    L.rs_tune(b"host_engine_direct", 1)
    L.rs_tune(b"host_engine_cold_launch", 1)


def _rand(rng, n):
    return rng.integers(0, 256, n, dtype=np.uint8)


@pytest.mark.parametrize("waves,group_waves,max_bytes,wg_units", [(8, 8, 1 << 20, 0), (1, 1, 1 << 20, 0),
                                                                 (16, 2, 128 << 10, 0), (3, 8, 8 << 20, 0),
                                                                 (8, 8, 1 << 20, 64), (5, 4, 1 << 20, 1000)])
def test_engine_calls_vs_oracle(rslib, orc, torch_dev, engine, waves, group_waves, max_bytes, wg_units):
    """Encode / Reconst / Update / Replace host calls of many shapes and sizes
    (tails, 8 KiB, 128 KiB; up to 8 output rows and 32 columns through the
    engine, larger shapes through the launch path) against the oracle, with
    the engine's workgroups, waves per workgroup and batch limit varied."""
    assert engine.rs_tune(b"host_engine_waves", waves) == 0
    assert engine.rs_tune(b"host_engine_group_waves", group_waves) == 0
    assert engine.rs_tune(b"host_engine_max_bytes", max_bytes) == 0
    assert engine.rs_tune(b"host_engine_wg_units", wg_units) == 0
    rng = np.random.default_rng(50 + waves + group_waves + wg_units)
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


@pytest.mark.parametrize("cold_launch", [1, 0])
def test_engine_idle_relaunch(rslib, orc, torch_dev, engine, cold_launch):
    """With a short idle window the engine leaves between spaced calls.
    cold_launch=1 (default): a call that finds it gone is served by the
    launch path and the engine restarts behind it, so only the first call
    rides the engine and every call starts an instance; cold_launch=0: a new
    instance serves each call.  Bursts share one instance either way."""
    assert engine.rs_tune(b"host_engine_idle_us", 50) == 0
    assert engine.rs_tune(b"host_engine_cold_launch", cold_launch) == 0
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
    assert calls == (1 if cold_launch else 6) and launches == 6, (cold_launch, calls, launches)
    assert engine.rs_tune(b"host_engine_idle_us", 100000) == 0
    assert engine.rs_tune(b"host_engine_life_us", 1000000) == 0
    for k in range(50):  # a burst: one instance
        v = [x.copy() for x in data] + [np.zeros(size, np.uint8) for _ in range(p)]
        r.Encode(v)
        assert all(np.array_equal(v[j], exp[j]) for j in range(d, d + p)), k
    calls2, launches2 = r.host_engine_stats()
    assert calls2 == calls + 50 and launches2 == launches + 1, (calls2, launches2)
    assert engine.rs_tune(b"host_engine_idle_us", 2000) == 0


def test_engine_waves_changed_on_live_handle(rslib, orc, torch_dev, engine):
    """host_engine_waves raised (and lowered) on a handle that has made more
    calls than the ring has slots: workgroups the old instance did not have
    start at the new instance's first call, so the next calls neither stall
    nor time out (advisor finding, engine.cpp slot-reuse wait)."""
    d, p, size = 10, 4, 8192
    r = rslib.New(d, p)
    rng = np.random.default_rng(71)
    data = [_rand(rng, size) for _ in range(d)]
    exp = [x.copy() for x in data] + [np.zeros(size, np.uint8) for _ in range(p)]
    assert orc.encode(d, p, exp) == 0
    for waves in (8, 16, 2, 64, 8):
        assert engine.rs_tune(b"host_engine_waves", waves) == 0
        for k in range(20):  # more calls than kEngineSlots (8) per setting
            v = [x.copy() for x in data] + [np.zeros(size, np.uint8) for _ in range(p)]
            t0 = time.perf_counter()
            r.Encode(v)
            assert time.perf_counter() - t0 < 1.0, (waves, k)
            assert all(np.array_equal(v[j], exp[j]) for j in range(d, d + p)), (waves, k)
    calls, launches = r.host_engine_stats()
    assert calls == 100 and launches >= 5, (calls, launches)


def test_engine_lifetime_bounds_device_sync(rslib, orc, torch_dev, engine):
    """While another thread keeps the engine busy with calls, a device-wide
    synchronisation still returns: each instance leaves after
    host_engine_life_us and the next call relaunches it."""
    torch = torch_dev
    assert engine.rs_tune(b"host_engine_life_us", 2000) == 0
    assert engine.rs_tune(b"host_engine_idle_us", 100000) == 0
    d, p, size = 10, 4, 8192
    r = rslib.New(d, p)
    rng = np.random.default_rng(72)
    data = [_rand(rng, size) for _ in range(d)]
    exp = [x.copy() for x in data] + [np.zeros(size, np.uint8) for _ in range(p)]
    assert orc.encode(d, p, exp) == 0
    stop, errors, count = threading.Event(), [], [0]

    def caller():
        try:
            while not stop.is_set():
                v = [x.copy() for x in data] + [np.zeros(size, np.uint8) for _ in range(p)]
                r.Encode(v)
                if not all(np.array_equal(v[j], exp[j]) for j in range(d, d + p)):
                    errors.append("mismatch")
                count[0] += 1
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))

    th = threading.Thread(target=caller)
    th.start()
    try:
        time.sleep(0.05)
        worst = 0.0
        for _ in range(20):
            t0 = time.perf_counter()
            torch.cuda.synchronize()
            worst = max(worst, time.perf_counter() - t0)
            time.sleep(0.005)
    finally:
        stop.set()
        th.join(30)
    assert not th.is_alive() and not errors, errors[:3]
    calls, launches = r.host_engine_stats()
    assert count[0] > 20 and launches >= 2, (count[0], launches)
    assert worst < 0.1, worst


@pytest.mark.parametrize("direct", [1, 0])
def test_engine_concurrent_threads_and_torch_sync(rslib, orc, torch_dev, engine, direct):
    """16 threads of mixed host calls on one handle (each ringing the engine,
    or coalesced batches through it), every result checked; then a
    device-wide torch sync right after a call returns promptly (the engine
    leaves within its idle window)."""
    assert engine.rs_tune(b"host_engine_direct", direct) == 0
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


def _registered_arena(rslib, nvec, size):
    """nvec vectors of `size` bytes, 4 KiB apart, in one page-aligned range
    registered with rs_host_register (unregister the returned base)."""
    pitch = (size + 4095) // 4096 * 4096
    arena = np.zeros(nvec * pitch + 4096, np.uint8)  # an ordinary heap array (freed with base)
    off = (-arena.ctypes.data) % 4096
    base = arena[off: off + nvec * pitch]
    rslib.host_register(base.ctypes.data, base.nbytes)
    return base, [base[i * pitch: i * pitch + size] for i in range(nvec)]


def test_engine_address_mode_registered_memory(rslib, orc, torch_dev, engine):
    """Calls whose vectors all lie in registered memory run through the
    engine straight over the caller's bytes (address mode: one address per
    vector, up to 32 inputs + 8 outputs), Encode / Reconst / Update / Replace
    against the oracle; a size that is not a multiple of 16 takes the launch
    path with the same bytes."""
    rng = np.random.default_rng(91)
    for d, p, size in [(10, 4, 8192), (32, 8, 4096), (3, 1, 16), (12, 4, 65536), (10, 4, 8192 + 8)]:
        r = rslib.New(d, p)
        base, v = _registered_arena(rslib, d + p, size)
        try:
            c0, _ = r.host_engine_stats()
            data = [_rand(rng, size) for _ in range(d)]
            for i in range(d):
                v[i][:] = data[i]
            for j in range(d, d + p):
                v[j][:] = 0x5A
            r.Encode(v)
            c1, _ = r.host_engine_stats()
            assert c1 - c0 == (1 if size % 16 == 0 else 0), (d, p, size, c0, c1)
            exp = [x.copy() for x in data] + [np.zeros(size, np.uint8) for _ in range(p)]
            assert orc.encode(d, p, exp) == 0
            for j in range(d, d + p):
                assert np.array_equal(v[j], exp[j]), ("encode", d, p, size, j)
            lost = sorted(int(x) for x in rng.choice(d + p, min(p, 3), replace=False))
            for i in lost:
                v[i][:] = 0
            r.Reconst(v, [], lost)
            for i in range(d + p):
                assert np.array_equal(v[i], exp[i]), ("reconst", d, p, size, lost, i)
            row = int(rng.integers(0, d))
            new = _rand(rng, size)
            old = v[row].copy()
            v[row][:] = new
            r.Update(old, v[row], row, v[d:])
            ref = [x.copy() for x in exp]
            ref[row] = new.copy()
            assert orc.encode(d, p, ref) == 0
            for j in range(d, d + p):
                assert np.array_equal(v[j], ref[j]), ("update", d, p, size, j)
            rows = sorted(int(x) for x in rng.choice(d, min(d, 2), replace=False))
            deltas = [_rand(rng, size) for _ in rows]
            r.Replace(deltas, rows, v[d:])
            for k, rr in enumerate(rows):
                ref[rr] = np.bitwise_xor(ref[rr], deltas[k])
            assert orc.encode(d, p, ref) == 0
            for j in range(d, d + p):
                assert np.array_equal(v[j], ref[j]), ("replace", d, p, size, rows, j)
        finally:
            rslib.host_unregister(base.ctypes.data)


def test_engine_address_mode_concurrent(rslib, orc, torch_dev, engine):
    """8 threads, each with its own registered stripe, Encode through the
    engine's address mode concurrently on one handle (calls serialise on the
    engine); every result checked."""
    d, p, size = 10, 4, 8192
    r = rslib.New(d, p)
    errors = []

    def worker(tid):
        rng = np.random.default_rng(300 + tid)
        base, v = _registered_arena(rslib, d + p, size)
        try:
            for it in range(30):
                data = [_rand(rng, size) for _ in range(d)]
                for i in range(d):
                    v[i][:] = data[i]
                r.Encode(v)
                exp = [x.copy() for x in data] + [np.zeros(size, np.uint8) for _ in range(p)]
                assert orc.encode(d, p, exp) == 0
                for j in range(d, d + p):
                    if not np.array_equal(v[j], exp[j]):
                        errors.append((tid, it, j))
                        return
        except Exception as e:  # noqa: BLE001
            errors.append((tid, repr(e)))
        finally:
            rslib.host_unregister(base.ctypes.data)

    th = [threading.Thread(target=worker, args=(t,)) for t in range(8)]
    for t in th:
        t.start()
    for t in th:
        t.join(120)
    assert not errors, errors[:5]
    calls, _ = r.host_engine_stats()
    assert calls >= 8 * 30


def test_engine_relaunch_under_concurrent_calls(rslib, orc, torch_dev, engine):
    """A 20 us idle window with 8 threads making calls at random intervals:
    workgroups leave while other threads' calls are in flight or about to be
    rung, and new instances resume them.  Every result is checked; no call
    is lost or computed twice (Update XORs into its parity)."""
    assert engine.rs_tune(b"host_engine_idle_us", 20) == 0
    d, p, size = 10, 4, 4096
    r = rslib.New(d, p)
    errors = []

    def worker(tid):
        rng = np.random.default_rng(700 + tid)
        base, v = _registered_arena(rslib, d + p, size)
        try:
            data = [_rand(rng, size) for _ in range(d)]
            for i in range(d):
                v[i][:] = data[i]
            r.Encode(v)
            for it in range(40):
                row = int(rng.integers(0, d))
                new = _rand(rng, size)
                old = v[row].copy()
                v[row][:] = new
                data[row] = new
                if tid % 2:
                    r.Update(old, v[row], row, v[d:])  # pageable old: coalesced batch path
                else:
                    r.Encode(v)  # registered: address mode
                exp = [x.copy() for x in data] + [np.zeros(size, np.uint8) for _ in range(p)]
                assert orc.encode(d, p, exp) == 0
                for j in range(d, d + p):
                    if not np.array_equal(v[j], exp[j]):
                        errors.append((tid, it, j))
                        return
                if rng.random() < 0.3:
                    time.sleep(float(rng.random()) * 0.0005)
        except Exception as e:  # noqa: BLE001
            errors.append((tid, repr(e)))
        finally:
            rslib.host_unregister(base.ctypes.data)

    th = [threading.Thread(target=worker, args=(t,)) for t in range(8)]
    for t in th:
        t.start()
    for t in th:
        t.join(120)
    assert not errors, errors[:5]
    calls, launches = r.host_engine_stats()
    assert calls > 0 and launches > 1, (calls, launches)


def test_engine_drain_before_stop(rslib, orc, torch_dev, engine):
    """Calls in flight when the instance is stopped for something other than a
    same-shape relaunch complete on their own shape (advisor finding, round 3:
    a workgroup that left at its life / idle limit before a call reached it,
    followed by a table-registry recycle or a shape change, used to have its
    done word raised past the call, which then returned with that
    workgroup's units never written).  Six threads of host Encode / Update
    calls with 100 us instance lives and a 20 us idle window, while one thread
    forces registry recycles (a 4-entry registry and device products over
    fresh matrices on the same handle) and another flips the engine's
    workgroup count and waves per workgroup.  Every host result is checked
    against the oracle and every device product against encode_numpy."""
    torch = torch_dev
    assert engine.rs_tune(b"host_engine_life_us", 100) == 0
    assert engine.rs_tune(b"host_engine_idle_us", 20) == 0
    L = engine
    assert L.rs_tune(b"table_registry_max", 4) == 0
    d, p, size = 10, 4, 8192
    r = rslib.New(d, p)
    errors, stop = [], threading.Event()

    def caller(tid):
        rng = np.random.default_rng(900 + tid)
        try:
            for it in range(60):
                data = [_rand(rng, size) for _ in range(d)]
                exp = [x.copy() for x in data] + [np.zeros(size, np.uint8) for _ in range(p)]
                assert orc.encode(d, p, exp) == 0
                v = [x.copy() for x in data] + [np.full(size, 0xA5, np.uint8) for _ in range(p)]
                r.Encode(v)
                if tid % 2:
                    row = int(rng.integers(0, d))
                    new = _rand(rng, size)
                    r.Update(v[row].copy(), new, row, v[d:])
                    v[row][:] = new
                    exp[row] = new.copy()
                    assert orc.encode(d, p, exp) == 0
                for j in range(d, d + p):
                    if not np.array_equal(v[j], exp[j]):
                        errors.append(("host", tid, it, j))
                        return
        except Exception as e:  # noqa: BLE001
            errors.append(("host", tid, repr(e)))

    def recycler():
        rng = np.random.default_rng(990)
        try:
            src = torch.randint(0, 256, (2, 6, 4096), dtype=torch.uint8, device="cuda:0")
            dst = torch.zeros((2, 3, 4096), dtype=torch.uint8, device="cuda:0")
            hsrc = src.cpu().numpy()
            while not stop.is_set():
                mat = rng.integers(0, 256, (3, 6), dtype=np.uint8)
                r.gf_matmul_batch(mat, src, None, dst, None)
                torch.cuda.synchronize()
                if not np.array_equal(dst.cpu().numpy(), orc.encode_numpy(mat, hsrc)):
                    errors.append(("device product", mat.tolist()))
                    return
        except Exception as e:  # noqa: BLE001
            errors.append(("recycler", repr(e)))

    def shaper():
        k = 0
        while not stop.is_set():
            L.rs_tune(b"host_engine_waves", (8, 4, 16, 8)[k % 4])
            L.rs_tune(b"host_engine_group_waves", (8, 2, 4, 8)[k % 4])
            k += 1
            time.sleep(0.002)

    callers = [threading.Thread(target=caller, args=(t,)) for t in range(6)]
    aux = [threading.Thread(target=recycler), threading.Thread(target=shaper)]
    try:
        for t in aux + callers:
            t.start()
        for t in callers:
            t.join(120)
    finally:
        stop.set()
        for t in aux:
            t.join(60)
        L.rs_tune(b"table_registry_max", 1 << 14)
    assert not any(t.is_alive() for t in callers + aux)
    assert not errors, errors[:5]
    calls, launches = r.host_engine_stats()
    assert calls >= 6 * 60 and launches > 2, (calls, launches)


def test_engine_cold_launch_concurrent(rslib, orc, torch_dev, engine):
    """The default cold path under concurrency: 8 threads call Encode /
    Update on one handle with random pauses, some longer than the engine's
    idle window, so calls after a quiet period take the launch path while the
    engine restarts behind them and the others ride the engine; every result
    against the oracle, and both paths were taken."""
    assert engine.rs_tune(b"host_engine_cold_launch", 1) == 0
    assert engine.rs_tune(b"host_engine_idle_us", 300) == 0
    d, p, size = 10, 4, 8192
    r = rslib.New(d, p)
    errors = []
    per = 25
    sync = threading.Barrier(8, timeout=60)

    def worker(tid):
        rng = np.random.default_rng(700 + tid)
        try:
            for it in range(per):
                if it % 5 == 0:  # every thread quiet at once for > the idle window, then all call
                    sync.wait()
                    time.sleep(0.002)
                data = [_rand(rng, size) for _ in range(d)]
                v = [x.copy() for x in data] + [np.zeros(size, np.uint8) for _ in range(p)]
                r.Encode(v)
                exp = [x.copy() for x in data] + [np.zeros(size, np.uint8) for _ in range(p)]
                assert orc.encode(d, p, exp) == 0
                if any(not np.array_equal(v[j], exp[j]) for j in range(d, d + p)):
                    errors.append((tid, it, "encode"))
                row = it % d
                new = _rand(rng, size)
                par = [x.copy() for x in v[d:]]
                r.Update(v[row], new, row, par)
                data[row] = new
                exp2 = [x.copy() for x in data] + [np.zeros(size, np.uint8) for _ in range(p)]
                assert orc.encode(d, p, exp2) == 0
                if any(not np.array_equal(par[j], exp2[d + j]) for j in range(p)):
                    errors.append((tid, it, "update"))
        except Exception as e:  # noqa: BLE001
            errors.append((tid, repr(e)))
            sync.abort()

    th = [threading.Thread(target=worker, args=(t,)) for t in range(8)]
    for t in th:
        t.start()
    for t in th:
        t.join(120)
    assert not any(t.is_alive() for t in th)
    assert not errors, errors[:5]
    calls, launches = r.host_engine_stats()
    assert 0 < calls < 8 * per * 2, (calls, launches)  # some calls rode the engine, some the launch path
    assert launches >= 2, (calls, launches)
