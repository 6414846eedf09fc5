"""Host memory handed to the library: rs_host_register / rs_host_unregister
(page spans shared by reference, device drain before a span leaves the
runtime) and the library-owned pool (rs_host_alloc / rs_host_free).

The reference's callers reuse their buffers freely (rs.go:101-111 retains
nothing), so the supported API must allow register -> unregister -> free ->
reuse of ordinary heap memory: the tests below register plain numpy heap
arrays (whose edge pages neighbouring heap objects share) and mappings they
unmap afterwards, and after every unregister ask both runtime layers
(tests/hip_ptr.py: hipPointerGetAttributes, hsa_amd_pointer_info) that no page
the library released is still registered.  Every result is checked against
the oracle (rs_oracle.c)."""
import os
import subprocess
import sys

import numpy as np
import pytest

import hip_ptr

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def torch_dev():
    import torch

    assert torch.cuda.is_available()
    torch.cuda.init()
    return torch


def _encode_ok(orc, r, d, p, v, rng):
    size = v[0].size
    for i in range(d):
        v[i][:] = rng.integers(0, 256, size, dtype=np.uint8)
    for j in range(d, d + p):
        v[j][:] = 0xA5
    r.Encode(v)
    exp = orc.encode_numpy(orc.gen_matrix(d, p).reshape(p, d), np.stack([x.copy() for x in v[:d]])[None])[0]
    return all(np.array_equal(v[d + j], exp[j]) for j in range(p))


def test_register_free_reuse_sequence_in_child(rslib, orc):
    """register -> host call -> unregister -> free -> reallocate -> pageable
    copy -> host call, in the two patterns round 3's tests used (page-aligned
    interior of a heap array; whole heap arrays sharing pages), then the
    library-owned pool in the same loop.  Run in a child process
    (tools/reg_reuse_probe.py), so a fault would end only that process."""
    env = dict(os.environ, RSAMD_PROBE_ITERS="12")
    out = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "tools", "reg_reuse_probe.py"), "lib",
                          "unaligned", "pool"], env=env, capture_output=True, text=True, timeout=400)
    print(out.stdout, out.stderr[-2000:])
    assert out.returncode == 0, out.stdout + out.stderr[-2000:]
    assert out.stdout.count(": exit 0") == 3, out.stdout


def test_registrations_sharing_pages(rslib, orc, torch_dev):
    """Two buffers that share a page registered one after the other: the
    second takes a reference on the shared page's span (a registration's
    partial edge pages are spans of their own) and registers only the pages no
    span covers; a's vectors that run over its edge-page spans stay zero-copy;
    unregistering the first leaves the second
    zero-copy (its host calls run straight over it, never through the
    coalesced staging path) and correct; the span leaves the runtime with the
    last registration, after which the same vectors are staged."""
    d, p, size = 10, 4, 4096
    L = rslib.lib()
    assert L.rs_tune(b"host_engine_direct", 0) == 0  # staged calls counted by host_call_stats
    try:
        r = rslib.New(d, p)
        rng = np.random.default_rng(11)
        spans0 = rslib.host_pool_stats()["spans"]
        arena = np.zeros(2 * (d + p) * size + 3 * 4096, np.uint8)  # an ordinary heap array
        off = (-arena.ctypes.data) % 4096 + 16  # a starts 16 bytes into a page
        a = arena[off: off + (d + p) * size]  # ends 16 bytes into its last page
        b = arena[off + a.nbytes: off + a.nbytes + 4080 + (d + p) * size]  # starts in that page
        va = [a[i * size:(i + 1) * size] for i in range(d + p)]
        vb = [b[4080 + i * size: 4080 + (i + 1) * size] for i in range(d + p)]  # b's vectors: its own pages
        rslib.host_register(a.ctypes.data, a.nbytes)
        rslib.host_register(b.ctypes.data, b.nbytes)
        # a: its partial first and last pages as spans of their own plus its
        # middle; b: a reference on a's last-page span plus its own pages
        assert rslib.host_pool_stats()["spans"] - spans0 == 4
        with pytest.raises(rslib.ErrInvalidArgument):
            rslib.host_register(a.ctypes.data, a.nbytes)  # same address twice

        def staged():
            return r.host_call_stats()[1]

        s0 = staged()
        assert _encode_ok(orc, r, d, p, va, rng) and _encode_ok(orc, r, d, p, vb, rng)
        assert staged() == s0  # both zero-copy
        rslib.host_unregister(a.ctypes.data)
        # only the shared page outlives a: b holds its one-page span
        assert rslib.host_pool_stats()["spans"] - spans0 == 2
        shared = (a.ctypes.data + a.nbytes) & ~4095
        assert hip_ptr.known_pages(a.ctypes.data, a.ctypes.data + a.nbytes, skip=(shared,)) == []
        assert hip_ptr.registered(shared)
        assert _encode_ok(orc, r, d, p, vb, rng)
        assert staged() == s0  # b still zero-copy
        assert _encode_ok(orc, r, d, p, va, rng)
        assert staged() == s0 + 1  # a staged now
        rslib.host_unregister(b.ctypes.data)
        assert rslib.host_pool_stats()["spans"] == spans0
        assert hip_ptr.known_pages(arena.ctypes.data, arena.ctypes.data + arena.nbytes) == []
        with pytest.raises(rslib.ErrInvalidArgument):
            rslib.host_unregister(b.ctypes.data)
        assert _encode_ok(orc, r, d, p, vb, rng)
        assert staged() == s0 + 2
    finally:
        L.rs_tune(b"host_engine_direct", 1)
    del va, vb, a, b, arena  # freed: the heap may hand these addresses out again


def test_pool_blocks_reused_and_zero_copy(rslib, orc, torch_dev):
    """rs_host_alloc blocks: host calls on them run straight over them (the
    engine's address mode), a freed block is handed out again without a new
    mapping, double frees and foreign pointers are refused, and pageable
    copies of fresh heap arrays in between stay correct."""
    torch = torch_dev
    d, p, size = 10, 4, 8192
    r = rslib.New(d, p)
    rng = np.random.default_rng(12)
    st0 = rslib.host_pool_stats()
    # (the copies between calls outlast the engine's idle window: keep the
    # engine serving such calls, so each call counts as an engine call)
    assert rslib.lib().rs_tune(b"host_engine_cold_launch", 0) == 0
    try:
        _pool_rounds(rslib, orc, torch, r, d, p, size, rng)
    finally:
        rslib.lib().rs_tune(b"host_engine_cold_launch", 1)
    st = rslib.host_pool_stats()
    assert st["blocks"] - st0["blocks"] <= 1 and st["in_use"] == st0["in_use"], (st0, st)
    with pytest.raises(rslib.ErrInvalidArgument):
        rslib.host_free(np.zeros(16, np.uint8).ctypes.data)


def _pool_rounds(rslib, orc, torch, r, d, p, size, rng):
    for it in range(6):
        buf = rslib.host_alloc((d + p) * size)
        assert buf.ctypes.data % 4096 == 0
        v = [buf[i * size:(i + 1) * size] for i in range(d + p)]
        c0, _ = r.host_engine_stats()
        assert _encode_ok(orc, r, d, p, v, rng), it
        c1, _ = r.host_engine_stats()
        assert c1 - c0 == 1, (it, c0, c1)
        addr = buf.ctypes.data
        del v
        rslib.host_free(buf)
        with pytest.raises(rslib.ErrInvalidArgument):
            rslib.host_free(addr)
        x = np.full(20 << 20, it, np.uint8)
        print(f"round {it}: pool block {addr:#x}, fresh array {x.ctypes.data:#x}-{x.ctypes.data + x.nbytes:#x}",
              flush=True)
        t = torch.from_numpy(x).cuda()
        torch.cuda.synchronize()
        assert int(t[-1].item()) == it


def _mapping_of(addr):
    """(start, end) of the /proc/self/maps entry holding addr."""
    with open("/proc/self/maps") as f:
        for line in f:
            lo, hi = (int(x, 16) for x in line.split()[0].split("-"))
            if lo <= addr < hi:
                return lo, hi
    return None


def test_pool_slabs_own_their_granules(rslib, torch_dev):
    """Pool blocks come from slabs of whole 2 MiB granules (KFD's SVM unit on
    MI355X): the mapping holding any block starts and ends on
    a 2 MiB boundary, so no other mapping (a caller's array the runtime maps
    in place for a pageable copy) shares a granule with registered pool
    memory; a small class's blocks are carved side by side from one slab."""
    g = 2 << 20
    blocks = [rslib.host_alloc(n) for n in (64 << 10, 64 << 10, 300 << 10, (3 << 20) + 1)]
    try:
        for b in blocks:
            m = _mapping_of(b.ctypes.data)
            assert m is not None and m[0] % g == 0 and m[1] % g == 0, (hex(b.ctypes.data), m)
        assert blocks[3].ctypes.data % g == 0  # a class of 4 MiB: a slab of its own
        x = np.full(20 << 20, 3, np.uint8)  # a fresh multi-MiB array mapped next to the pool
        t = torch_dev.from_numpy(x).cuda()
        torch_dev.cuda.synchronize()
        assert int(t[-1].item()) == 3
    finally:
        for b in blocks:
            rslib.host_free(b)


def test_concurrent_register_unregister_shared_pages(rslib, torch_dev):
    """Two threads register and unregister buffers that share pages (one
    mapping, the threads' ranges overlapping by half a page) 200 times each:
    no call fails.  An unregister holds the registry until the runtime has
    dropped its dead spans, so the other thread never asks the runtime to
    register pages it still holds."""
    import mmap
    import threading

    import reedsolomon_amd as rs

    page = mmap.PAGESIZE
    m = mmap.mmap(-1, 8 * page)
    base = np.frombuffer(m, dtype=np.uint8)
    views = [base[page // 2: 3 * page + page // 2], base[3 * page: 6 * page]]  # share the page at 3 * page
    errs = []

    def worker(v):
        try:
            for _ in range(200):
                rs.host_register(v.ctypes.data, v.nbytes)
                rs.host_unregister(v.ctypes.data)
        except Exception as e:  # noqa: BLE001
            errs.append(repr(e))

    th = [threading.Thread(target=worker, args=(v,)) for v in views]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs, errs[:3]
    assert hip_ptr.known_pages(base.ctypes.data, base.ctypes.data + base.nbytes) == []
    del views, base
    m.close()  # unmapped: the next mapping may land here


def _libc():
    import ctypes

    c = ctypes.CDLL(None, use_errno=True)
    c.mmap.restype = ctypes.c_void_p
    c.mmap.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_long]
    c.munmap.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    return c


def test_unregister_releases_pages_a_neighbour_does_not_share(rslib, orc, torch_dev):
    """Advisor round 4: A and B share one page; A is unregistered, A's own
    pages are unmapped and mapped afresh at the same addresses (what an
    allocator trim + regrow does), and a new buffer C registered there must
    get new pinning: its zero-copy host calls write the pages the CPU sees.
    Were A's whole span kept alive by B's reference, C would take that stale
    pinning and the parity would land in the old physical pages."""
    import ctypes

    c = _libc()
    PROT_RW, MAP_PRIV_ANON, MAP_FIXED = 0x3, 0x22, 0x10
    page = 4096
    npages = 24
    base = c.mmap(None, npages * page, PROT_RW, MAP_PRIV_ANON, -1, 0)
    assert base not in (None, ctypes.c_void_p(-1).value)
    d, p, size = 4, 2, 16 * 1024  # 6 vectors x 16 KiB = 24 pages
    r = rslib.New(d, p)
    rng = np.random.default_rng(5)
    try:
        a_lo, a_len = base + 64, 12 * page - 64 - 32  # A: pages 0..11, its last page shared with B
        b_lo, b_len = a_lo + a_len, 4 * page + 32  # B: from the end of A (inside page 11) on
        rslib.host_register(a_lo, a_len)
        rslib.host_register(b_lo, b_len)
        # A's host calls once, so its pages were used zero-copy
        arr = np.ctypeslib.as_array((ctypes.c_uint8 * (npages * page)).from_address(base))
        va = [arr[64 + i * 1024: 64 + (i + 1) * 1024] for i in range(d + p)]
        assert _encode_ok(orc, r, d, p, va, rng)
        rslib.host_unregister(a_lo)
        # A's own pages left both runtime layers; the page B shares did not
        assert hip_ptr.known_pages(base, base + 11 * page) == []
        assert hip_ptr.registered(base + 11 * page)
        # trim + regrow of A's exclusive pages 0..10: new physical pages, same addresses
        assert c.munmap(base, 11 * page) == 0
        got = c.mmap(base, 11 * page, PROT_RW, MAP_PRIV_ANON | MAP_FIXED, -1, 0)
        assert got == base
        # C: the fresh pages, page-aligned (no page shared with B)
        rslib.host_register(base, 11 * page)
        assert rslib.host_device_pointer(base, 11 * page)
        arr = np.ctypeslib.as_array((ctypes.c_uint8 * (11 * page)).from_address(base))
        vc = [arr[i * 4096: (i + 1) * 4096] for i in range(d + p)]
        for it in range(3):
            assert _encode_ok(orc, r, d, p, vc, rng), it
        rslib.host_unregister(base)
        rslib.host_unregister(b_lo)
        assert hip_ptr.known_pages(base, base + npages * page) == []
    finally:
        c.munmap(base, npages * page)


def test_unregister_does_not_wait_out_engine_idle(rslib, orc, torch_dev):
    """An unregister after a host call asks the resident engine to leave
    instead of draining behind its idle window (advisor round 4): with the
    idle window raised to 50 ms, register -> Encode -> unregister takes far
    less than 50 ms, and the next call (engine relaunched) is still correct."""
    import time

    d, p, size = 10, 4, 8192
    L = rslib.lib()
    assert L.rs_tune(b"host_engine_idle_us", 50000) == 0
    try:
        r = rslib.New(d, p)
        rng = np.random.default_rng(21)
        buf = np.zeros((d + p) * size + 4096, np.uint8)  # an ordinary heap array
        off = (-buf.ctypes.data) % 4096
        v = [buf[off + i * size: off + (i + 1) * size] for i in range(d + p)]
        times = []
        for it in range(5):
            rslib.host_register(buf[off:].ctypes.data, (d + p) * size)
            assert _encode_ok(orc, r, d, p, v, rng), it
            t0 = time.perf_counter()
            rslib.host_unregister(buf[off:].ctypes.data)
            times.append(time.perf_counter() - t0)
            assert hip_ptr.known_pages(buf.ctypes.data, buf.ctypes.data + buf.nbytes) == [], it
            # the caller's whole pages are no longer GPU-mapped (KFD SVM, the revoke)
            assert hip_ptr.gpu_mapped_pages(buf[off:].ctypes.data, buf[off:].ctypes.data + (d + p) * size) == [], it
            assert _encode_ok(orc, r, d, p, v, rng), it  # pageable now
        print("unregister ms", [round(x * 1e3, 3) for x in times])
        assert sorted(times)[2] < 0.02, times
    finally:
        L.rs_tune(b"host_engine_idle_us", 2000)


def test_host_calls_proceed_during_unregister_drain(rslib, orc, torch_dev):
    """rs_host_unregister drains the devices without holding the registry:
    host calls on another registered buffer keep running (and stay correct)
    while a second thread registers / unregisters an ordinary heap array in a
    loop.  Then the round-5 fault's sequence: the array is freed, arrays of
    the sizes the next test allocated (tests/test_gpu_jit.py::_padded, the
    1.3 MB copy that failed) are allocated and copied to the device through
    the runtime's pageable path, every byte checked, with no page of them
    still registered beforehand."""
    import threading

    torch = torch_dev
    d, p, size = 10, 4, 8192
    r = rslib.New(d, p)
    keep = rslib.host_alloc((d + p) * size)
    vk = [keep[i * size:(i + 1) * size] for i in range(d + p)]
    churn = np.zeros(64 * 4096, np.uint8)  # an ordinary heap array
    stop = threading.Event()
    errs = []

    def churner():
        try:
            while not stop.is_set():
                rslib.host_register(churn.ctypes.data, churn.nbytes)
                rslib.host_unregister(churn.ctypes.data)
        except Exception as e:  # noqa: BLE001
            errs.append(repr(e))

    t = threading.Thread(target=churner)
    t.start()
    try:
        rng = np.random.default_rng(3)
        for it in range(200):
            if not _encode_ok(orc, r, d, p, vk, rng):
                errs.append(("mismatch", it))
                break
    finally:
        stop.set()
        t.join(60)
    rslib.host_free(keep)
    assert not errs, errs[:3]
    lo, hi = churn.ctypes.data, churn.ctypes.data + churn.nbytes
    assert hip_ptr.known_pages(lo, hi) == []
    assert hip_ptr.gpu_mapped_pages(lo, hi) == []  # (KFD SVM: the caller's whole pages revoked)
    del churn
    rng = np.random.default_rng(510)
    for shape in [(3, 10, 16), (2, 10, 2064), (3, 10, 4112), (2, 10, 65632), (2, 5, 65632), (2, 10, (1 << 20) + 16),
                  (64 * 4096,)]:
        host = rng.integers(0, 256, shape, dtype=np.uint8)
        assert hip_ptr.known_pages(host.ctypes.data, host.ctypes.data + host.nbytes) == [], shape
        dev = torch.from_numpy(host).cuda()
        torch.cuda.synchronize()
        assert np.array_equal(dev.cpu().numpy(), host), shape


def test_unregister_revokes_gpu_mapping(rslib, torch_dev):
    """hipHostRegister grants the GPU in-place access to the range through
    KFD's shared-virtual-memory ranges and hipHostUnregister leaves it
    (tools/ptr_state_probe.py): rs_host_unregister takes it back for the
    caller's whole pages, so memory the caller frees is not left GPU-mapped
    (each later trim of it by the allocator would have the kernel tear down a
    GPU mapping, evicting the process's queues).  A partial edge page keeps
    the runtime's state (a neighbour may be in a runtime copy); with
    host_unregister_revoke 0 the runtime's own behaviour shows."""
    L = rslib.lib()
    a = np.zeros(40 * 4096 + 123, np.uint8)  # an ordinary heap array, unaligned
    lo, hi = a.ctypes.data, a.ctypes.data + a.nbytes
    inner = ((lo + 4095) & ~4095) + 4096
    if hip_ptr.gpu_access(inner) == "unknown":
        pytest.skip("no ROCr SVM attribute API")
    # (no precondition on the pages: in a full run an earlier test's pageable
    # torch copy may have left this reused heap range GPU-mapped already; the
    # revoke below covers that case as well)
    rslib.host_register(lo, a.nbytes)
    assert hip_ptr.registered(inner) and hip_ptr.gpu_access(inner) == "in-place"
    rslib.host_unregister(lo)
    assert not hip_ptr.registered(inner)
    assert hip_ptr.gpu_mapped_pages(lo, hi) == []
    try:
        assert L.rs_tune(b"host_unregister_revoke", 0) == 0
        rslib.host_register(lo, a.nbytes)
        rslib.host_unregister(lo)
        assert not hip_ptr.registered(inner)
        assert hip_ptr.gpu_access(inner) == "in-place"  # the runtime's own unregister leaves the mapping
    finally:
        L.rs_tune(b"host_unregister_revoke", 1)
    rslib.host_register(lo, a.nbytes)  # registering again after a revoke works, and revokes again
    assert hip_ptr.gpu_access(inner) == "in-place"
    rslib.host_unregister(lo)
    assert hip_ptr.gpu_mapped_pages(lo, hi) == []

