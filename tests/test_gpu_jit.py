"""Run-time compiled bit-sliced kernels (jit.cpp): products with 5-16 output
rows over matrices known only at run time — the primitive (rs_gf_matmul_batch,
gmu.go:4-9 / encodePart rs.go:175-203), Reconst of 5-16 lost vectors
(rs.go:221-380), Update / Replace with 8 parity rows (rs.go:424-570) and the
Encode of codes without a build-time network (matrix.go:37-54) — compared
byte-for-byte with the CPU oracle.  rs_tune("jit", 2) compiles on the
launching thread, so every launch below runs the compiled kernel (the
counters say so); one test covers the default background compile.
"""
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
def jit_sync(rslib):
    L = rslib.lib()
    assert L.rs_tune(b"jit", 2) == 0
    yield
    L.rs_tune(b"jit", 1)
    L.rs_tune(b"jit_min_bytes", 8 << 20)


def _padded(torch, rng, S, v, n, pad):
    """[S, v, n] view of a [S, v, n + pad] device buffer (16-byte aligned rows
    when n + pad is, so the vector body runs and n % 16 bytes take the tail)."""
    host = rng.integers(0, 256, (S, v, n + pad), dtype=np.uint8)
    t = torch.from_numpy(host).cuda()
    return t[:, :, :n], host[:, :, :n]


@pytest.mark.parametrize("rows,cols", [(5, 10), (6, 10), (7, 12), (8, 10), (8, 16), (8, 32), (5, 1), (8, 3),
                                       (9, 10), (12, 16), (16, 16), (16, 32), (8, 64)])
def test_jit_matmul_vs_oracle(rslib, orc, torch_dev, jit_sync, rows, cols):
    torch = torch_dev
    rng = np.random.default_rng(rows * 100 + cols)
    mat = rng.integers(0, 256, (rows, cols), dtype=np.uint8)
    r = rslib.New(10, 4)
    before = rslib.jit_stats()["launches"]
    for S, n, pad in [(3, 16, 0), (2, 2048 + 16, 0), (3, 4096 + 5, 11), (2, 65536 + 96, 0), (2, (1 << 20) + 3, 13)]:
        src, hsrc = _padded(torch, rng, S, cols, n, pad)
        dst, hdst = _padded(torch, rng, S, rows, n, pad)
        r.gf_matmul_batch(mat, src, None, dst, None)
        torch.cuda.synchronize()
        assert np.array_equal(dst.cpu().numpy(), orc.encode_numpy(mat, hsrc)), (rows, cols, S, n)
        # accumulate (updateOnly): dst ^= mat x src
        dst2, hdst2 = _padded(torch, rng, S, rows, n, pad)
        r.gf_matmul_batch(mat, src, None, dst2, None, accumulate=True)
        torch.cuda.synchronize()
        assert np.array_equal(dst2.cpu().numpy(), hdst2 ^ orc.encode_numpy(mat, hsrc)), (rows, cols, S, n, "acc")
    st = rslib.jit_stats()
    # every aligned launch above, overwrite and XOR-accumulate, ran the compiled kernel
    assert st["launches"] >= before + 10, st
    assert st["failed"] == 0, st


@pytest.mark.parametrize("d,p,lost", [(10, 8, [0, 1, 2, 3, 4, 5, 6, 7]), (10, 8, [1, 3, 5, 7, 9]),
                                      (10, 8, [0, 2, 4, 11, 13, 17]), (10, 8, [12, 13, 14, 15, 16, 17]),
                                      (16, 8, [0, 3, 6, 9, 12, 15, 18, 21]), (20, 7, [2, 4, 6, 8, 10, 12, 14]),
                                      (20, 12, list(range(0, 24, 2))), (16, 16, list(range(16))),
                                      (40, 8, [1, 5, 9, 13, 17, 21, 33, 45])])
def test_jit_reconst_5_to_8_lost(rslib, orc, torch_dev, jit_sync, d, p, lost):
    """Reconst of 5-16 lost vectors (data and parity mixed) on a batch: the
    rebuilt stripes equal the encoded originals, on both layouts."""
    torch = torch_dev
    rng = np.random.default_rng(d * 1000 + sum(lost))
    r = rslib.New(d, p)
    G = orc.gen_matrix(d, p).reshape(p, d)
    S, n = 4, 65536 + 48
    host = rng.integers(0, 256, (S, d + p, n), dtype=np.uint8)
    host[:, d:] = orc.encode_numpy(G, host[:, :d])
    before = rslib.jit_stats()["launches"]
    buf = torch.from_numpy(host).cuda()
    buf[:, lost] = 0x5A
    r.reconst_batch(buf, [], lost)
    torch.cuda.synchronize()
    assert np.array_equal(buf.cpu().numpy(), host), (d, p, lost)
    data = torch.from_numpy(np.ascontiguousarray(host[:, :d])).cuda()
    par = torch.from_numpy(np.ascontiguousarray(host[:, d:])).cuda()
    for v in lost:
        (data[:, v] if v < d else par[:, v - d]).fill_(0x33)
    r.reconst_batch_split(data, par, [], lost)
    torch.cuda.synchronize()
    assert np.array_equal(data.cpu().numpy(), host[:, :d]) and np.array_equal(par.cpu().numpy(), host[:, d:])
    assert rslib.jit_stats()["launches"] > before


def test_jit_multi_pattern_fallback(rslib, orc, torch_dev, jit_sync):
    """rs_reconst_batch_multi with 5-8-output patterns on non-contiguous
    stripes: each pattern's grouped launch maps its stripes through the
    device stripe-id list; untouched stripes stay bit-identical."""
    torch = torch_dev
    d, p, S, n = 10, 8, 12, 8192
    rng = np.random.default_rng(77)
    r = rslib.New(d, p)
    G = orc.gen_matrix(d, p).reshape(p, d)
    host = rng.integers(0, 256, (S, d, n), dtype=np.uint8)
    hpar = orc.encode_numpy(G, host)
    pats = [[0, 1, 2, 3, 4, 5, 6, 7], [2, 5, 8, 10, 12, 16], [10, 11, 12, 13, 14], 0, [1, 9, 11, 15, 17]]
    masks = np.zeros(S, np.uint64)
    for s in range(S):
        pt = pats[s % len(pats)]
        masks[s] = 0 if pt == 0 else sum(1 << v for v in pt)
    data = torch.from_numpy(host.copy()).cuda()
    par = torch.from_numpy(hpar.copy()).cuda()
    for s in range(S):
        for v in range(d + p):
            if (int(masks[s]) >> v) & 1:
                (data[s, v] if v < d else par[s, v - d]).fill_(0xEE)
    rslib.lib().rs_tune(b"jit_min_bytes", 0)
    r.reconst_batch_multi(data, par, masks)
    torch.cuda.synchronize()
    assert np.array_equal(data.cpu().numpy(), host) and np.array_equal(par.cpu().numpy(), hpar)


def test_jit_update_replace_8_parity(rslib, orc, torch_dev, jit_sync):
    """Update and Replace on a 10+8 batch (8-row XOR-accumulate products over
    2 and 3 columns, compiled, the old parity loaded up front) equal
    re-encoding the new data."""
    torch = torch_dev
    d, p, S, n = 10, 8, 3, 65536 + 32
    rng = np.random.default_rng(5)
    r = rslib.New(d, p)
    G = orc.gen_matrix(d, p).reshape(p, d)
    host = rng.integers(0, 256, (S, d + p, n), dtype=np.uint8)
    host[:, d:] = orc.encode_numpy(G, host[:, :d])
    buf = torch.from_numpy(host.copy()).cuda()
    new = rng.integers(0, 256, (S, n), dtype=np.uint8)
    before = rslib.jit_stats()["launches"]
    r.update_batch(torch.from_numpy(np.ascontiguousarray(host[:, 4])).cuda(), torch.from_numpy(new).cuda(), 4, buf)
    torch.cuda.synchronize()
    host[:, 4] = new
    exp = orc.encode_numpy(G, host[:, :d])
    got = buf.cpu().numpy()
    assert np.array_equal(got[:, d:], exp)
    rows = [1, 6, 8]
    repl = rng.integers(0, 256, (S, len(rows), n), dtype=np.uint8)
    r.replace_batch(torch.from_numpy(repl).cuda(), rows, buf)
    torch.cuda.synchronize()
    # Replace: the listed rows were zero when the parity was made (rs.go:492-529)
    base = host[:, :d].copy()
    base[:, rows] = 0
    par0 = orc.encode_numpy(G, base)
    base[:, rows] = repl
    exp2 = exp ^ orc.encode_numpy(G, base) ^ par0
    assert np.array_equal(buf.cpu().numpy()[:, d:], exp2)
    assert rslib.jit_stats()["launches"] >= before + 2


@pytest.mark.parametrize("d,p", [(16, 8), (9, 7), (14, 6)])
def test_jit_encode_without_build_time_network(rslib, orc, torch_dev, jit_sync, d, p):
    """Encode of codes whose generator has no generated network: interleaved
    [S][d+p][n] (256-lane workgroups when d+p >= 18) and split layouts."""
    torch = torch_dev
    rng = np.random.default_rng(d * 10 + p)
    r = rslib.New(d, p)
    G = orc.gen_matrix(d, p).reshape(p, d)
    for S, n in [(3, 16), (4, 65536 + 96), (2, 1 << 20)]:
        host = rng.integers(0, 256, (S, d + p, n), dtype=np.uint8)
        host[:, d:] = 0xA5
        exp = orc.encode_numpy(G, host[:, :d])
        buf = torch.from_numpy(host).cuda()
        r.encode_batch(buf)
        data = torch.from_numpy(np.ascontiguousarray(host[:, :d])).cuda()
        par = torch.full((S, p, n), 0xA5, dtype=torch.uint8, device="cuda")
        r.encode_batch_split(data, par)
        torch.cuda.synchronize()
        assert np.array_equal(buf.cpu().numpy()[:, d:], exp), (d, p, S, n)
        assert np.array_equal(par.cpu().numpy(), exp), (d, p, S, n, "split")


def test_jit_background_compile(rslib, orc, torch_dev):
    """Default mode on the assembly backend (comgr, tens of ms per matrix):
    the first launch of a new matrix only counts it, the second runs the
    perm-table kernels and queues a compile (jit_min_launches 2); once the
    compile is done the next launch runs the compiled kernel; all give the
    same bytes."""
    torch = torch_dev
    L = rslib.lib()
    assert L.rs_tune(b"jit", 1) == 0 and L.rs_tune(b"jit_backend", 1) == 0
    L.rs_tune(b"jit_min_bytes", 0)
    try:
        rng = np.random.default_rng(4242)
        mat = rng.integers(0, 256, (7, 11), dtype=np.uint8)
        r = rslib.New(10, 4)
        S, n = 2, 32768
        src = torch.from_numpy(rng.integers(0, 256, (S, 11, n), dtype=np.uint8)).cuda()
        exp = orc.encode_numpy(mat, src.cpu().numpy())
        st0 = rslib.jit_stats()
        dst = torch.zeros((S, 7, n), dtype=torch.uint8, device="cuda")
        for k in range(2):
            dst.zero_()
            r.gf_matmul_batch(mat, src, None, dst, None)
            torch.cuda.synchronize()
            assert np.array_equal(dst.cpu().numpy(), exp)
            assert rslib.jit_stats()["launches"] == st0["launches"]  # not compiled yet: perm-table kernels
            if k == 0:
                time.sleep(0.5)
                assert rslib.jit_stats()["compiled"] == st0["compiled"]  # one launch: counted, not queued
        t0 = time.time()
        while rslib.jit_stats()["compiled"] == st0["compiled"] and time.time() - t0 < 60:
            time.sleep(0.05)
        assert rslib.jit_stats()["compiled"] == st0["compiled"] + 1
        dst.zero_()
        r.gf_matmul_batch(mat, src, None, dst, None)
        torch.cuda.synchronize()
        assert np.array_equal(dst.cpu().numpy(), exp)
        assert rslib.jit_stats()["launches"] == st0["launches"] + 1
        _fork_child_sees_fresh_jit(rslib)
    finally:
        L.rs_tune(b"jit_min_bytes", 8 << 20)
        L.rs_tune(b"jit_backend", 2)


def _fork_child_sees_fresh_jit(rslib):
    """Advisor r05: a forked child inherits the compile worker's object but not
    its thread (and possibly its mutex held).  The pthread_atfork handler gives
    the child a fresh one: its counters start at zero, and taking the lock
    cannot hang.  The child makes no HIP call and leaves with os._exit."""
    import os

    assert rslib.jit_stats()["compiled"] > 0
    rfd, wfd = os.pipe()
    pid = os.fork()
    if pid == 0:  # child
        try:
            os.write(wfd, str(rslib.jit_stats()["compiled"]).encode())
        finally:
            os._exit(0)
    os.close(wfd)
    t0 = time.time()
    while True:
        done, status = os.waitpid(pid, os.WNOHANG)
        if done:
            break
        if time.time() - t0 > 20:
            os.kill(pid, 9)
            os.waitpid(pid, 0)
            raise AssertionError("forked child hung in rs_jit_stats (inherited lock)")
        time.sleep(0.01)
    got = os.read(rfd, 64).decode()
    os.close(rfd)
    assert os.WIFEXITED(status) and os.WEXITSTATUS(status) == 0
    assert got == "0", got


def test_jit_concurrent_threads_background(rslib, orc, torch_dev):
    """Background mode (assembly backend) under concurrency: 4 threads, each
    with its own handle, stream and matrix, launch repeatedly while their
    compiles are queued, run and loaded; every launch's bytes equal the
    oracle's, whichever kernel ran it."""
    import threading

    torch = torch_dev
    L = rslib.lib()
    assert L.rs_tune(b"jit", 1) == 0 and L.rs_tune(b"jit_backend", 1) == 0
    L.rs_tune(b"jit_min_bytes", 0)
    errors = []
    try:
        rng = np.random.default_rng(9090)
        jobs = []
        for t in range(4):
            rows, cols = 5 + t, 9 + 2 * t
            mat = rng.integers(0, 256, (rows, cols), dtype=np.uint8)
            src = rng.integers(0, 256, (3, cols, 16384 + 16 * t), dtype=np.uint8)
            jobs.append((mat, src, orc.encode_numpy(mat, src)))
        st0 = rslib.jit_stats()

        def worker(i):
            try:
                mat, hsrc, exp = jobs[i]
                r = rslib.New(10, 4)
                s = torch.cuda.Stream()
                src = torch.from_numpy(hsrc).cuda()
                dst = torch.empty((hsrc.shape[0], mat.shape[0], hsrc.shape[2]), dtype=torch.uint8, device="cuda")
                t0 = time.time()
                n = 0
                while time.time() - t0 < 60:
                    dst.fill_(0x5A)
                    torch.cuda.current_stream().synchronize()
                    r.gf_matmul_batch(mat, src, None, dst, None, stream=s)
                    s.synchronize()
                    if not np.array_equal(dst.cpu().numpy(), exp):
                        errors.append((i, n))
                        return
                    n += 1
                    if n >= 8 and rslib.jit_stats()["compiled"] >= st0["compiled"] + 4:
                        break
            except Exception as e:  # noqa: BLE001
                errors.append((i, repr(e)))

        th = [threading.Thread(target=worker, args=(i,)) for i in range(4)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        assert not errors, errors
        st = rslib.jit_stats()
        assert st["compiled"] == st0["compiled"] + 4 and st["failed"] == st0["failed"], (st0, st)
        assert st["launches"] > st0["launches"], (st0, st)
    finally:
        L.rs_tune(b"jit_min_bytes", 8 << 20)
        L.rs_tune(b"jit_backend", 2)


def test_jit_machine_code_first_sight_policy(rslib, orc, torch_dev):
    """Default mode on the default (machine-code) backend: a launch whose
    estimated loss on the table kernels exceeds the estimated time to build
    its kernel compiles at FIRST sight, on the launching thread, and runs it
    (a one-off erasure pattern of a wide code); a small launch of a fresh
    matrix runs on the table kernels until its launches have lost that much,
    then compiles.  Bytes equal the oracle's (small) or the no-compile run
    (large)."""
    torch = torch_dev
    L = rslib.lib()
    assert L.rs_tune(b"jit", 1) == 0 and L.rs_tune(b"jit_backend", 2) == 0
    rng = np.random.default_rng(777)
    r = rslib.New(10, 4)
    # large: 96 rows x 16 columns, 4 stripes of 1 MiB vectors (470 MB moved:
    # ~590 us estimated loss on the wide table kernel, ~380 us to build)
    rows, cols, S, n = 96, 16, 4, 1 << 20
    mat = rng.integers(0, 256, (rows, cols), dtype=np.uint8)
    src = torch.randint(0, 256, (S, cols, n), dtype=torch.uint8, device="cuda")
    ref = torch.zeros((S, rows, n), dtype=torch.uint8, device="cuda")
    assert L.rs_tune(b"jit", 0) == 0
    r.gf_matmul_batch(mat, src, None, ref, None)  # the table kernels' bytes
    assert L.rs_tune(b"jit", 1) == 0
    st0 = rslib.jit_stats()
    dst = torch.zeros_like(ref)
    r.gf_matmul_batch(mat, src, None, dst, None)
    torch.cuda.synchronize()
    st1 = rslib.jit_stats()
    assert st1["compiled"] == st0["compiled"] + 1 and st1["launches"] == st0["launches"] + 1, (st0, st1)
    assert torch.equal(dst, ref)
    # small: 7 x 11 over 2 x 32 KiB: ~1.2 MB per launch, a few ns lost each
    mat = rng.integers(0, 256, (7, 11), dtype=np.uint8)
    src = torch.from_numpy(rng.integers(0, 256, (2, 11, 32768), dtype=np.uint8)).cuda()
    exp = orc.encode_numpy(mat, src.cpu().numpy())
    dst = torch.zeros((2, 7, 32768), dtype=torch.uint8, device="cuda")
    for k in range(3):
        r.gf_matmul_batch(mat, src, None, dst, None)
        torch.cuda.synchronize()
        assert np.array_equal(dst.cpu().numpy(), exp)
    st2 = rslib.jit_stats()
    assert st2["compiled"] == st1["compiled"] and st2["launches"] == st1["launches"], (st1, st2)


def test_jit_prepare_then_first_launch_runs_compiled(rslib, orc, torch_dev):
    """rs_jit_prepare (default mode, no recurrence needed): after preparing the
    16+8 Encode, its first launch (a small one, below jit_min_bytes) already
    runs the compiled kernel; bytes equal the oracle's."""
    torch = torch_dev
    assert rslib.lib().rs_tune(b"jit", 1) == 0
    d, p = 16, 8
    r = rslib.New(d, p)
    r.jit_prepare()
    rng = np.random.default_rng(616)
    host = rng.integers(0, 256, (3, d + p, 65536), dtype=np.uint8)
    exp = orc.encode_numpy(orc.gen_matrix(d, p).reshape(p, d), host[:, :d])
    buf = torch.from_numpy(host).cuda()
    before = rslib.jit_stats()["launches"]
    r.encode_batch(buf)
    torch.cuda.synchronize()
    assert np.array_equal(buf.cpu().numpy()[:, d:], exp)
    assert rslib.jit_stats()["launches"] == before + 1


_DISK_SCRIPT = r'''
import json, os, sys
sys.path.insert(0, ROOT)
import numpy as np
import torch
import reedsolomon_amd as rs
from oracle import oracle
L = rs.lib()
assert L.rs_tune(b"jit", int(sys.argv[1])) == 0
rng = np.random.default_rng(5151)
mat = rng.integers(0, 256, (12, 20), dtype=np.uint8)
src_h = rng.integers(0, 256, (2, 20, 65536), dtype=np.uint8)
exp = oracle.encode_numpy(mat, src_h)
r = rs.New(10, 4)
src = torch.from_numpy(src_h).cuda()
dst = torch.zeros((2, 12, 65536), dtype=torch.uint8, device="cuda")
r.gf_matmul_batch(mat, src, None, dst, None)
torch.cuda.synchronize()
print(json.dumps({"ok": bool(np.array_equal(dst.cpu().numpy(), exp)), "jit": rs.jit_stats(),
                  "cache": rs.jit_cache_stats()}))
'''


def test_jit_disk_cache_across_processes(rslib, tmp_path):
    """The on-disk code-object cache: process A compiles a 12 x 20 matrix and
    writes its code object; process B's FIRST launch of the same matrix (the
    default background mode, which would otherwise only count it) loads the
    file and runs the compiled kernel with no compile; a corrupted file is
    rejected and recompiled.  Every launch's bytes equal the oracle's."""
    import json
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    # (the disk cache serves the comgr / hiprtc backends; the machine-code
    # backend builds a kernel about as fast as it would read the file)
    env = dict(os.environ, RSAMD_JIT_CACHE_DIR=str(tmp_path / "jit"), RSAMD_JIT_DISK_CACHE="1",
               RSAMD_JIT_BACKEND="1")
    script = "ROOT = %r\n" % root + _DISK_SCRIPT

    def run(mode):
        out = subprocess.run([sys.executable, "-c", script, str(mode)], env=env, capture_output=True, text=True,
                             timeout=240)
        assert out.returncode == 0, out.stderr[-3000:]
        return json.loads(out.stdout.strip().splitlines()[-1])

    a = run(2)  # compile on the launching thread
    assert a["ok"] and a["jit"]["compiled"] == 1 and a["jit"]["launches"] == 1, a
    assert a["cache"]["misses"] == 1 and a["cache"]["writes"] == 1, a
    files = list((tmp_path / "jit").glob("*.co"))
    assert len(files) == 1, files
    b = run(1)  # default mode: first sight, loaded from disk, compiled kernel runs
    assert b["ok"] and b["jit"]["compiled"] == 0 and b["jit"]["launches"] == 1, b
    assert b["cache"]["hits"] == 1 and b["cache"]["writes"] == 0, b
    raw = bytearray(files[0].read_bytes())
    raw[len(raw) // 2] ^= 0xFF  # corrupt the code: the checksum rejects it
    files[0].write_bytes(bytes(raw))
    c = run(2)
    assert c["ok"] and c["cache"]["rejects"] == 1 and c["jit"]["compiled"] == 1 and c["cache"]["writes"] == 1, c
    # the cache holds code the process runs: a directory or file others may
    # write is neither read nor written (advisor finding, round 3)
    os.chmod(tmp_path / "jit", 0o777)
    d = run(1)
    assert d["ok"] and d["cache"]["hits"] == 0 and d["cache"]["writes"] == 0, d
    os.chmod(tmp_path / "jit", 0o700)
    for f in (tmp_path / "jit").glob("*.co"):
        os.chmod(f, 0o666)
    e = run(1)
    assert e["ok"] and e["cache"]["hits"] == 0, e
    for f in (tmp_path / "jit").glob("*.co"):
        os.chmod(f, 0o600)
    g = run(1)
    assert g["ok"] and g["cache"]["hits"] == 1, g


def test_jit_eviction_off_the_launch_path(rslib, orc, torch_dev, jit_sync):
    """More distinct matrices than the kernel table holds (256), each compiled
    on first sight (jit=2) and launched: the table fills, a launch queues the
    eviction on the library's worker instead of draining the device itself
    (advisor round 4), the worker drops the older half after the device
    drain, and every launch before, during and after stays bit-exact against
    the oracle (evicted matrices that come back are compiled again)."""
    import time

    torch = torch_dev
    rng = np.random.default_rng(2024)
    r = rslib.New(10, 4)
    S, n = 2, 4096
    src_h = rng.integers(0, 256, (S, 6, n), dtype=np.uint8)
    src = torch.from_numpy(src_h).cuda()
    t0 = rslib.jit_table_stats()
    mats = [rng.integers(0, 256, (5, 6), dtype=np.uint8) for _ in range(300)]
    for i, mat in enumerate(mats + mats[:20]):  # the first 20 again at the end: evicted, compiled afresh
        dst = torch.zeros((S, 5, n), dtype=torch.uint8, device="cuda")
        r.gf_matmul_batch(mat, src, None, dst, None)
        if i % 7 == 0 or i >= 290:
            torch.cuda.synchronize()
            assert np.array_equal(dst.cpu().numpy(), orc.encode_numpy(mat, src_h)), i
    torch.cuda.synchronize()
    deadline = time.time() + 30  # the worker's eviction runs asynchronously
    while rslib.jit_table_stats()["evictions"] == t0["evictions"] and time.time() < deadline:
        time.sleep(0.05)
    st = rslib.jit_table_stats()
    assert st["evictions"] > t0["evictions"], (t0, st)
    assert st["entries"] <= 256, st
    assert rslib.jit_stats()["failed"] == 0
