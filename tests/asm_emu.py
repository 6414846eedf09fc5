"""A small CPU emulator for the gfx950 assembly the run-time kernel generator
emits (reedsolomon_amd/csrc/jit_asm.cpp): test infrastructure, so the
generated kernels' arithmetic and addressing can be checked against the
oracle without a GPU (tests/test_jit_asm.py).

Only the instruction subset the generator uses is implemented, with the
semantics of the CDNA ISA: scalar loads from the kernel-argument block and
from device memory, SALU integer ops and branches (s_getpc / s_setpc long
jumps included), VALU bitwise ops on 64 lanes (numpy vectors), and
buffer_load / buffer_store_dwordx2 through 128-bit buffer descriptors with
range checking (out-of-range lanes read 0, their stores are dropped).
Every access completes at once, but the wait counts are checked: vector
memory operations retire in issue order at `s_waitcnt vmcnt(N)` (loads and
stores share the counter on gfx9), scalar loads only at `lgkmcnt(0)` (they
may return out of order), and reading or overwriting a register whose load
has not been waited for raises `WaitcntError` — the hardware would have
used stale data.  So does `v_readfirstlane` of a VGPR the instruction just
before it wrote: the hardware needs one wait state there and otherwise reads
the old value (measured on MI355X, tools/asm_probe/wave_id.s).

Workgroups with LDS (the shared-column kernels): ds_write_b128 /
ds_read_b128 / ds_read_b64 on a per-workgroup LDS of the size the kernel
descriptor declares (bounds and alignment checked); reads land at
`lgkmcnt(0)`, or at `lgkmcnt(N)` for all but the newest N (LDS reads
return in order; scalar loads may still be out then).  LDS-DMA loads (`buffer_load_dwordx4 ...
lds`: 16 bytes per lane written to LDS at M0 + 16 * lane) count on vmcnt like
other vector memory loads, and an LDS read of bytes whose DMA has not been
waited for raises `WaitcntError`.  The waves of a workgroup run in rounds
from one s_barrier to the next, in alternating order, and a wave that reads
LDS bytes another wave wrote in the same round, or writes bytes another
wave read or wrote in it, raises `LdsRaceError`: without the barrier
between them the hardware's result would depend on timing.
"""
from __future__ import annotations

import re

import numpy as np

M32 = 0xFFFFFFFF


class Memory:
    """Flat device memory: a byte array starting at `base`."""

    def __init__(self, size: int, base: int = 0x100000):
        self.base = base
        self.buf = np.zeros(size, np.uint8)
        self.top = 0

    def alloc(self, n: int, align: int = 256) -> int:
        self.top = (self.top + align - 1) // align * align
        addr = self.base + self.top
        self.top += n
        assert self.top <= self.buf.size, "emulated memory full"
        return addr

    def view(self, addr: int, n: int) -> np.ndarray:
        o = addr - self.base
        assert 0 <= o and o + n <= self.buf.size, hex(addr)
        return self.buf[o:o + n]


def _parse(src: str):
    prog, labels = [], {}
    for raw in src.splitlines():
        line = raw.split(";")[0].strip()
        if not line or line.startswith("."):
            m = re.match(r"^(\.L\w+|\w+):$", line)
            if m:
                labels[m.group(1)] = len(prog)
            continue
        m = re.match(r"^(\.L\w+|\w+):$", line)
        if m:
            labels[m.group(1)] = len(prog)
            continue
        op, _, rest = line.partition(" ")
        prog.append((op, rest.strip()))
    return prog, labels


def _regs(tok: str):
    """'v[4:5]' -> ('v', 4, 2); 's12' -> ('s', 12, 1); 'm0' -> ('s', 124, 1)"""
    if tok == "m0":
        return "s", 124, 1
    m = re.match(r"^([sv])\[(\d+):(\d+)\]$", tok)
    if m:
        a, b = int(m.group(2)), int(m.group(3))
        return m.group(1), a, b - a + 1
    m = re.match(r"^([sv])(\d+)$", tok)
    if m:
        return m.group(1), int(m.group(2)), 1
    return None


class WaitcntError(AssertionError):
    pass


class LdsRaceError(AssertionError):
    pass


class _Dma:
    """An outstanding LDS-DMA load in a wave's vmcnt queue: the LDS bytes
    [lo, hi) it writes (it has no VGPR destination)."""

    def __init__(self, lo: int, hi: int):
        self.lo, self.hi = lo, hi

    def __contains__(self, vgpr) -> bool:
        return False

    def overlaps(self, lo: int, hi: int) -> bool:
        return self.lo < hi and lo < self.hi


class Lds:
    """A workgroup's LDS plus, per barrier round, who wrote / read each byte."""

    def __init__(self, size: int, nw: int):
        self.buf = np.zeros(max(size, 16), np.uint8)
        self.size = size
        self.writer = np.full(self.buf.size, -1, np.int16)
        self.readers = np.zeros((nw, self.buf.size), bool)

    def new_round(self):
        self.writer[:] = -1
        self.readers[:] = False

    def _span(self, wave, addr, write, n=16):
        if addr % n or addr < 0 or addr + n > self.size:
            raise AssertionError(f"wave {wave}: LDS access at {addr} out of bounds / unaligned (size {self.size})")
        sl = slice(addr, addr + n)
        w = self.writer[sl]
        if np.any((w >= 0) & (w != wave)):
            raise LdsRaceError(f"wave {wave}: LDS bytes {addr}.. written by wave {int(w.max())} in this round")
        if write:
            others = np.delete(self.readers[:, sl], wave, axis=0)
            if others.any():
                raise LdsRaceError(f"wave {wave}: LDS bytes {addr}.. read by another wave in this round")
            self.writer[sl] = wave
        else:
            self.readers[wave, sl] = True
        return sl


class Wave:
    def __init__(self, emu, karg_addr, wg, tid0, lds=None):
        self.emu = emu
        self.lds = lds
        self.wid = tid0 // 64
        self.s = [0] * 128
        self.v = np.zeros((256, 64), np.uint64)
        self.s[0], self.s[1] = karg_addr & M32, karg_addr >> 32
        self.s[2], self.s[3] = wg
        # work-item id x in bits 0-9; the bits above (packed y / z ids) hold
        # junk here, so code that depends on them fails
        self.v[0] = np.arange(tid0, tid0 + 64, dtype=np.uint64) | (0x2A5 << 10)
        self.scc = 0
        self.vm = []        # outstanding vector memory ops, issue order: set of load-destination VGPRs
        self.lgkm = set()   # SGPRs of outstanding scalar loads
        self.lds_q = []     # outstanding LDS ops in issue order: (VGPRs, is_write); they complete in order
        self.pc = 0
        self.prev_vdst = None  # VGPR the previous instruction wrote (VALU), for the readlane hazard


    # wait-count checks
    def _chk(self, kind, idx, n, write=False):
        for i in range(idx, idx + n):
            if kind == "v" and any(i in d for d in self.vm):
                raise WaitcntError(f"pc {self.pc}: v{i} {'written' if write else 'read'} before its load was waited for")
            # an LDS read's destination may be neither read nor written before it
            # lands; an LDS write's data registers may be read but not overwritten
            if kind == "v" and any(i in regs and (write or not wr) for regs, wr in self.lds_q):
                raise WaitcntError(f"pc {self.pc}: v{i} {'written' if write else 'read'} before its LDS op completed")
            if kind == "s" and i in self.lgkm:
                raise WaitcntError(f"pc {self.pc}: s{i} {'written' if write else 'read'} before its load was waited for")

    def _use(self, tok, write=False):
        r = _regs(tok)
        if r:
            self._chk(r[0], r[1], r[2], write)

    # operand values
    def sval(self, tok: str) -> int:
        r = _regs(tok)
        self._use(tok)
        if r and r[0] == "s":
            if r[2] == 1:
                return self.s[r[1]]
            return self.s[r[1]] | (self.s[r[1] + 1] << 32)
        return int(tok, 0) & 0xFFFFFFFFFFFFFFFF

    def vval(self, tok: str) -> np.ndarray:
        r = _regs(tok)
        self._use(tok)
        if r and r[0] == "v":
            return self.v[r[1]] & M32
        return np.full(64, self.sval(tok) & M32, np.uint64)

    def run(self, prog, labels):
        """A generator: yields at every s_barrier, returns at s_endpgm."""
        pc = 0
        emu = self.emu
        while True:
            op, rest = prog[pc]
            self.pc = pc
            pc += 1
            prev, self.prev_vdst = self.prev_vdst, None
            ops = [t.strip() for t in re.split(r",\s*(?![^\[]*\])", rest)] if rest else []
            if op == "s_endpgm":
                return
            if op == "s_waitcnt":
                for m_ in re.finditer(r"(vmcnt|lgkmcnt)\((\d+)\)", rest):
                    n = int(m_.group(2))
                    if m_.group(1) == "vmcnt":
                        while len(self.vm) > n:
                            self.vm.pop(0)
                    elif n == 0:
                        self.lgkm.clear()
                        self.lds_q.clear()
                    else:
                        # LDS reads return in order, scalar loads in any order:
                        # a nonzero count retires the LDS reads older than the
                        # newest n (whatever scalar loads are still out, they
                        # only add to the count) and no scalar load
                        while len(self.lds_q) > n:
                            self.lds_q.pop(0)
                continue
            if op == "s_barrier":
                yield "barrier"
                continue
            if op == "s_nop":
                continue
            if op == "ds_read_b64":
                assert self.lds is not None, "LDS access in a kernel without LDS"
                off = 0
                for m_ in rest.split():
                    if m_.startswith("offset:"):
                        off = int(m_.split(":")[1])
                dr, ar = _regs(ops[0]), _regs(ops[1].split()[0])
                self._chk("v", ar[1], 1)
                self._chk("v", dr[1], 2, write=True)
                addr = self.v[ar[1]].astype(np.int64) + off
                lo, hi = int(addr.min()), int(addr.max()) + 8
                if any(isinstance(d, _Dma) and d.overlaps(lo, hi) for d in self.vm):
                    raise WaitcntError(f"pc {self.pc}: LDS bytes {lo}..{hi} read before their LDS-DMA was waited for")
                for lane in range(64):
                    sl = self.lds._span(self.wid, int(addr[lane]), False, 8)
                    w = self.lds.buf[sl].view(np.uint32)
                    self.v[dr[1], lane], self.v[dr[1] + 1, lane] = int(w[0]), int(w[1])
                self.lds_q.append(({dr[1], dr[1] + 1}, False))
                continue
            if op == "buffer_load_dwordx4" and rest.split()[-1] == "lds":
                assert self.lds is not None, "LDS-DMA in a kernel without LDS"
                voff = self.vval(ops[0]).astype(np.int64)
                sr = _regs(ops[1])
                self._chk("s", sr[1], 4)
                self._chk("s", 124, 1)
                m0 = self.s[124]
                d0, d1, d2 = self.s[sr[1]], self.s[sr[1] + 1], self.s[sr[1] + 2]
                base, nrec = d0 | ((d1 & 0xFFFF) << 32), d2
                assert "offset:" not in rest, "LDS-DMA with an instruction offset (its LDS semantics are not modelled)"
                for lane in range(64):
                    o = int(voff[lane])
                    sl = self.lds._span(self.wid, m0 + 16 * lane, True)
                    self.lds.buf[sl] = emu.mem.view(base + o, 16) if o + 16 <= nrec else 0
                self.vm.append(_Dma(m0, m0 + 16 * 64))
                continue
            if op in ("ds_write_b128", "ds_read_b128"):
                assert self.lds is not None, "LDS access in a kernel without LDS"
                mods = rest.split()
                off = 0
                for m_ in mods:
                    if m_.startswith("offset:"):
                        off = int(m_.split(":")[1])
                if op == "ds_write_b128":
                    ar, dr = _regs(ops[0]), _regs(ops[1].split()[0])
                    self._chk("v", ar[1], 1)
                    self._chk("v", dr[1], 4)
                    addr = self.v[ar[1]].astype(np.int64) + off
                    lo, hi = int(addr.min()), int(addr.max()) + 16
                    if any(isinstance(d, _Dma) and d.overlaps(lo, hi) for d in self.vm):
                        raise WaitcntError(f"pc {self.pc}: LDS bytes {lo}..{hi} written while an LDS-DMA into them is outstanding")
                    for lane in range(64):
                        sl = self.lds._span(self.wid, int(addr[lane]), True)
                        self.lds.buf[sl] = np.array([self.v[dr[1] + q, lane] for q in range(4)],
                                                    np.uint32).view(np.uint8)
                    self.lds_q.append(({dr[1] + q for q in range(4)}, True))
                else:
                    dr, ar = _regs(ops[0]), _regs(ops[1].split()[0])
                    self._chk("v", ar[1], 1)
                    self._chk("v", dr[1], 4, write=True)
                    addr = self.v[ar[1]].astype(np.int64) + off
                    lo, hi = int(addr.min()), int(addr.max()) + 16
                    if any(isinstance(d, _Dma) and d.overlaps(lo, hi) for d in self.vm):
                        raise WaitcntError(f"pc {self.pc}: LDS bytes {lo}..{hi} read before their LDS-DMA was waited for")
                    for lane in range(64):
                        sl = self.lds._span(self.wid, int(addr[lane]), False)
                        w = self.lds.buf[sl].view(np.uint32)
                        for q in range(4):
                            self.v[dr[1] + q, lane] = int(w[q])
                    self.lds_q.append(({dr[1] + q for q in range(4)}, False))
                continue
            if ops and op not in ("s_cbranch_scc1", "s_cbranch_scc0", "s_branch", "s_cmp_eq_u64", "s_cmp_eq_u32",
                                  "s_cmp_ge_u32", "s_setpc_b64", "buffer_store_dwordx2", "ds_write_b128",
                                  "buffer_load_dwordx4"):
                self._use(ops[0], write=True)  # the destination
            if op == "s_load_dword" or op == "s_load_dwordx2":
                d, base, off = ops[0], ops[1], int(ops[2], 0)
                addr = self.sval(base) + off
                n = 1 if op == "s_load_dword" else 2
                r = _regs(d)
                for k in range(n):
                    self.s[r[1] + k] = emu.read32(addr + 4 * k)
                    self.lgkm.add(r[1] + k)
                continue
            if op == "s_mov_b32":
                self.s[_regs(ops[0])[1]] = self.sval(ops[1]) & M32
                continue
            if op in ("s_add_u32", "s_addc_u32", "s_mul_i32", "s_mul_hi_u32", "s_and_b32", "s_lshl_b32", "s_lshr_b32",
                      "s_sub_u32", "s_or_b32"):
                d = _regs(ops[0])[1]
                a = self.sval(ops[1]) & M32
                b = self._imm_expr(ops[2], labels, pc) if op in ("s_add_u32", "s_addc_u32") else self.sval(ops[2]) & M32
                b &= M32
                if op == "s_add_u32":
                    t = a + b
                    self.s[d], self.scc = t & M32, int(t >> 32)
                elif op == "s_addc_u32":
                    t = a + b + self.scc
                    self.s[d], self.scc = t & M32, int(t >> 32)
                elif op == "s_mul_i32":
                    self.s[d] = (a * b) & M32
                elif op == "s_mul_hi_u32":
                    self.s[d] = (a * b) >> 32
                elif op == "s_and_b32":
                    self.s[d] = a & b
                    self.scc = int(self.s[d] != 0)
                elif op == "s_or_b32":
                    self.s[d] = a | b
                    self.scc = int(self.s[d] != 0)
                elif op == "s_sub_u32":
                    self.s[d], self.scc = (a - b) & M32, int(b > a)
                elif op == "s_lshr_b32":
                    self.s[d] = a >> (b & 31)
                    self.scc = int(self.s[d] != 0)
                else:
                    self.s[d] = (a << (b & 31)) & M32
                    self.scc = int(self.s[d] != 0)
                continue
            if op == "s_lshl_b64":
                r = _regs(ops[0])
                x = (self.sval(ops[1]) << int(ops[2], 0)) & 0xFFFFFFFFFFFFFFFF
                self.s[r[1]], self.s[r[1] + 1] = x & M32, x >> 32
                continue
            if op == "s_cmp_eq_u64":
                self.scc = int(self.sval(ops[0]) == (int(ops[1], 0) & 0xFFFFFFFFFFFFFFFF))
                continue
            if op == "s_cmp_eq_u32":
                self.scc = int((self.sval(ops[0]) & M32) == (self.sval(ops[1]) & M32))
                continue
            if op == "s_cmp_ge_u32":
                self.scc = int((self.sval(ops[0]) & M32) >= (self.sval(ops[1]) & M32))
                continue
            if op == "s_cbranch_scc1":
                if self.scc:
                    pc = labels[ops[0]]
                continue
            if op == "s_cbranch_scc0":
                if not self.scc:
                    pc = labels[ops[0]]
                continue
            if op == "s_branch":
                pc = labels[ops[0]]
                continue
            if op == "s_getpc_b64":  # the "pc" of the next instruction, as an index
                r = _regs(ops[0])
                self.s[r[1]], self.s[r[1] + 1] = pc, 0
                continue
            if op == "s_setpc_b64":
                pc = self.sval(ops[0])
                continue
            # ---- VALU (64 lanes)
            if op == "v_readfirstlane_b32":
                if prev is not None and _regs(ops[1])[1] == prev:
                    raise WaitcntError(f"pc {self.pc}: v_readfirstlane of v{prev} right after a VALU wrote it")
                self.s[_regs(ops[0])[1]] = int(self.vval(ops[1])[0])
                continue
            if op in ("v_and_b32", "v_xor_b32", "v_add_u32", "v_lshlrev_b32", "v_lshrrev_b32", "v_mov_b32"):
                d = _regs(ops[0])[1]
                if op == "v_mov_b32":
                    self.v[d] = self.vval(ops[1])
                    self.prev_vdst = d
                    continue
                a, b = self.vval(ops[1]), self.vval(ops[2])
                if op == "v_and_b32":
                    x = a & b
                elif op == "v_xor_b32":
                    x = a ^ b
                elif op == "v_add_u32":
                    x = (a + b) & M32
                elif op == "v_lshlrev_b32":
                    x = (b << (a & 31)) & M32
                else:
                    x = b >> (a & 31)
                self.v[d] = x
                self.prev_vdst = d
                continue
            if op == "v_bfi_b32":
                d = _regs(ops[0])[1]
                m, x, y = self.vval(ops[1]), self.vval(ops[2]), self.vval(ops[3])
                self.v[d] = (m & x) | ((~m & M32) & y)
                self.prev_vdst = d
                continue
            if op == "v_bitop3_b32":
                d = _regs(ops[0])[1]
                parts = ops[3].split()
                assert parts[1] == "bitop3:0x96", ops
                self.v[d] = self.vval(ops[1]) ^ self.vval(ops[2]) ^ self.vval(parts[0])
                self.prev_vdst = d
                continue
            if op in ("buffer_load_dwordx2", "buffer_store_dwordx2"):
                vr = _regs(ops[0])
                voff = self.vval(ops[1]).astype(np.int64)
                sr = _regs(ops[2])
                self._chk("s", sr[1], 4)
                if op == "buffer_store_dwordx2":
                    self._chk("v", vr[1], 2)
                self.vm.append({vr[1], vr[1] + 1} if op == "buffer_load_dwordx2" else set())
                d0, d1, d2 = self.s[sr[1]], self.s[sr[1] + 1], self.s[sr[1] + 2]
                base = d0 | ((d1 & 0xFFFF) << 32)
                nrec = d2
                mods = ops[3].split()[1:]
                imm = 0
                for m_ in mods:
                    if m_.startswith("offset:"):
                        imm = int(m_.split(":")[1])
                off = voff + imm
                for lane in range(64):
                    o = int(off[lane])
                    inr = o + 8 <= nrec
                    if op == "buffer_load_dwordx2":
                        if inr:
                            w = emu.mem.view(base + o, 8).view(np.uint32)
                            self.v[vr[1], lane], self.v[vr[1] + 1, lane] = int(w[0]), int(w[1])
                        else:
                            self.v[vr[1], lane] = self.v[vr[1] + 1, lane] = 0
                    elif inr:
                        w = np.array([self.v[vr[1], lane], self.v[vr[1] + 1, lane]], np.uint32)
                        emu.mem.view(base + o, 8)[:] = w.view(np.uint8)
                continue
            raise NotImplementedError(f"{op} {rest}")

    def _imm_expr(self, tok, labels, pc):
        m = re.match(r"^\((\.L\w+)-(\.L\w+)\)(&4294967295|>>32)$", tok)
        if m:
            # long jumps: the emulator's "pc" is an instruction index and
            # s_getpc gave the index after it (the .Lpc label's position)
            delta = labels[m.group(1)] - labels[m.group(2)]
            return delta & M32 if m.group(3) == "&4294967295" else (delta >> 32) & M32
        return self.sval(tok)


class Emu:
    def __init__(self, mem: Memory):
        self.mem = mem
        self.karg = None

    def read32(self, addr: int) -> int:
        if self.karg is not None and self.karg[0] <= addr < self.karg[0] + len(self.karg[1]):
            o = addr - self.karg[0]
            return int.from_bytes(self.karg[1][o:o + 4], "little")
        return int(self.mem.view(addr, 4).view(np.uint32)[0])

    def launch(self, src: str, karg: bytes, grid, nw: int):
        prog, labels = _parse(src)
        m = re.search(r"\.amdhsa_group_segment_fixed_size\s+(\d+)", src)
        lds_size = int(m.group(1)) if m else 0
        self.karg = (0x7F0000000000, karg)
        for y in range(grid[1]):
            for x in range(grid[0]):
                lds = Lds(lds_size, nw) if lds_size else None
                live = [Wave(self, self.karg[0], (x, y), 64 * w, lds).run(prog, labels) for w in range(nw)]
                rnd = 0
                while live:
                    if lds is not None:
                        lds.new_round()
                    order = live if rnd % 2 == 0 else live[::-1]
                    still = []
                    for g in order:
                        try:
                            next(g)
                            still.append(g)
                        except StopIteration:
                            pass
                    if still and len(still) != len(live):
                        raise AssertionError("a wave ended while others wait at a barrier")
                    live = [g for g in live if g in still]
                    rnd += 1
