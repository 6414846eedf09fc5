#!/usr/bin/env python3
"""How many XOR instructions would a common-subexpression pass over the bit
matrix save in the run-time bit-sliced networks (jit_asm.cpp)?  VERDICT r05
"next" item 5: 64+64, 128+128 and 200+56 Encode are VALU-bound,
76 % of their instructions being the one v_bitop3 (xor3) per output plane,
row and column.

The generated kernel streams columns: a wave holds one column's 8 bit-planes
and its 16 rows x 8 planes of accumulators (128 VGPRs), so every sharing
scheme is per column (or per column group a wave can hold).  For each 16-row
path of the Encode matrix (matrix.go:37-54: Cauchy rows, GF(2^8)/0x11d) this
tool counts the XOR-class VALU instructions per column:

  current  - what jit_asm.cpp emits: per 4-plane half, every subset of 2-4
             planes some output uses, built with one XOR from a smaller one,
             then one xor3 / xor per output plane with a nonzero form;
  cse1     - a greedy CSE over the column's 128 output forms (8 planes):
             repeatedly materialise the pair or triple of signals (one v_xor
             or v_xor3 each) whose substitution saves the most accumulate
             instructions, an accumulate absorbing up to two signals
             (acc ^ s1 ^ s2); the column's outputs then cost ceil(terms/2);
  cse2     - the same over PAIRS of columns (16 planes, two columns held at
             once, 8 more VGPRs): each output absorbs both columns' signals.

It prints per code: instructions per column per path and the reduction of
cse1 / cse2 against current.  No GPU, no oracle: the GF(2^8) field is built
here from its polynomial.

Usage: python tools/cse_xor_count.py [d+p ...]   (default 32+32 64+64 128+128 200+56)
"""
import itertools
import sys

import numpy as np

POLY = 0x11D


def gf_tables():
    exp = [0] * 512
    log = [0] * 256
    x = 1
    for i in range(255):
        exp[i] = x
        log[x] = i
        x <<= 1
        if x & 0x100:
            x ^= POLY
    for i in range(255, 512):
        exp[i] = exp[i - 255]
    return exp, log


EXP, LOG = gf_tables()


def gmul(a, b):
    if a == 0 or b == 0:
        return 0
    return EXP[LOG[a] + LOG[b]]


def ginv(a):
    return EXP[255 - LOG[a]]


def gen_matrix(d, p):
    """Parity rows of makeEncodeMatrix (matrix.go:37-54): G[j][i] = 1 / ((d + j) ^ i)."""
    return [[ginv((d + j) ^ i) for i in range(d)] for j in range(p)]


def forms(coef):
    """Output plane b of coef * x as an 8-bit mask of input planes."""
    cols = [gmul(coef, 1 << i) for i in range(8)]  # image of each input bit
    return [sum(((cols[i] >> b) & 1) << i for i in range(8)) for b in range(8)]


def current_cost(col_forms):
    """jit_asm.cpp combine(): subsets per half (the `need` closure), then one
    update per output plane with a nonzero form."""
    n = 0
    for half in range(2):
        have = {1 << b for b in range(4)}
        used = {(m >> (4 * half)) & 15 for m in col_forms} - {0}
        need = set()
        for m in used:
            x = m
            while x and x not in have and x not in need:
                need.add(x)
                x ^= x & -x
        n += len(need)
    n += sum(1 for m in col_forms if m)
    return n


def acc_cost(t):
    return (t + 1) // 2 if t else 0


def cse_cost(outs, nsig):
    """Greedy CSE with xor3-aware accounting.  outs: list of sets of signal ids
    (the input planes 0..nsig-1 to start with).  Returns the instruction
    count: materialised signals + sum over outputs of ceil(terms / 2)."""
    outs = [set(o) for o in outs if o]
    built = 0
    nxt = nsig
    while True:
        best, best_gain = None, 0
        cand = {}
        for o in outs:
            if len(o) < 2:
                continue
            s = sorted(o)
            t = len(s)
            g2 = acc_cost(t) - acc_cost(t - 1)
            for pr in itertools.combinations(s, 2):
                cand[pr] = cand.get(pr, 0) + g2
            if t >= 3:
                g3 = acc_cost(t) - acc_cost(t - 2)
                for tr in itertools.combinations(s, 3):
                    cand[tr] = cand.get(tr, 0) + g3
        for k, g in cand.items():
            if g - 1 > best_gain:
                best, best_gain = k, g - 1
        if best is None:
            break
        ks = set(best)
        for o in outs:
            if ks <= o:
                o -= ks
                o.add(nxt)
        nxt += 1
        built += 1
    return built + sum(acc_cost(len(o)) for o in outs)


def planes(mask, base=0):
    return {base + i for i in range(8) if mask >> i & 1}


def path_costs(G, rows, d):
    cur = c1 = c2 = 0
    for c in range(d):
        f = [m for r in rows for m in forms(G[r][c])]
        cur += current_cost(f)
        c1 += cse_cost([planes(m) for m in f], 8)
    for c in range(0, d, 2):
        cs = [c] + ([c + 1] if c + 1 < d else [])
        outs = []
        for r in rows:
            fr = [forms(G[r][x]) for x in cs]
            for b in range(8):
                o = set()
                for k, x in enumerate(cs):
                    o |= planes(fr[k][b], 8 * k)
                outs.append(o)
        c2 += cse_cost(outs, 16)
    return cur, c1, c2


def main():
    codes = sys.argv[1:] or ["32+32", "64+64", "128+128", "200+56"]
    print(f"{'code':>9} {'paths':>5} | {'current':>9} {'cse1':>9} {'cse2':>9} | per column and path: "
          f"{'cur':>6} {'cse1':>6} {'cse2':>6} | cse1 vs cur, cse2 vs cur")
    for code in codes:
        d, p = (int(x) for x in code.split("+"))
        G = gen_matrix(d, p)
        tot = np.zeros(3)
        npaths = (p + 15) // 16
        for k in range(npaths):
            rows = list(range(16 * k, min(p, 16 * k + 16)))
            tot += path_costs(G, rows, d)
        per = tot / (d * npaths)
        print(f"{code:>9} {npaths:>5} | {tot[0]:>9.0f} {tot[1]:>9.0f} {tot[2]:>9.0f} | {'':>20}"
              f"{per[0]:>6.1f} {per[1]:>6.1f} {per[2]:>6.1f} | {100 * (1 - tot[1] / tot[0]):+.1f} %, "
              f"{100 * (1 - tot[2] / tot[0]):+.1f} %", flush=True)


if __name__ == "__main__":
    main()
