"""Generate tests/golden/vectors.json — golden input/output vectors.

TEST INFRASTRUCTURE. Inputs come from a seeded counter-mode splitmix64 stream,
one per (seed, stripe, vector) (`stream` below; tests regenerate the same
bytes). Outputs come from the CPU oracle (oracle/rs_oracle.c), which is
itself pinned to the reference's tables and KATs by tests/test_oracle.py.
The reference (Go) cannot run in this image, so these vectors pin the oracle
and the HIP path to each other over time. They are not reference outputs.

    python tests/golden/make_vectors.py          # rewrite vectors.json
    python tests/golden/make_vectors.py --check  # exit 1 if it would change

Contents (SURVEY.md 8c "Golden vectors"):
  encode    10+4 and 12+4 at sizes {1,15,16,17,31,33,255,1024,8192,1 MiB}:
            sha256 of the p parity vectors concatenated; parity hex for sizes <= 33
  reconst   10+4 @ 8 KiB, every C(14,1..4) erasure pattern (1470), with
            garbage in lost vectors: per-pattern sha256 of the rebuilt
            vectors for 1-2 losses, one sha256 over all patterns' outputs
  update    10+4 @ 8 KiB, every data row: sha256 of the updated parity
  replace   10+4 @ 8 KiB, rn = 1..6 (rows 0..rn-1 replaced by zero): sha256 of parity
"""
from __future__ import annotations

import hashlib
import itertools
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
OUT = os.path.join(HERE, "vectors.json")

SEED = 0x5EED
ENCODE_SHAPES = [(10, 4), (12, 4)]
ENCODE_SIZES = [1, 15, 16, 17, 31, 33, 255, 1024, 8192, 1 << 20]
HEX_MAX = 33
STRIPE_SIZE = 8192
_M64 = (1 << 64) - 1
_GOLDEN = np.uint64(0x9E3779B97F4A7C15)


def _mix(z: np.ndarray) -> np.ndarray:
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def stream(stripe: int, vect: int, n: int, seed: int = SEED) -> np.ndarray:
    """n bytes of the splitmix64 stream for (seed, stripe, vect)."""
    key = _mix(np.array([(seed * 0x100000001B3 + stripe * 0x10001 + vect) & _M64], np.uint64))[0]
    words = (n + 7) // 8
    ctr = np.arange(1, words + 1, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = _mix(key + ctr * _GOLDEN)
    return z.view(np.uint8)[:n].copy()


def stripe_data(d: int, size: int, stripe: int = 0):
    return [stream(stripe, i, size) for i in range(d)]


def sha(vs) -> str:
    h = hashlib.sha256()
    for v in vs:
        h.update(np.ascontiguousarray(v).tobytes())
    return h.hexdigest()


def reconst_patterns(n: int = 14, max_lost: int = 4):
    return [list(c) for k in range(1, max_lost + 1) for c in itertools.combinations(range(n), k)]


def garbage(lost: int, size: int) -> np.ndarray:
    return stream(9999, lost, size)


def make(orc) -> dict:
    out = {"_generator": "tests/golden/make_vectors.py", "_seed": SEED, "encode": [], "reconst": {},
           "update": [], "replace": []}
    for d, p in ENCODE_SHAPES:
        for size in ENCODE_SIZES:
            v = stripe_data(d, size) + [np.zeros(size, np.uint8) for _ in range(p)]
            assert orc.encode(d, p, v) == 0
            e = {"d": d, "p": p, "size": size, "parity_sha256": sha(v[d:])}
            if size <= HEX_MAX:
                e["parity_hex"] = [x.tobytes().hex() for x in v[d:]]
            out["encode"].append(e)

    d, p, size = 10, 4, STRIPE_SIZE
    full = stripe_data(d, size) + [np.zeros(size, np.uint8) for _ in range(p)]
    assert orc.encode(d, p, full) == 0
    per, h = {}, hashlib.sha256()
    for lost in reconst_patterns(d + p):
        v = [x.copy() for x in full]
        for i in lost:
            v[i] = garbage(i, size)
        assert orc.reconst(d, p, v, [], lost) == 0
        rebuilt = [v[i] for i in lost]
        for x in rebuilt:
            h.update(x.tobytes())
        if len(lost) <= 2:
            per[",".join(map(str, lost))] = sha(rebuilt)
    out["reconst"] = {"d": d, "p": p, "size": size, "patterns": len(reconst_patterns(d + p)),
                      "all_sha256": h.hexdigest(), "per_pattern_sha256": per}

    for row in range(d):
        new = stream(1, row, size)
        par = [x.copy() for x in full[d:]]
        assert orc.update(d, p, full[row], new, row, par) == 0
        out["update"].append({"row": row, "parity_sha256": sha(par)})

    for rn in range(1, 7):
        rows = list(range(rn))
        par = [x.copy() for x in full[d:]]
        assert orc.replace(d, p, [full[i] for i in rows], rows, par) == 0
        out["replace"].append({"rn": rn, "rows": rows, "parity_sha256": sha(par)})
    return out


def main() -> int:
    sys.path.insert(0, ROOT)
    from oracle import oracle

    oracle.build()
    text = json.dumps(make(oracle), indent=1, sort_keys=True) + "\n"
    if "--check" in sys.argv:
        return 0 if open(OUT).read() == text else 1
    open(OUT, "w").write(text)
    return 0


if __name__ == "__main__":
    sys.exit(main())
