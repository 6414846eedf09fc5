#!/usr/bin/env python3
"""Extract the reference's own table data into binary test fixtures.

Run in the build container (where /root/reference exists); the outputs are
committed under tests/golden/ so the GPU box never reads /root/reference.

Fixtures written (pure data — inputs/expected outputs, no source text):
  ref_inverse_tbl.bin   256 B    gftbl.go:12  inverseTbl
  ref_mul_tbl.bin       65536 B  gftbl.go:14  mulTbl[256][256]
  ref_low_high_tbl.bin  8192 B   gftbl.go:16  lowHighTbl
  isal_mul_tbl.bin      65536 B  gftbl_test.go:56 intelMulTbl (ISA-L gf_mul table)
"""
import os
import re
import sys

REF = "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden")
HEX = re.compile(r"0x[0-9a-fA-F]+")


def var_bytes(text: str, name: str) -> bytes:
    m = re.search(r"var\s+" + name + r"\s*=", text)
    if not m:
        raise SystemExit(f"{name} not found")
    start = text.index("{", m.end())
    depth, i = 0, start
    while True:
        c = text[i]
        if c == "{":
            depth += 1
        elif c == "}":
            depth -= 1
            if depth == 0:
                break
        i += 1
    return bytes(int(h, 16) for h in HEX.findall(text[start:i + 1]))


def main() -> int:
    if not os.path.isdir(REF):
        print("reference not present; fixtures are already committed", file=sys.stderr)
        return 0
    os.makedirs(OUT, exist_ok=True)
    tbl = open(os.path.join(REF, "gftbl.go")).read()
    tst = open(os.path.join(REF, "gftbl_test.go")).read()
    items = {
        "ref_inverse_tbl.bin": (var_bytes(tbl, "inverseTbl"), 256),
        "ref_mul_tbl.bin": (var_bytes(tbl, "mulTbl"), 65536),
        "ref_low_high_tbl.bin": (var_bytes(tbl, "lowHighTbl"), 8192),
        "isal_mul_tbl.bin": (var_bytes(tst, "intelMulTbl"), 65536),
    }
    for fn, (data, size) in items.items():
        assert len(data) == size, (fn, len(data))
        with open(os.path.join(OUT, fn), "wb") as f:
            f.write(data)
        print(f"wrote {fn} ({len(data)} B)")
    return 0


if __name__ == "__main__":
    sys.exit(main())
