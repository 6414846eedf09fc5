"""Build provenance: the library names the sources it was built from.

reedsolomon_amd/build.py stamps SHA-256 of the sources and flags into
librsamd.so (rs_build_id); a rebuild is due exactly when that stamp differs
from the tree's digest (not on file times, which a snapshot copy resets).
CPU only: the library is loaded, no device call is made.
"""
import os
import shutil

import pytest

from reedsolomon_amd import build as B


def test_loaded_library_matches_tree():
    import reedsolomon_amd as rs

    info = rs.build_info()
    assert len(info["build_id"]) == 64
    assert info["build_id"] == B.library_digest(B.LIB)
    assert info["matches_tree"], info
    assert not B.needs_build()


def test_flipping_one_source_byte_requires_a_rebuild(tmp_path):
    # Work on a copy of the sources (never on the tree itself: other test
    # processes may be loading the library): flip one byte, the digest moves
    # and needs_build() says so; restore it and the stamp matches again.
    deps = []
    for p in B.DEPS + [os.path.abspath(B.__file__)]:
        q = tmp_path / os.path.basename(p)
        shutil.copyfile(p, q)
        deps.append(str(q))
    base = B.source_digest(deps)
    target = next(q for q in deps if q.endswith("kernels.hip"))
    with open(target, "rb") as f:
        data = bytearray(f.read())
    orig = data[100]
    data[100] ^= 0x01
    with open(target, "wb") as f:
        f.write(data)
    assert B.source_digest(deps) != base
    fake_lib = tmp_path / "lib.so"
    fake_lib.write_bytes(b"\x7fELF...." + b"RSAMD_BUILD_ID=" + base.encode() + b"\0tail")
    assert B.library_digest(str(fake_lib)) == base
    assert B.needs_build(str(fake_lib), deps=deps, experiments=False)
    data[100] = orig
    with open(target, "wb") as f:
        f.write(data)
    assert B.source_digest(deps) == base
    assert not B.needs_build(str(fake_lib), deps=deps, experiments=False)


def test_flags_are_part_of_the_digest():
    assert B.source_digest(experiments=False) != B.source_digest(experiments=True)


@pytest.mark.parametrize("blob", [b"", b"no stamp here", b"RSAMD_BUILD_ID=unstamped\0"])
def test_unstamped_library_needs_build(tmp_path, blob):
    lib = tmp_path / "x.so"
    lib.write_bytes(blob)
    assert B.library_digest(str(lib)) is None
    assert B.needs_build(str(lib))
