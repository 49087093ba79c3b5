"""CPU: the -b mode (snappy_compress_bst, src/snappy_compression_tree.c:291-306
with the BST matcher src/BST.c:30-82) as libsnappy_amd.so computes it on host
threads (csrc/bst_host.c).  Pinned by tests/golden/golden_bst.json, every
output of which the compiled reference wrote (oracle/gen_golden.py bst), and
live against oracle/_ref where it is present.  No kernel is launched here:
the -b stream's round trip through the GPU decoder is in test_gpu_parity.py."""
import hashlib
import os
import subprocess
import tempfile

import pytest

import datagen
import snappy_amd
from golden_inputs import make_input

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden", "golden_bst.json")
EXE = os.path.join(ROOT, "lightweight-snappy_amd", "snappy")


def sha(b):
    return hashlib.sha256(b).hexdigest()


@pytest.fixture(scope="module")
def golden_bst():
    import json
    with open(GOLD) as f:
        return json.load(f)


def test_golden_bst_entries(golden_bst):
    assert len(golden_bst["entries"]) >= 200
    for e in golden_bst["entries"]:
        data = make_input(e["spec"])
        assert sha(data) == e["in_sha256"], e["name"]
        got = snappy_amd.compress_bst(data)
        assert len(got) == e["out_len"] and sha(got) == e["out_sha256"], e["name"]
        if "out_hex" in e:
            assert got.hex() == e["out_hex"], e["name"]


@pytest.mark.parametrize("threads", ["1", "3", "16"])
def test_bst_thread_count_invariant(threads, golden_bst):
    # blocks are independent: any number of host threads writes the same bytes
    e = next(x for x in golden_bst["entries"] if x["name"] == "text_3MiB")
    data = make_input(e["spec"])
    env = dict(os.environ, SNAPPY_AMD_BST_THREADS=threads)
    code = ("import sys, hashlib; sys.path[:0] = [%r, %r]; import snappy_amd; from golden_inputs import make_input;"
            "print(hashlib.sha256(snappy_amd.compress_bst(make_input(%r))).hexdigest())"
            % (os.path.join(ROOT, "lightweight-snappy_amd"), os.path.join(ROOT, "tests"), e["spec"]))
    r = subprocess.run(["python3", "-c", code], env=env, capture_output=True, text=True, check=True)
    assert r.stdout.strip() == e["out_sha256"]
    assert len(data) == e["in_len"]


def test_bst_multi_chunk_against_reference():
    # more than one 32 MiB read of the FILE* path and a ragged tail, against
    # the compiled reference where it exists (else the buffer API's own bytes,
    # which the golden set pins)
    data = (datagen.make("T", (40 << 20) + 4321, 77).tobytes() + datagen.make("R", 3 << 20, 78).tobytes())
    buf = snappy_amd.compress_bst(data)
    ref_so = os.path.join(ROOT, "oracle", "_ref", "libsnappy_ref.so")
    if os.path.exists(ref_so):
        import oracle
        assert buf == oracle.ref_compress_bst(data)
    with tempfile.TemporaryDirectory() as d:
        src, out = os.path.join(d, "in"), os.path.join(d, "in.snp")
        open(src, "wb").write(data)
        subprocess.run([EXE, "-b", src, out], check=True, capture_output=True)
        assert open(out, "rb").read() == buf


def test_bst_cli_golden_and_empty(golden_bst):
    e = next(x for x in golden_bst["entries"] if x["name"] == "text_1000000")
    with tempfile.TemporaryDirectory() as d:
        src, out = os.path.join(d, "in"), os.path.join(d, "in.snp")
        open(src, "wb").write(make_input(e["spec"]))
        subprocess.run([EXE, "-b", src, out], check=True, capture_output=True)
        assert sha(open(out, "rb").read()) == e["out_sha256"]
        open(src, "wb").write(b"")
        subprocess.run([EXE, "-b", src, out], check=True, capture_output=True)
        assert open(out, "rb").read() == b""  # no block: not even the preamble (as the reference)
    # -b writes no block index
    assert subprocess.run([EXE, "-b", "-i", "x", "y"], capture_output=True).returncode != 0


@pytest.mark.skipif(not os.path.exists(os.path.join(ROOT, "oracle", "_ref", "libsnappy_ref.so")),
                    reason="the compiled reference exists only in the build container")
def test_bst_live_against_reference():
    import oracle
    for kind, n, seed in [("T", 5 << 20, 11), ("L", 1 << 20, 3), ("P", 2 << 20, 4), ("Z", 300000, 0),
                          ("R", 70000, 9)]:
        data = datagen.make(kind, n, seed).tobytes()
        assert snappy_amd.compress_bst(data) == oracle.ref_compress_bst(data), (kind, n)
