"""CPU: the oracle (clean-room C restatement) against the golden vectors the
compiled reference produced (tests/golden/golden.json), plus live checks
against the reference itself when oracle/_ref is built (this container)."""
import hashlib
import os

import numpy as np
import pytest

import datagen
import oracle
from golden_inputs import build_stream, make_input, random_ops

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HAVE_REF = os.path.exists(os.path.join(ROOT, "oracle", "_ref", "libsnappy_ref.so"))


def sha(b):
    return hashlib.sha256(b).hexdigest()


def test_golden_entries(golden):
    assert len(golden["entries"]) > 200
    for e in golden["entries"]:
        data = make_input(e["spec"])
        assert sha(data) == e["in_sha256"], e["name"]
        out = oracle.compress(data)
        assert len(out) == e["out_len"], e["name"]
        assert sha(out) == e["out_sha256"], e["name"]
        if "out_hex" in e:
            assert out.hex() == e["out_hex"]
        assert oracle.decompress(out) == data, e["name"]


def test_appendix_b_prefixes(golden):
    # SURVEY.md Appendix B, measured on the reference: sha256(out)[:16]
    want = {"abc": "70642598ff367aaa", "a_x20": "0ea0dc35bbe371aa", "hello": "b52b4c7bcf79946a",
            "zeros_1MiB": "f70b8f5b6dac7c3e", "iota64_1MiB": "4a0ab33443b1e544", "lcg1_1MiB": "fa34153ab8b0f4da",
            "license": "866fe1185146abb7", "license_1MiB": "57c1f99e662156b6", "license_65537": "8c6760518d96d4ab"}
    got = {e["name"]: e["out_sha256"][:16] for e in golden["entries"]}
    for k, v in want.items():
        assert got[k] == v, k


def test_decoder_vectors(golden):
    for v in golden["decoder_vectors"]:
        assert oracle.decompress(bytes.fromhex(v["stream_hex"])).hex() == v["out_hex"], v["name"]


def test_varint_kats(golden):
    import ctypes
    for k in golden["varint"]:
        buf = ctypes.create_string_buffer(16)
        n = oracle.orc().oracle_varint_encode(k["n"], buf)
        assert buf.raw[:n].hex() == k["hex"]


def test_streams_32k(golden):
    s = golden["streams_32k"]
    a = datagen.make("T", s["spec"]["size"], s["spec"]["seed"])
    assert sha(a.tobytes()) == s["in_sha256"]
    payload, offs = oracle.compress_streams(a, s["chunk"])
    assert payload.size == s["out_len"]
    assert sha(payload.tobytes()) == s["out_sha256"]
    assert sha(offs.astype(np.uint64).tobytes()) == s["offsets_sha256"]
    back = oracle.decompress_streams(payload, offs, a.size, s["chunk"])
    assert np.array_equal(back, a)


def test_text_ratio_band():
    # the synthetic "enwik8-like" text must sit in the survey's 1.7-2.0 band
    a = datagen.make("T", 8 << 20, 1234)
    out = oracle.compress(a.tobytes())
    assert 1.7 <= a.size / len(out) <= 2.0


def test_decoder_rejects_bad_streams():
    good = oracle.compress(b"abcdabcdabcdabcdabcdabcd")
    with pytest.raises(ValueError):
        oracle.decompress(good[:-3])  # truncated
    with pytest.raises(ValueError):
        oracle.decompress(bytes([8, 0]) + b"a" + bytes([(7 - 1) << 2 | 2, 9, 0]))  # offset beyond output


@pytest.mark.skipif(not HAVE_REF, reason="reference build only in the build container")
def test_oracle_matches_reference_live():
    rng = np.random.default_rng(5)
    for trial in range(40):
        n = int(rng.integers(0, 200000))
        kind = "TRPZ"[trial % 4]
        data = datagen.make(kind, n, trial).tobytes()
        if trial % 5 == 0 and n > 100:  # mixed text/random splices
            data = data[: n // 2] + datagen.make("R", n - n // 2, trial).tobytes()
        assert oracle.compress(data) == oracle.ref_compress(data)


def _xblock_stream(v):
    if "random" in v:
        r = v["random"]
        return build_stream(random_ops(r["seed"], r["n_out"], r["max_off"]))
    return build_stream(v["ops"])


def test_xblock_vectors(golden):
    # streams whose elements straddle 65,536-byte blocks and whose copies reach
    # into earlier blocks: the oracle decodes them exactly as the reference did
    assert len(golden["xblock_vectors"]) >= 15
    for v in golden["xblock_vectors"]:
        stream = _xblock_stream(v)
        assert len(stream) == v["stream_len"] and sha(stream) == v["stream_sha256"], v["name"]
        out = oracle.decompress(stream)
        assert len(out) == v["out_len"] and sha(out) == v["out_sha256"], v["name"]


@pytest.mark.skipif(not HAVE_REF, reason="reference build only in the build container")
def test_oracle_decoder_matches_reference_on_foreign_streams():
    for seed in range(100, 112):
        stream = build_stream(random_ops(seed, 150_000 + 37_000 * (seed % 5), 131072))
        n = len(oracle.decompress(stream))
        assert oracle.decompress(stream) == oracle.ref_decompress(stream, n)


def test_parallel_stream_equals_serial(golden):
    """compress_parallel (blocks on threads: the checker of the multi-GiB GPU
    streams) gives the reference's bytes on every golden entry, and compress()'s on
    multi-block text, random and repeat inputs with ragged ends."""
    for e in golden["entries"]:  # the reference's own outputs
        data = np.frombuffer(make_input(e["spec"]), np.uint8).copy()
        assert sha(oracle.compress_parallel(data, threads=4).tobytes()) == e["out_sha256"], e["name"]
    for kind, n in (("T", (5 << 20) + 12345), ("R", 3 << 20), ("P", (2 << 20) + 1), ("T", 65536), ("T", 1)):
        a = datagen.make(kind, n, 7)
        assert oracle.compress_parallel(a, threads=8).tobytes() == oracle.compress(a.tobytes()), (kind, n)
    assert oracle.compress_parallel(np.empty(0, np.uint8)).size == 0


DIGEST_T1234_5G = "4217993e6c71c372"  # bytes [5 GiB, 5 GiB + 3 MiB) of T seed 1234 (bench.py's text)
DIGEST_T4321 = "6a90134750bb6f50"  # the first 2 MiB of T seed 4321 (decode10g's tile)


def test_datagen_text_known_digests():
    """The text generator is pinned: bench inputs on the GPU box (and every
    measurement in profiles/) are these bytes."""
    a = np.empty(3 << 20, dtype=np.uint8)
    datagen.fill(a, "T", 1234, offset=5 << 30, threads=4)
    b = datagen.make("T", 2 << 20, 4321)
    assert hashlib.sha256(a.tobytes()).hexdigest()[:16] == DIGEST_T1234_5G
    assert hashlib.sha256(b.tobytes()).hexdigest()[:16] == DIGEST_T4321
