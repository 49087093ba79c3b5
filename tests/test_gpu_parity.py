"""GPU parity: the HIP path (through the C ABI) against the golden vectors of
the compiled reference and against the oracle on the same seeded inputs.
Integer/byte work: the bar is bit-exact."""
import hashlib
import os
import subprocess
import tempfile

import numpy as np
import pytest

import datagen
import oracle
import snappy_amd
from golden_inputs import build_stream, make_input, random_ops

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def sha(b):
    return hashlib.sha256(b).hexdigest()


def progress(msg: str) -> None:
    """Long tests note their progress in $SNAPPY_TEST_PROGRESS (tools/gpu_session.sh
    points it under gpurun_out/, so a slow test is not taken for a silent hang)."""
    path = os.environ.get("SNAPPY_TEST_PROGRESS")
    if path:
        with open(path, "a") as f:
            f.write(msg + "\n")


def to_dev(a: np.ndarray):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def test_golden_entries_host_api(golden):
    for e in golden["entries"]:
        data = make_input(e["spec"])
        out = snappy_amd.compress(data)
        assert len(out) == e["out_len"], e["name"]
        assert sha(out) == e["out_sha256"], e["name"]
        assert snappy_amd.decompress(out) == data, e["name"]


def test_decoder_vectors(golden):
    for v in golden["decoder_vectors"]:
        assert snappy_amd.decompress(bytes.fromhex(v["stream_hex"])).hex() == v["out_hex"], v["name"]


def test_single_layout_device(codec):
    for kind, n, seed in [("T", 3 << 20, 99), ("R", 1 << 20, 1), ("P", 1 << 20, 2), ("T", 1000000, 1234),
                          ("Z", 200001, 0), ("T", 65536 * 5 + 17, 4)]:
        a = datagen.make(kind, n, seed)
        comp, offs = codec.compress_tensor(to_dev(a), layout=snappy_amd.SINGLE)
        want = oracle.compress(a.tobytes())
        assert comp.cpu().numpy().tobytes() == want, (kind, n)
        back = codec.decompress_tensor(comp, offs, n, layout=snappy_amd.SINGLE)
        assert np.array_equal(back.cpu().numpy(), a)


def test_streams_32k_device(codec, golden):
    s = golden["streams_32k"]
    a = datagen.make("T", s["spec"]["size"], s["spec"]["seed"])
    comp, offs = codec.compress_tensor(to_dev(a), chunk=s["chunk"], layout=snappy_amd.STREAMS)
    assert comp.numel() == s["out_len"]
    assert sha(comp.cpu().numpy().tobytes()) == s["out_sha256"]
    assert sha(offs.cpu().numpy().astype(np.uint64).tobytes()) == s["offsets_sha256"]
    back = codec.decompress_tensor(comp, offs, a.size, chunk=s["chunk"], layout=snappy_amd.STREAMS)
    assert np.array_equal(back.cpu().numpy(), a)


@pytest.mark.parametrize("chunk", [1, 17, 4096, 32768, 65535, 65536])
def test_streams_chunk_sizes(codec, chunk):
    n = 300000 if chunk > 16 else 2000
    a = datagen.make("T", n, chunk)
    comp, offs = codec.compress_tensor(to_dev(a), chunk=chunk, layout=snappy_amd.STREAMS)
    want, want_offs = oracle.compress_streams(a, chunk)
    assert comp.cpu().numpy().tobytes() == want.tobytes()
    assert np.array_equal(offs.cpu().numpy().astype(np.uint64), want_offs)
    back = codec.decompress_tensor(comp, offs, n, chunk=chunk, layout=snappy_amd.STREAMS)
    assert np.array_equal(back.cpu().numpy(), a)


def test_reference_stream_index_and_decode(codec, golden):
    # a reference-produced .snp has no block index: K5 builds it on the GPU
    import torch
    for name in ("text_3MiB", "license_1MiB", "random_1MiB", "edge_T_131073", "zeros_1MiB"):
        e = next(x for x in golden["entries"] if x["name"] == name)
        data = make_input(e["spec"])
        stream = oracle.compress(data)  # == reference bytes (pinned by test_oracle)
        assert sha(stream) == e["out_sha256"]
        d = torch.from_numpy(np.frombuffer(stream, dtype=np.uint8).copy()).cuda()
        n, offs = codec.index_tensor(d)
        assert n == len(data)
        back = codec.decompress_tensor(d, offs, n, layout=snappy_amd.SINGLE)
        assert back.cpu().numpy().tobytes() == data


def test_decoder_errors():
    good = oracle.compress(datagen.make("T", 5000, 1).tobytes())
    with pytest.raises(snappy_amd.SnappyError) as ei:
        snappy_amd.decompress(good[:-5])
    assert ei.value.code in (snappy_amd.ERR_TRUNCATED, snappy_amd.ERR_OVERRUN)
    bad_off = bytes([8, 0]) + b"a" + bytes([(7 - 1) << 2 | 2, 9, 0])
    with pytest.raises(snappy_amd.SnappyError) as ei:
        snappy_amd.decompress(bad_off)
    assert ei.value.code == snappy_amd.ERR_OFFSET
    with pytest.raises(snappy_amd.SnappyError):
        snappy_amd.decompress(b"\x80\x80\x80")


def test_empty_and_tiny():
    assert snappy_amd.compress(b"") == b""
    assert snappy_amd.decompress(b"") == b""
    for n in range(0, 40):
        data = bytes((i * 37) % 5 for i in range(n))
        out = snappy_amd.compress(data)
        assert out == oracle.compress(data)
        assert snappy_amd.decompress(out) == data


def test_file_api_header_quirk():
    import io
    data = datagen.make("T", 100000, 3).tobytes()
    fo = io.BytesIO()
    snappy_amd.snappy_compress(io.BytesIO(data), 123456789, fo)  # header = the caller's input_size
    assert fo.getvalue()[:4] == snappy_amd.varint_encode(123456789)
    assert fo.getvalue()[4:] == oracle.compress(data)[3:]
    fo2 = io.BytesIO()
    snappy_amd.snappy_compress(io.BytesIO(b""), 10, fo2)  # empty read -> nothing written
    assert fo2.getvalue() == b""


def test_gpu_library_is_a_product_build():
    """The library these GPU tests load (SNAPPY_AMD_LIB may point elsewhere)
    reports product knobs for both kernel halves (test_abi.assert_product_config)."""
    from test_abi import assert_product_config
    assert_product_config(snappy_amd.build_config())


def golden_bst():
    import json
    with open(os.path.join(ROOT, "tests", "golden", "golden_bst.json")) as f:
        return json.load(f)


def test_cli_round_trip(golden):
    exe = os.path.join(ROOT, "lightweight-snappy_amd", "snappy")
    e = next(x for x in golden["entries"] if x["name"] == "text_1000000")
    data = make_input(e["spec"])
    with tempfile.TemporaryDirectory() as d:
        src, snp, dec = (os.path.join(d, x) for x in ("in", "in.snp", "in.dec"))
        open(src, "wb").write(data)
        subprocess.run([exe, "-c", "-r", src, snp], check=True, capture_output=True)
        assert sha(open(snp, "rb").read()) == e["out_sha256"]
        subprocess.run([exe, "-d", snp, dec], check=True, capture_output=True)
        assert open(dec, "rb").read() == data
        # -b: the reference's BST-matcher stream (host threads), decoded on the GPU
        eb = next(x for x in golden_bst()["entries"] if x["name"] == "text_1000000")
        subprocess.run([exe, "-b", src, snp], check=True, capture_output=True)
        assert sha(open(snp, "rb").read()) == eb["out_sha256"]
        subprocess.run([exe, "-d", snp, dec], check=True, capture_output=True)
        assert open(dec, "rb").read() == data


def test_cli_streaming_multi_chunk():
    """snappy_compress(FILE*) streams 64 MiB chunks through two pipeline slots:
    a 150 MiB mixed input (text, random, zeros; not a multiple of 65,536) must
    come out byte-identical to the one-shot reference stream."""
    exe = os.path.join(ROOT, "lightweight-snappy_amd", "snappy")
    data = np.concatenate([datagen.make("T", 70 << 20, 41), datagen.make("R", 30 << 20, 42),
                           np.zeros(10 << 20, np.uint8), datagen.make("T", (40 << 20) + 12345, 43)]).tobytes()
    want = oracle.compress(data)
    with tempfile.TemporaryDirectory() as d:
        src, snp, dec = (os.path.join(d, x) for x in ("in", "in.snp", "in.dec"))
        open(src, "wb").write(data)
        subprocess.run([exe, "-c", src, snp], check=True, capture_output=True)
        got = open(snp, "rb").read()
        assert len(got) == len(want) and got == want
        subprocess.run([exe, "-d", snp, dec], check=True, capture_output=True)
        assert open(dec, "rb").read() == data


DROPIN = os.path.join(ROOT, "oracle", "_ref", "snappy_dropin")


@pytest.mark.skipif(not os.path.exists(DROPIN), reason="oracle/_ref/snappy_dropin is built by build() where "
                                                       "/root/reference exists and travels with the tree")
def test_reference_cli_dropin(golden):
    """The reference's own src/cmd.c (with IO_utils.c and result.c), unchanged,
    linked against libsnappy_amd.so (oracle/Makefile `snappy_dropin`) and run
    on the GPU: -c of configs[0]'s 1,000,000-byte text gives the reference's
    golden bytes, -d restores it; the 150 MiB mixed file (three 64 MiB
    pipeline chunks) comes out equal to the one-shot reference stream and
    round-trips; -b writes the reference's BST-matcher bytes.  src/cmd.c:86-98
    calls snappy_compress / snappy_compress_bst / snappy_decompress."""
    e = next(x for x in golden["entries"] if x["name"] == "text_1000000")
    one = make_input(e["spec"])
    mixed = np.concatenate([datagen.make("T", 70 << 20, 41), datagen.make("R", 30 << 20, 42),
                            np.zeros(10 << 20, np.uint8), datagen.make("T", (40 << 20) + 12345, 43)]).tobytes()
    with tempfile.TemporaryDirectory() as d:
        for name, data, want_sha in (("text_1000000", one, e["out_sha256"]), ("mixed_150MiB", mixed, None)):
            src, snp, dec = (os.path.join(d, f"{name}{x}") for x in ("", ".snp", ".dec"))
            open(src, "wb").write(data)
            r = subprocess.run([DROPIN, "-c", "-r", src, snp], capture_output=True, text=True, timeout=120)
            assert r.returncode == 0, r.stderr
            assert "MB/s" in r.stdout  # src/result.c's report: the reference CLI ran to its end
            got = open(snp, "rb").read()
            if want_sha:
                assert sha(got) == want_sha, name
            else:
                assert got == oracle.compress(data), name
            r = subprocess.run([DROPIN, "-d", "-r", snp, dec], capture_output=True, text=True, timeout=120)
            assert r.returncode == 0, r.stderr
            assert open(dec, "rb").read() == data, name
            progress(f"dropin {name}: ok")
        # src/cmd.c:93-94: -b calls snappy_compress_bst; the reference's -b bytes
        eb = next(x for x in golden_bst()["entries"] if x["name"] == "text_1000000")
        src, snp, dec = (os.path.join(d, f"bst{x}") for x in ("", ".snp", ".dec"))
        open(src, "wb").write(one)
        r = subprocess.run([DROPIN, "-b", src, snp], capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr
        assert sha(open(snp, "rb").read()) == eb["out_sha256"]
        r = subprocess.run([DROPIN, "-d", snp, dec], capture_output=True, text=True, timeout=120)
        assert r.returncode == 0 and open(dec, "rb").read() == one, r.stderr


def test_full_size_streams_1gib(codec):
    """BASELINE.json configs[1] at full size: 1 GiB of 32 KiB text streams,
    bit-exact against the (threaded) oracle and round-tripped on the GPU."""
    import torch
    n, chunk = 1 << 30, 32768
    a = datagen.make("T", n, 1234)
    comp, offs = codec.compress_tensor(to_dev(a), chunk=chunk, layout=snappy_amd.STREAMS)
    want, want_offs = oracle.compress_streams(a, chunk, threads=16)
    got = comp.cpu().numpy()
    assert got.size == want.size
    assert np.array_equal(offs.cpu().numpy().astype(np.uint64), want_offs)
    assert np.array_equal(got, want)
    back = codec.decompress_tensor(comp, offs, n, chunk=chunk, layout=snappy_amd.STREAMS)
    assert torch.equal(back, to_dev(a))


@pytest.mark.timeout(900)
def test_config3_64gib_full_stream(codec):
    """BASELINE configs[3] at its full size on one GPU: 64 GiB of 32 KiB text
    streams, generated as bench.py generates them (kind T, seed 1234, by
    offset) and compressed in bench.py's 8 GiB pieces.  Every unit offset and
    every byte of the 64 GiB compressed stream are checked against the oracle
    (per GiB: the oracle's payload by 128-bit xxh3 digest, its 32,768 stream
    offsets exactly), and every piece round-trips on the GPU."""
    import torch
    import xxhash
    GiB, C = 1 << 30, 32768
    n, piece, per = 64 * GiB, 8 * GiB, GiB // C
    torch.cuda.empty_cache()
    x = torch.empty(n, dtype=torch.uint8, device="cuda")
    host = np.empty(GiB, dtype=np.uint8)
    want_dig, want_offs = [], []
    for o in range(0, n, GiB):
        datagen.fill(host, "T", 1234, offset=o, threads=16)
        x[o:o + GiB].copy_(torch.from_numpy(host))
        w, wo = oracle.compress_streams(host, C, threads=16)
        want_dig.append(xxhash.xxh3_128_digest(w))
        want_offs.append(wo)
        del w
        progress(f"config3: oracle {o // GiB + 1} / 64 GiB")
    del host
    out = torch.empty(codec.max_output(piece, C, snappy_amd.STREAMS), dtype=torch.uint8, device="cuda")
    offs = torch.empty(piece // C + 1, dtype=torch.int64, device="cuda")
    back = torch.empty(piece, dtype=torch.uint8, device="cuda")
    total = 0
    for p0 in range(0, n, piece):
        clen = codec.compress_ptr_ex(x.data_ptr() + p0, piece, C, snappy_amd.STREAMS, 0, n, out.data_ptr(),
                                     offs.data_ptr())
        ho = offs.cpu().numpy().astype(np.uint64)
        assert int(ho[-1]) == clen
        for k in range(piece // GiB):
            g, u0, u1 = p0 // GiB + k, k * per, (k + 1) * per
            assert np.array_equal(ho[u0:u1 + 1] - ho[u0], want_offs[g]), g
            assert xxhash.xxh3_128_digest(out[int(ho[u0]):int(ho[u1])].cpu().numpy()) == want_dig[g], g
        codec.decompress_ptr_ex(out.data_ptr(), offs.data_ptr(), piece, C, snappy_amd.STREAMS, 0, n,
                                back.data_ptr())
        assert torch.equal(back, x[p0:p0 + piece]), p0
        total += clen
        progress(f"config3: piece at {p0 // GiB} GiB checked")
    assert 1.75 < n / total < 1.9
    del x, out, back
    torch.cuda.empty_cache()


def test_timings_before_any_launch_leave_no_pending_error():
    """A context that has timed nothing yet (bench.py --overlap's decode codec
    before its first decode) reads its timings, then another context on the
    same thread compresses and decodes: the launch-error checks must report
    only their own launches' errors (round 4: an elapsed time of an unrecorded
    event stayed pending and failed the next compress as a HIP error)."""
    import torch
    idle = snappy_amd.Codec(0)
    idle.enable_timing(True)
    assert idle.last_timings() == (0.0, 0.0, 0.0)
    c = snappy_amd.Codec(0)
    c.enable_timing(True)
    a = datagen.make("T", 1 << 20, 5)
    x = to_dev(a)
    comp, offs = c.compress_tensor(x, chunk=32768, layout=snappy_amd.STREAMS)
    idle.last_timings()
    back = c.decompress_tensor(comp, offs, x.numel(), chunk=32768, layout=snappy_amd.STREAMS)
    assert torch.equal(back, x)
    k1, k3, k4 = c.last_timings()
    assert k1 > 0 and k3 > 0 and k4 > 0


def test_default_stream_ordering(codec):
    """A tensor written on torch's default stream (the legacy null stream, which
    the binding maps to the context's own stream) is compressed only after that
    write: a long spin kernel, then the copy, then compress_tensor at once.
    (With a non-blocking own stream the compress raced the copy: round 3's
    decode10g test compressed half-written input.)"""
    import torch
    assert torch.cuda.current_stream().cuda_stream == 0
    a = datagen.make("T", 64 << 20, 99)
    src = to_dev(a)
    x = torch.zeros_like(src)
    torch.cuda.synchronize()
    torch.cuda._sleep(200_000_000)  # ~0.1 s on the default stream
    x.copy_(src)
    comp, offs = codec.compress_tensor(x, chunk=32768, layout=snappy_amd.STREAMS)
    want, _ = oracle.compress_streams(a, 32768, threads=16)
    assert np.array_equal(comp.cpu().numpy(), want)


@pytest.mark.parametrize("kind,seed", [("R", 1), ("P", 2)])
def test_full_size_extremes_1gib(codec, kind, seed):
    """configs[2]: 1 GiB random (all-literal) and 64-byte repeat (all-copy),
    one SINGLE stream each, bit-exact over the whole stream against the oracle
    (its blocks compressed on 16 host threads) and round-tripped."""
    import torch
    n = 1 << 30
    a = datagen.make(kind, n, seed)
    comp, offs = codec.compress_tensor(to_dev(a), layout=snappy_amd.SINGLE)
    if kind == "R":
        assert 0.9999 < n / comp.numel() < 1.0  # ~every block one 65,536-byte literal
    else:
        assert 20.0 < n / comp.numel() < 21.5
    want = oracle.compress_parallel(a, threads=16)
    assert np.array_equal(comp.cpu().numpy(), want)
    back = codec.decompress_tensor(comp, offs, n, layout=snappy_amd.SINGLE)
    assert torch.equal(back, to_dev(a))


def _index_both(codec, d):
    """(code, n, offsets) from the chunk-parallel K5p and from the serial K5."""
    res = []
    for serial in (False, True):
        codec.set_option(snappy_amd.OPT_SERIAL_INDEX, int(serial))
        try:
            n, offs = codec.index_tensor(d)
            res.append((0, n, offs.cpu().numpy().copy()))
        except snappy_amd.SnappyError as e:
            res.append((e.code, None, None))
        finally:
            codec.set_option(snappy_amd.OPT_SERIAL_INDEX, 0)
    return res


def test_parallel_index_matches_serial_and_compressor(codec):
    # K5p (chunk-parallel boundary finder) vs the serial K5 walk vs the block
    # index the compressor itself produced, on streams whose elements cross
    # chunk edges in every way: text, all-literal (65,536-byte literals span
    # four chunks), all-copy, and a mix with zero runs
    rng = np.random.default_rng(5)
    mixed = np.concatenate([datagen.make("T", 3 << 20, 9), datagen.make("R", 1 << 20, 3),
                            np.zeros(777_777, np.uint8), datagen.make("P", 1 << 20, 4),
                            rng.integers(0, 4, 500_001, dtype=np.uint8), datagen.make("T", 2 << 20, 10)])
    for a in (datagen.make("T", 24 << 20, 21), datagen.make("R", 6 << 20, 1), datagen.make("P", 6 << 20, 2), mixed):
        x = to_dev(a)
        comp, offs = codec.compress_tensor(x, chunk=snappy_amd.BLOCK, layout=snappy_amd.SINGLE)
        want = offs.cpu().numpy()
        (c1, n1, o1), (c2, n2, o2) = _index_both(codec, comp)
        assert c1 == 0 and c2 == 0
        assert n1 == n2 == a.size
        assert np.array_equal(o1, want) and np.array_equal(o2, want)


def test_parallel_index_chains_that_never_converge(codec):
    """K5a's per-lane fallback: a stream of 2-byte copy-1 elements (01 01: length 4,
    offset 1) parses as a valid element at EVERY byte, so the chains entered at even
    and odd bytes of a chunk never meet; likewise 3-byte copy-2 elements whose
    offset bytes are again valid copy-2 tags (period 3).  Index = serial walk, and
    the decode equals the oracle's."""
    import torch
    lit = bytes(range(200)) * 3  # 600-byte literal: tag 61 << 2, length - 1 in 2 bytes
    for unit, elen, count in (((1, 1), 4, 3_000_000), ((2, 2, 2), 1, 2_000_000)):
        # 01 01: copy-1, length 4, offset 1; 02 02 02: copy-2, length 1, offset 514
        n = len(lit) + elen * count
        stream = snappy_amd.varint_encode(n) + bytes([61 << 2, 599 & 0xFF, 599 >> 8]) + lit + bytes(unit) * count
        want = oracle.decompress(stream)
        assert len(want) == n
        d = torch.from_numpy(np.frombuffer(stream, dtype=np.uint8).copy()).cuda()
        (c1, n1, o1), (c2, n2, o2) = _index_both(codec, d)
        assert c1 == c2 == 0 and n1 == n2 == n and np.array_equal(o1, o2)
        back = codec.decompress_tensor(d, torch.from_numpy(o1).cuda(), n1, layout=snappy_amd.SINGLE)
        assert back.cpu().numpy().tobytes() == want


def test_decode_dense_short_elements(codec):
    """K4 batches of up to three 64-position halves merge at most 64 elements and
    drop the rest (the next batch starts after the last kept one): a stream of
    2- and 3-byte elements -- 1-byte literals, copy-1 of 4-11 bytes and copy-2 of
    1-3 bytes at offsets 1-40 -- fills 64 lanes in every batch and puts most copy
    sources inside the same 64-byte pass.  Decoded as one SINGLE stream (K5p index
    + K4) and as the host API does it, both equal to the oracle's decode."""
    import torch
    from golden_inputs import SplitMix64
    rng = SplitMix64(2024)
    ops, total = [], 0
    while total < (3 << 20):
        r = rng.below(10)
        if r < 4 or total < 64:
            ops.append(["lit", 1, rng.below(1 << 30)])
            total += 1
        elif r < 8:
            ln = 4 + rng.below(8)
            ops.append(["copy", ln, 1 + rng.below(min(40, total)), 1])
            total += ln
        else:
            ln = 1 + rng.below(3)
            ops.append(["copy", ln, 1 + rng.below(min(40, total)), 2])
            total += ln
    stream = build_stream(ops)
    want = oracle.decompress(stream)
    assert len(want) == total
    assert snappy_amd.decompress(stream) == want
    d = torch.from_numpy(np.frombuffer(stream, dtype=np.uint8).copy()).cuda()
    n, offs = codec.index_tensor(d)  # K5p (chunk-parallel index)
    assert n == total
    back = codec.decompress_tensor(d, offs, total, layout=snappy_amd.SINGLE)
    assert back.cpu().numpy().tobytes() == want


def test_parallel_index_errors_match_serial(codec):
    import torch
    a = datagen.make("T", 6 << 20, 33)
    comp, _ = codec.compress_tensor(to_dev(a), chunk=snappy_amd.BLOCK, layout=snappy_amd.SINGLE)
    raw = comp.cpu().numpy()
    rng = np.random.default_rng(7)
    cases = [raw[:-1], raw[: raw.size // 2], raw[: raw.size - 70000]]
    for _ in range(6):  # byte flips in the middle: error or a different but consistent parse
        b = raw.copy()
        pos = rng.integers(1 << 16, raw.size - (1 << 16), 4)
        b[pos] ^= rng.integers(1, 255, 4, dtype=np.uint8)
        cases.append(b)
    for b in cases:
        d = torch.from_numpy(np.ascontiguousarray(b)).cuda()
        (c1, n1, o1), (c2, n2, o2) = _index_both(codec, d)
        assert c1 == c2
        if c1 == 0:
            assert n1 == n2 and np.array_equal(o1, o2)


def test_decoder_fuzz_corrupted_streams():
    """Corrupted / truncated / garbage streams through the host decoder (index walk +
    K4): never a crash or hang; whenever the GPU path accepts a stream its output is the
    oracle decoder's output for it."""
    rng = np.random.default_rng(2024)
    base = [oracle.compress(datagen.make(k, n, s).tobytes())
            for k, n, s in (("T", 5000, 1), ("T", 200_000, 2), ("R", 70_000, 3), ("P", 150_000, 4))]
    cases = []
    for b in base:
        a = np.frombuffer(b, dtype=np.uint8)
        for _ in range(25):
            c = a.copy()
            k = int(rng.integers(1, 6))
            pos = rng.integers(min(3, a.size - 1), a.size, k)
            c[pos] = rng.integers(0, 256, k, dtype=np.uint8)
            cases.append(c.tobytes())
        for cut in rng.integers(1, a.size, 10):
            cases.append(b[:int(cut)])
    for n in (17, 1000, 70_000):
        hdr = snappy_amd.varint_encode(n)
        cases.append(hdr + rng.integers(0, 256, n // 2, dtype=np.uint8).tobytes())
    accepted = rejected = 0
    for i, c in enumerate(cases):
        try:
            want = oracle.decompress(c)
        except ValueError:
            want = None
        try:
            got = snappy_amd.decompress(c)
        except snappy_amd.SnappyError:
            got = None
        # the GPU path accepts exactly the streams the oracle decoder accepts
        assert (got is None) == (want is None), (i, len(c))
        if got is None:
            rejected += 1
        else:
            accepted += 1
            assert got == want, i
    assert accepted >= 4 and rejected >= 4


def test_streams_decoder_fuzz_device(codec):
    """Byte flips in a STREAMS payload (index kept): the block-parallel decoder
    reports a per-unit error or decodes exactly what the oracle decodes for that unit."""
    import torch
    chunk = 32768
    a = datagen.make("T", 64 * chunk, 77)
    comp, offs = codec.compress_tensor(to_dev(a), chunk=chunk, layout=snappy_amd.STREAMS)
    raw = comp.cpu().numpy()
    o = offs.cpu().numpy().astype(np.int64)
    rng = np.random.default_rng(99)
    for trial in range(12):
        c = raw.copy()
        k = 40 if trial < 6 else 2  # many flips (some unit always breaks) or few (often all decode)
        pos = rng.integers(0, raw.size, k)
        c[pos] ^= rng.integers(1, 256, k, dtype=np.uint8)
        want = []
        for u in range(64):  # the oracle decodes unit u to exactly `chunk` bytes, or rejects it
            try:
                w = oracle.decompress(c[o[u]:o[u + 1]].tobytes())
                want.append(w if len(w) == chunk else None)
            except ValueError:
                want.append(None)
        d = torch.from_numpy(c).cuda()
        try:
            back = codec.decompress_tensor(d, offs, a.size, chunk=chunk, layout=snappy_amd.STREAMS)
            ok = True
        except snappy_amd.SnappyError:
            ok = False
        assert ok == all(w is not None for w in want), trial
        if ok:  # every unit decoded: each must equal the oracle's decode of that unit
            got = back.cpu().numpy()
            for u in range(64):
                assert got[u * chunk:(u + 1) * chunk].tobytes() == want[u]


def _xblock_stream(v):
    if "random" in v:
        r = v["random"]
        return build_stream(random_ops(r["seed"], r["n_out"], r["max_off"]))
    return build_stream(v["ops"])


def test_xblock_vectors_host_api(golden):
    """Streams the reference decodes whose elements straddle 65,536-byte blocks
    and whose copies reach into earlier blocks (golden outputs of the compiled
    reference): the drop-in decoder must produce the same bytes."""
    for v in golden["xblock_vectors"]:
        stream = _xblock_stream(v)
        assert sha(stream) == v["stream_sha256"], v["name"]
        out = snappy_amd.decompress(stream)
        assert len(out) == v["out_len"] and sha(out) == v["out_sha256"], v["name"]


def test_xblock_vectors_device_index(codec, golden):
    """Same vectors through the HBM API: the block index with straddle entries
    from both index builders (chunk-parallel K5p and serial K5), then the
    two-pass block decoder."""
    import torch
    for v in golden["xblock_vectors"]:
        stream = _xblock_stream(v)
        d = torch.from_numpy(np.frombuffer(stream, dtype=np.uint8).copy()).cuda()
        res = _index_both(codec, d)
        (c1, n1, o1), (c2, n2, o2) = res
        assert c1 == 0 and c2 == 0, v["name"]
        assert n1 == n2 == v["out_len"] and np.array_equal(o1, o2), v["name"]
        back = codec.decompress_tensor(d, torch.from_numpy(o1).cuda(), n1, layout=snappy_amd.SINGLE)
        assert sha(back.cpu().numpy().tobytes()) == v["out_sha256"], v["name"]


def test_foreign_streams_large(codec):
    """Seeded random foreign streams of 8-48 MiB (every block straddles and
    copies into its predecessors, a long pass-2 dependency chain), against the
    oracle decoder."""
    import torch
    for seed, n_out, max_off in [(301, 8 << 20, 131072), (302, 24 << 20, 65535), (303, 48 << 20, 1 << 20)]:
        stream = build_stream(random_ops(seed, n_out, max_off))
        want = oracle.decompress(stream)
        assert len(want) == n_out
        assert snappy_amd.decompress(stream) == want, seed
        d = torch.from_numpy(np.frombuffer(stream, dtype=np.uint8).copy()).cuda()
        n, offs = codec.index_tensor(d)
        back = codec.decompress_tensor(d, offs, n, layout=snappy_amd.SINGLE)
        assert back.cpu().numpy().tobytes() == want, seed


def test_decode10g_full_size(codec):
    """BASELINE configs[4] at full size: one SINGLE stream of >= 10 GB
    (18.5 GB of text, 282,000+ blocks, compressed in 8 GiB pieces as bench.py
    does), decoded in one K4 launch with a global block index whose
    compressed offsets pass 2^32.  The whole stream is bit-exact against the
    oracle and the whole decode equals the input."""
    import torch
    GiB, B = 1 << 30, 65536
    n = (18_500_000_000 // B) * B
    base = torch.from_numpy(datagen.make("T", GiB, 4321)).cuda()
    x = torch.empty(n, dtype=torch.uint8, device="cuda")
    for o in range(0, n, GiB):  # the text GiB tiled (decoder input variety is per block)
        m = min(GiB, n - o)
        x[o:o + m] = base[:m]
    del base
    piece = 8 * GiB
    out = torch.empty(sum(codec.max_output(min(piece, n - o), B, snappy_amd.SINGLE) for o in range(0, n, piece)),
                      dtype=torch.uint8, device="cuda")
    codec._bind_stream()
    idx, pos, clens = [], 0, []
    for o in range(0, n, piece):
        m = min(piece, n - o)
        offs = torch.empty(m // B + 2, dtype=torch.int64, device="cuda")
        clen = codec.compress_ptr_ex(x.data_ptr() + o, m, B, snappy_amd.SINGLE, snappy_amd.NO_PREAMBLE if o else 0,
                                     n, out.data_ptr() + pos, offs.data_ptr())
        idx.append(offs[:(m + B - 1) // B] + pos)
        pos += clen
        clens.append(clen)
    idx = torch.cat(idx + [torch.tensor([pos], dtype=torch.int64, device="cuda")])
    assert pos >= 10_000_000_000 and idx.numel() == n // B + 1, (clens, float(x[:GiB].float().mean()))
    back = torch.empty(n, dtype=torch.uint8, device="cuda")
    codec.decompress_ptr(out.data_ptr(), idx.data_ptr(), n, B, snappy_amd.SINGLE, back.data_ptr())
    assert torch.equal(back, x)
    del back
    # the whole stream against the oracle: the input is one text GiB tiled, and
    # blocks are compressed independently, so tile t's blocks must be the bytes
    # of tile 0's (checked on the GPU) and tile 0 is the oracle's stream of that
    # GiB (checked on the host) with the preamble of n instead of 2^30
    hidx = idx.cpu().numpy()
    per, units = GiB // B, n // B
    hdr = snappy_amd.varint_encode(n)
    t0 = out[len(hdr):int(hidx[per])]
    for t in range(1, (n + GiB - 1) // GiB):
        u0, u1 = t * per, min((t + 1) * per, units)
        seg = out[int(hidx[u0]):int(hidx[u1])]
        ref = out[len(hdr):int(hidx[u1 - u0])]  # tile 0's first u1 - u0 blocks
        assert seg.numel() == ref.numel() and torch.equal(seg, ref), t
    base_h = np.empty(GiB, dtype=np.uint8)
    datagen.fill(base_h, "T", 4321, threads=16)
    want = oracle.compress_parallel(base_h, threads=16)
    hb = len(snappy_amd.varint_encode(GiB))
    assert np.array_equal(t0.cpu().numpy(), want[hb:])
    assert out[:len(hdr)].cpu().numpy().tobytes() == hdr


def _index_file(n, entries):
    import struct
    return struct.pack("<QQQ", snappy_amd.IDX_MAGIC, n, len(entries)) + struct.pack(f"<{len(entries)}Q", *entries)


def test_cli_sidecar_index():
    """`snappy -c -i` writes <out>.idx next to the stream (the
    streaming compressor's per-chunk indexes, shifted; 150 MiB = 3 pipeline
    chunks); it equals the index the GPU index pass builds, and `snappy -d -i`
    decodes with it.  An index of another stream is refused."""
    import torch
    exe = os.path.join(ROOT, "lightweight-snappy_amd", "snappy")
    data = np.concatenate([datagen.make("T", 90 << 20, 51), datagen.make("R", 40 << 20, 52),
                           datagen.make("T", (20 << 20) + 777, 53)]).tobytes()
    with tempfile.TemporaryDirectory() as d:
        src, snp, dec = (os.path.join(d, x) for x in ("in", "in.snp", "in.dec"))
        open(src, "wb").write(data)
        subprocess.run([exe, "-c", "-i", src, snp], check=True, capture_output=True)
        stream = open(snp, "rb").read()
        assert stream == oracle.compress(data)
        n, ent = snappy_amd.read_index(open(snp + ".idx", "rb").read())
        assert n == len(data)
        codec = snappy_amd.Codec(0)
        try:
            dn, offs = codec.index_tensor(torch.from_numpy(np.frombuffer(stream, dtype=np.uint8).copy()).cuda())
        finally:
            codec.close()
        assert dn == len(data) and ent == [int(v) for v in offs.cpu().numpy()]
        subprocess.run([exe, "-d", "-i", snp, dec], check=True, capture_output=True)
        assert open(dec, "rb").read() == data
        # a foreign index: refused, nothing decoded from it
        other = oracle.compress(data[:-1])
        open(snp, "wb").write(other)
        r = subprocess.run([exe, "-d", "-i", snp, dec], capture_output=True)
        assert r.returncode != 0


def test_decompress_with_sidecar_index_xblock(codec, golden):
    """A sidecar index with straddle entries (from the GPU index pass) drives
    the host decoder of the cross-block vectors."""
    import torch
    for v in golden["xblock_vectors"][:6]:
        stream = _xblock_stream(v)
        n, offs = codec.index_tensor(torch.from_numpy(np.frombuffer(stream, dtype=np.uint8).copy()).cuda())
        idx = _index_file(n, [int(x) for x in offs.cpu().numpy()])
        out = snappy_amd.decompress_indexed(stream, idx)
        assert sha(out) == v["out_sha256"], v["name"]


def test_index_misaligned_stream(codec):
    """K5p on a stream at an odd device address (a foreign buffer at any
    offset): the same index as at an aligned address, decoded bit-exact (the
    chunk-parallel path, not the one-wave serial fallback of round 2)."""
    import torch
    a = datagen.make("T", 24 << 20, 61)
    comp, offs = codec.compress_tensor(to_dev(a), layout=snappy_amd.SINGLE)
    clen = comp.numel()
    for shift in (1, 2, 3):
        buf = torch.zeros(clen + 8, dtype=torch.uint8, device="cuda")
        buf[shift:shift + clen] = comp
        got = torch.empty_like(offs)
        n = codec.index_ptr(buf.data_ptr() + shift, clen, got.data_ptr(), offs.numel())
        assert n == a.size and torch.equal(got, offs), shift
        back = torch.empty(a.size, dtype=torch.uint8, device="cuda")
        codec.decompress_ptr(buf.data_ptr() + shift, got.data_ptr(), n, snappy_amd.BLOCK, snappy_amd.SINGLE,
                             back.data_ptr())
        assert torch.equal(back.cpu(), torch.from_numpy(a)), shift
    # an index buffer one entry short is refused, not silently left without its last entry
    with pytest.raises(snappy_amd.SnappyError) as ei:
        codec.index_ptr(comp.data_ptr(), clen, got.data_ptr(), offs.numel() - 1)
    assert ei.value.code == snappy_amd.ERR_CAPACITY


def test_tampered_sidecar_index_refused(codec):
    """a sidecar index whose middle entries point past the stream
    or go backwards is refused with ERR_INDEX before any kernel reads it."""
    a = datagen.make("T", 3 << 20, 62)
    stream = oracle.compress(a.tobytes())
    _, offs = codec.compress_tensor(to_dev(a), layout=snappy_amd.SINGLE)
    ent = [int(v) for v in offs.cpu().numpy()]
    assert snappy_amd.decompress_indexed(stream, _index_file(a.size, ent)) == a.tobytes()
    for k, v in ((7, len(stream) + 4096), (20, ent[19] - 1), (1, 1 << 39)):
        bad = list(ent)
        bad[k] = v
        with pytest.raises(snappy_amd.SnappyError) as ei:
            snappy_amd.decompress_indexed(stream, _index_file(a.size, bad))
        assert ei.value.code == snappy_amd.ERR_INDEX, k
    with pytest.raises(snappy_amd.SnappyError) as ei:  # trailing bytes / short file
        snappy_amd.decompress_indexed(stream, _index_file(a.size, ent) + b"\0")
    assert ei.value.code == snappy_amd.ERR_INDEX
    # well-formed (in bounds, monotone) but not the stream's element boundaries:
    # an entry moved one byte into an element, either way, in the middle or at
    # the last block, is refused as ERR_INDEX, never decoded into other bytes
    for k, d in ((1, 1), (1, -1), (20, 1), (20, -1), (len(ent) - 2, 1), (len(ent) - 2, -1)):
        bad = list(ent)
        bad[k] += d
        with pytest.raises(snappy_amd.SnappyError) as ei:
            snappy_amd.decompress_indexed(stream, _index_file(a.size, bad))
        assert ei.value.code == snappy_amd.ERR_INDEX, (k, d)
    with pytest.raises(snappy_amd.SnappyError) as ei:
        snappy_amd.read_index(b"SNPA")
    assert ei.value.code == snappy_amd.ERR_INDEX


def test_device_index_past_stream_end_fails_cleanly(codec):
    """The HBM API trusts its index, but K4 never reads past the stream end the
    last entry names: a middle entry beyond it is a per-unit error, and the
    context decodes the next (good) stream normally."""
    import torch
    a = datagen.make("T", 4 << 20, 63)
    x = to_dev(a)
    comp, offs = codec.compress_tensor(x, layout=snappy_amd.SINGLE)
    bad = offs.clone()
    bad[3] = offs[-1] + (1 << 30)
    with pytest.raises(snappy_amd.SnappyError):
        codec.decompress_tensor(comp, bad, a.size, layout=snappy_amd.SINGLE)
    back = codec.decompress_tensor(comp, offs, a.size, layout=snappy_amd.SINGLE)
    assert torch.equal(back, x)
    # an entry moved forward inside an element: K4 itself refuses it (the
    # previous block's chain does not end there)
    bad = offs.clone()
    bad[5] += 1
    with pytest.raises(snappy_amd.SnappyError) as ei:
        codec.decompress_tensor(comp, bad, a.size, layout=snappy_amd.SINGLE)
    assert ei.value.code == snappy_amd.ERR_INDEX


@pytest.mark.parametrize("chunk", [17, 4095, 32768, 65535, 65536])
def test_any_alignment_long_literals_and_short_copies(codec, chunk):
    """K4's aligned-dword long-literal copy and its pass paths at every stream
    and output alignment: incompressible data (literals longer than the
    window) and short-period data (copies whose source lies in the same
    64-byte pass), decoded from a stream shifted by 0-3 bytes into an output
    shifted by 0-3 bytes; nothing outside the output may be written."""
    import torch
    layout = snappy_amd.SINGLE if chunk == 65536 else snappy_amd.STREAMS
    n = 3 * 65536 + 1234
    for kind, seed in (("R", 5), ("K", 7)):
        a = datagen.make(kind, n, seed, period=3) if kind == "K" else datagen.make(kind, n, seed)
        comp, offs = codec.compress_tensor(to_dev(a), chunk=chunk, layout=layout)
        c = comp.cpu().numpy()
        for s_in in range(4):
            d = torch.zeros(c.size + 8, dtype=torch.uint8, device="cuda")
            d[s_in:s_in + c.size] = comp
            for s_out in range(4):
                out = torch.full((n + 8,), 0xA5, dtype=torch.uint8, device="cuda")
                codec._bind_stream()  # torch's stream: the copies above are ordered before the decode
                codec.decompress_ptr(d.data_ptr() + s_in, offs.data_ptr(), n, chunk, layout, out.data_ptr() + s_out)
                torch.cuda.synchronize()
                got = out.cpu().numpy()
                assert np.array_equal(got[s_out:s_out + n], a), (kind, chunk, s_in, s_out)
                assert (got[:s_out] == 0xA5).all() and (got[s_out + n:] == 0xA5).all(), (kind, chunk, s_in, s_out)


def test_file_api_positions_and_pipes():
    """The FILE* entry points from arbitrary stream positions and through pipes
    (src/snappy_compression.h:8, src/snappy_decompression.h:15): compress a
    pipe into a regular file after a prefix, decode from an offset inside a
    file into a pipe, and decode from a pipe (the whole-read path); every
    output must equal the one-shot stream / the input, the FILE* positions
    must end where stdio leaves them, and the prefix must be untouched."""
    import ctypes
    libc = ctypes.CDLL(None)
    for fn, res, args in (("fopen", ctypes.c_void_p, [ctypes.c_char_p, ctypes.c_char_p]),
                          ("popen", ctypes.c_void_p, [ctypes.c_char_p, ctypes.c_char_p]),
                          ("fclose", ctypes.c_int, [ctypes.c_void_p]), ("pclose", ctypes.c_int, [ctypes.c_void_p]),
                          ("fseek", ctypes.c_int, [ctypes.c_void_p, ctypes.c_long, ctypes.c_int]),
                          ("ftell", ctypes.c_long, [ctypes.c_void_p]),
                          ("fwrite", ctypes.c_size_t, [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_void_p])):
        getattr(libc, fn).restype = res
        getattr(libc, fn).argtypes = args
    lib = snappy_amd.lib()
    data = np.concatenate([datagen.make("T", (9 << 20) + 777, 5), datagen.make("R", 3 << 20, 6)]).tobytes()
    want = oracle.compress(data)
    prefix = b"PREFIX-" * 1000
    with tempfile.TemporaryDirectory() as d:
        src, snp, dec, dec2 = (os.path.join(d, x) for x in ("in", "in.snp", "dec", "dec2"))
        open(src, "wb").write(data)
        # compress: a pipe in, a regular file out after a prefix
        fi = libc.popen(f"cat {src}".encode(), b"r")
        fo = libc.fopen(snp.encode(), b"wb")
        assert libc.fwrite(prefix, 1, len(prefix), fo) == len(prefix)
        lib.snappy_compress(ctypes.c_void_p(fi), ctypes.c_ulonglong(len(data)), ctypes.c_void_p(fo))
        assert lib.snappy_amd_last_status() == 0
        assert libc.ftell(fo) == len(prefix) + len(want)
        libc.pclose(fi)
        libc.fclose(fo)
        blob = open(snp, "rb").read()
        assert blob[:len(prefix)] == prefix and blob[len(prefix):] == want
        # decompress: from an offset inside the file, into a pipe
        fi = libc.fopen(snp.encode(), b"rb")
        assert libc.fseek(fi, len(prefix), 0) == 0
        fo = libc.popen(f"cat > {dec}".encode(), b"w")
        assert lib.snappy_decompress(ctypes.c_void_p(fi), ctypes.c_void_p(fo)) == 0
        assert libc.ftell(fi) == len(blob)
        libc.fclose(fi)
        assert libc.pclose(fo) == 0
        assert open(dec, "rb").read() == data
        # decompress: a pipe in (read whole), a regular file out after a prefix
        open(snp + ".raw", "wb").write(want)
        fi = libc.popen(f"cat {snp}.raw".encode(), b"r")
        fo = libc.fopen(dec2.encode(), b"wb")
        assert libc.fwrite(prefix, 1, len(prefix), fo) == len(prefix)
        assert lib.snappy_decompress(ctypes.c_void_p(fi), ctypes.c_void_p(fo)) == 0
        assert libc.ftell(fo) == len(prefix) + len(data)
        libc.pclose(fi)
        libc.fclose(fo)
        out = open(dec2, "rb").read()
        assert out[:len(prefix)] == prefix and out[len(prefix):] == data


def test_foreign_streams_many_seeds(codec):
    """Twenty more seeded foreign streams (1-3 MiB: literals of every header
    width, copies of every kind and distance, overlapping and in-pass copies,
    elements straddling blocks), decoded by the block-parallel path and by the
    drop-in host API, against the oracle decoder."""
    import torch
    for seed in range(401, 421):
        n_out = (1 << 20) + (seed * 104729) % (2 << 20)
        stream = build_stream(random_ops(seed, n_out, [64, 2048, 65535, 1 << 20][seed % 4], max_lit=[70, 700, 70000][seed % 3]))
        want = oracle.decompress(stream)
        assert len(want) == n_out
        d = torch.from_numpy(np.frombuffer(stream, dtype=np.uint8).copy()).cuda()
        n, offs = codec.index_tensor(d)
        back = codec.decompress_tensor(d, offs, n, layout=snappy_amd.SINGLE)
        assert back.cpu().numpy().tobytes() == want, seed
        assert snappy_amd.decompress(stream) == want, seed


def test_file_api_mapped_outputs():
    """The FILE* writers that map their output file (IoFile::map_out: outputs
    >= 64 MiB on a regular file): a file opened "wb" (write-only, so the mapping
    goes through a read-write reopen) after a prefix, and one opened "r+b" whose
    old content runs past the new output (kept, size unchanged), in both
    directions; the results, file sizes and final FILE* positions equal those
    of the pwrite path (SNAPPY_AMD_NO_MMAP=1)."""
    import ctypes
    libc = ctypes.CDLL(None)
    for fn, res, args in (("fopen", ctypes.c_void_p, [ctypes.c_char_p, ctypes.c_char_p]),
                          ("fclose", ctypes.c_int, [ctypes.c_void_p]),
                          ("fseek", ctypes.c_int, [ctypes.c_void_p, ctypes.c_long, ctypes.c_int]),
                          ("ftell", ctypes.c_long, [ctypes.c_void_p]),
                          ("fwrite", ctypes.c_size_t, [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_void_p])):
        getattr(libc, fn).restype = res
        getattr(libc, fn).argtypes = args
    lib = snappy_amd.lib()
    data = np.concatenate([datagen.make("T", (150 << 20) + 4321, 8), datagen.make("R", 20 << 20, 9)]).tobytes()
    want = oracle.compress_parallel(np.frombuffer(data, np.uint8).copy()).tobytes()
    prefix = b"HEAD-" * 999
    tail = b"OLD-TAIL" * ((len(data) + 12345) // 8)  # longer than any output below
    results = {}
    with tempfile.TemporaryDirectory(dir="/dev/shm" if os.path.isdir("/dev/shm") else None) as d:
        src = os.path.join(d, "in")
        open(src, "wb").write(data)
        for mm in ("1", None):
            if mm:
                os.environ["SNAPPY_AMD_NO_MMAP"] = mm
            try:
                for mode in ("wb", "r+b"):
                    snp, dec = os.path.join(d, f"c_{mode}"), os.path.join(d, f"d_{mode}")
                    for path in (snp, dec):
                        open(path, "wb").write(prefix + (tail if mode == "r+b" else b""))
                    fi, fo = libc.fopen(src.encode(), b"rb"), libc.fopen(snp.encode(), mode.encode())
                    if mode == "wb":  # ("wb" truncated the file: the prefix again, through stdio)
                        assert libc.fwrite(prefix, 1, len(prefix), fo) == len(prefix)
                    assert libc.fseek(fo, len(prefix), 0) == 0
                    lib.snappy_compress(ctypes.c_void_p(fi), ctypes.c_ulonglong(len(data)), ctypes.c_void_p(fo))
                    assert lib.snappy_amd_last_status() == 0
                    cpos = libc.ftell(fo)
                    libc.fclose(fi), libc.fclose(fo)
                    fi, fo = libc.fopen(snp.encode(), b"rb"), libc.fopen(dec.encode(), mode.encode())
                    if mode == "wb":
                        assert libc.fwrite(prefix, 1, len(prefix), fo) == len(prefix)
                    assert libc.fseek(fi, len(prefix), 0) == 0 and libc.fseek(fo, len(prefix), 0) == 0
                    if mode == "r+b":  # the stream ends before the old tail: decode exactly the stream
                        open(snp + ".s", "wb").write(want)
                        libc.fclose(fi)
                        fi = libc.fopen((snp + ".s").encode(), b"rb")
                    assert lib.snappy_decompress(ctypes.c_void_p(fi), ctypes.c_void_p(fo)) == 0
                    dpos = libc.ftell(fo)
                    libc.fclose(fi), libc.fclose(fo)
                    cblob, dblob = open(snp, "rb").read(), open(dec, "rb").read()
                    assert cpos == len(prefix) + len(want) and dpos == len(prefix) + len(data), (mm, mode)
                    assert cblob[:len(prefix)] == prefix and cblob[len(prefix):cpos] == want, (mm, mode)
                    assert dblob[:len(prefix)] == prefix and dblob[len(prefix):dpos] == data, (mm, mode)
                    if mode == "wb":
                        assert len(cblob) == cpos and len(dblob) == dpos, (mm, mode)
                    else:  # the old content past the output is untouched, the size unchanged
                        size = len(prefix) + len(tail)
                        assert len(cblob) == size and cblob[cpos:] == tail[cpos - len(prefix):], (mm, mode)
                        assert len(dblob) == size and dblob[dpos:] == tail[dpos - len(prefix):], (mm, mode)
                    results[(mm, mode)] = (len(cblob), len(dblob), cpos, dpos)
            finally:
                os.environ.pop("SNAPPY_AMD_NO_MMAP", None)
    for mode in ("wb", "r+b"):
        assert results[("1", mode)] == results[(None, mode)]


def test_file_api_mapped_output_error_leaves_file():
    """A FILE* decode that fails after its output was mapped (a 100 MiB header
    over a corrupt body) leaves the output file as it was: the same size (even
    with the FILE* positioned past its end, where stdio would not have extended
    it) and the same bytes; the pwrite path (SNAPPY_AMD_NO_MMAP=1) agrees."""
    import ctypes
    libc = ctypes.CDLL(None)
    for fn, res, args in (("fopen", ctypes.c_void_p, [ctypes.c_char_p, ctypes.c_char_p]),
                          ("fclose", ctypes.c_int, [ctypes.c_void_p]),
                          ("fseek", ctypes.c_int, [ctypes.c_void_p, ctypes.c_long, ctypes.c_int])):
        getattr(libc, fn).restype = res
        getattr(libc, fn).argtypes = args
    lib = snappy_amd.lib()
    n = 100 << 20
    rng = np.random.default_rng(11)
    body = bytes([0x01]) + rng.integers(0, 256, 3 << 20, dtype=np.uint8).tobytes()  # copy-1 at output 0: bad offset
    stream = snappy_amd.varint_encode(n) + body
    prefix = b"KEEP-ME-" * 512
    with tempfile.TemporaryDirectory(dir="/dev/shm" if os.path.isdir("/dev/shm") else None) as d:
        src = os.path.join(d, "bad.snp")
        open(src, "wb").write(stream)
        for mm in ("1", None):
            if mm:
                os.environ["SNAPPY_AMD_NO_MMAP"] = mm
            try:
                for mode, seek in (("r+b", 0), ("r+b", 4096)):
                    dec = os.path.join(d, f"out_{mm}_{seek}")
                    open(dec, "wb").write(prefix)
                    fi, fo = libc.fopen(src.encode(), b"rb"), libc.fopen(dec.encode(), mode.encode())
                    assert libc.fseek(fo, len(prefix) + seek, 0) == 0
                    rc = lib.snappy_decompress(ctypes.c_void_p(fi), ctypes.c_void_p(fo))
                    libc.fclose(fi), libc.fclose(fo)
                    assert rc != 0, (mm, seek)
                    assert open(dec, "rb").read() == prefix, (mm, seek)
            finally:
                os.environ.pop("SNAPPY_AMD_NO_MMAP", None)


def test_host_api_concurrent_threads():
    """Reentrancy: four threads compress and decompress different
    inputs through the host-buffer API at once, and two threads run the FILE*
    pipelines on two files at once; each call leases its own pooled host
    context, every output equals the oracle's, and the pool keeps the idle
    contexts (at least one per concurrent caller) until released."""
    import ctypes
    import threading
    lib = snappy_amd.lib()
    lib.snappy_amd_host_release()
    inputs = [datagen.make(k, n, s).tobytes() for k, n, s in
              (("T", (24 << 20) + 7, 61), ("R", 9 << 20, 62), ("T", 40 << 20, 63), ("P", 17 << 20, 64))]
    wants = [oracle.compress(x) for x in inputs]
    errs = []
    start = threading.Barrier(len(inputs))

    def work(i):
        try:
            start.wait()
            for _ in range(3):
                c = snappy_amd.compress(inputs[i])
                assert c == wants[i], i
                assert snappy_amd.decompress(c) == inputs[i], i
        except Exception as e:  # noqa: BLE001
            errs.append((i, repr(e)))

    th = [threading.Thread(target=work, args=(i,)) for i in range(len(inputs))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs, errs
    assert lib.snappy_amd_host_pool_size() >= 2
    # the FILE* pipelines, two files at once
    libc = ctypes.CDLL(None)
    libc.fopen.restype = ctypes.c_void_p
    libc.fopen.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
    libc.fclose.argtypes = [ctypes.c_void_p]
    files = [inputs[2] + inputs[0], inputs[1] * 12]  # 64 MiB+ (two chunks) and 108 MiB
    with tempfile.TemporaryDirectory(dir="/dev/shm" if os.path.isdir("/dev/shm") else None) as d:
        def file_work(i):
            try:
                src, snp, dec = (os.path.join(d, f"{i}{x}").encode() for x in ("", ".snp", ".dec"))
                open(src, "wb").write(files[i])
                start2.wait()
                fi, fo = libc.fopen(src, b"rb"), libc.fopen(snp, b"wb")
                lib.snappy_compress(ctypes.c_void_p(fi), ctypes.c_ulonglong(len(files[i])), ctypes.c_void_p(fo))
                assert lib.snappy_amd_last_status() == 0
                libc.fclose(ctypes.c_void_p(fi)), libc.fclose(ctypes.c_void_p(fo))
                fi, fo = libc.fopen(snp, b"rb"), libc.fopen(dec, b"wb")
                assert lib.snappy_decompress(ctypes.c_void_p(fi), ctypes.c_void_p(fo)) == 0
                libc.fclose(ctypes.c_void_p(fi)), libc.fclose(ctypes.c_void_p(fo))
                assert open(snp, "rb").read() == oracle.compress(files[i]), i
                assert open(dec, "rb").read() == files[i], i
            except Exception as e:  # noqa: BLE001
                errs.append(("file", i, repr(e)))

        start2 = threading.Barrier(2)
        th = [threading.Thread(target=file_work, args=(i,)) for i in range(2)]
        for t in th:
            t.start()
        for t in th:
            t.join()
    assert not errs, errs
    assert lib.snappy_amd_host_release() == 0 and lib.snappy_amd_host_pool_size() == 0


def test_host_device_selection():
    lib = snappy_amd.lib()
    assert lib.snappy_amd_host_set_device(0) == 0 and lib.snappy_amd_host_get_device() == 0
    assert lib.snappy_amd_host_set_device(4096) == snappy_amd.ERR_DEVICE
    assert lib.snappy_amd_host_set_device(-1) == 0


def test_multi_device_buffer_api(golden):
    """snappy_compress_buffer_multi / snappy_decompress_buffer_multi with the
    one device of the box listed 1-3 times (a context and a thread each): the
    stream equals the one-device stream (the reference's bytes), the decode
    splits into block ranges; streams whose ranges are not self-contained
    (the reference-decodable cross-block vectors) still decode exactly."""
    for kind, n, seed in (("T", (9 << 20) + 12345, 71), ("R", 3 << 20, 72), ("T", 65536 * 2, 73), ("T", 100, 74)):
        data = datagen.make(kind, n, seed).tobytes()
        want = oracle.compress(data)
        for devs in ([0], [0, 0], [0, 0, 0]):
            got = snappy_amd.compress_multi(data, devs)
            assert got == want, (kind, n, devs)
            assert snappy_amd.decompress_multi(got, devs) == data, (kind, n, devs)
    assert snappy_amd.compress_multi(b"", [0, 0]) == b""
    for v in golden["xblock_vectors"]:
        stream = _xblock_stream(v)
        out = snappy_amd.decompress_multi(stream, [0, 0, 0])
        assert len(out) == v["out_len"] and sha(out) == v["out_sha256"], v["name"]
    with pytest.raises(snappy_amd.SnappyError):
        snappy_amd.decompress_multi(want[:-3], [0, 0])
    # malformed streams (bytes flipped in the later ranges): the same outcome --
    # error code, or bytes -- as the one-device decode, whichever range fails first
    rng = np.random.default_rng(75)
    data = datagen.make("T", 9 << 20, 76).tobytes()
    base = oracle.compress(data)

    def outcome(f, b):
        try:
            return f(b)
        except snappy_amd.SnappyError as e:
            return e.code

    codes = set()
    for t in range(12):
        bad = bytearray(base)
        for p in rng.integers(len(base) // 4, len(base), 1 + t % 3):
            bad[int(p)] ^= int(rng.integers(1, 256))
        bad = bytes(bad)
        one = outcome(snappy_amd.decompress, bad)
        codes.add(one if isinstance(one, int) else 0)
        assert outcome(lambda b: snappy_amd.decompress_multi(b, [0, 0, 0]), bad) == one, t
    assert len(codes) > 1, codes  # the corruptions reach more than one kind of outcome


def test_decompress_file_bogus_length():
    """A preamble declaring more than the stream could ever produce (10 bytes
    claiming 2^40) is refused before any output is mapped or preallocated: the
    output file keeps its size and its allocated blocks.  A plausible length
    over a corrupt body fails in the decoder, and the blocks preallocated for
    it past the file's end are released (st_blocks back to the old value)."""
    import ctypes
    libc = ctypes.CDLL(None)
    libc.fopen.restype = ctypes.c_void_p
    libc.fopen.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
    libc.fclose.argtypes = [ctypes.c_void_p]
    lib = snappy_amd.lib()
    rng = np.random.default_rng(12)
    bogus = snappy_amd.varint_encode(1 << 40) + b"\x00abc"
    corrupt = snappy_amd.varint_encode(80 << 20) + bytes([0x01]) + rng.integers(0, 256, 4 << 20, np.uint8).tobytes()
    prefix = b"KEEP" * 1024
    with tempfile.TemporaryDirectory(dir="/dev/shm" if os.path.isdir("/dev/shm") else None) as d:
        for name, stream, want in (("bogus", bogus, snappy_amd.ERR_TRUNCATED), ("corrupt", corrupt, None)):
            src, dec = os.path.join(d, name), os.path.join(d, name + ".out")
            open(src, "wb").write(stream)
            for mm in ("1", None):
                if mm:
                    os.environ["SNAPPY_AMD_NO_MMAP"] = mm
                try:
                    open(dec, "wb").write(prefix)
                    before = os.stat(dec)
                    fi, fo = libc.fopen(src.encode(), b"rb"), libc.fopen(dec.encode(), b"ab")
                    rc = lib.snappy_decompress(ctypes.c_void_p(fi), ctypes.c_void_p(fo))
                    libc.fclose(ctypes.c_void_p(fi)), libc.fclose(ctypes.c_void_p(fo))
                    assert rc != 0 and (want is None or rc == want), (name, mm, rc)
                    fi, fo = libc.fopen(src.encode(), b"rb"), libc.fopen(dec.encode(), b"r+b")
                    rc = lib.snappy_decompress(ctypes.c_void_p(fi), ctypes.c_void_p(fo))
                    libc.fclose(ctypes.c_void_p(fi)), libc.fclose(ctypes.c_void_p(fo))
                    assert rc != 0 and (want is None or rc == want), (name, mm, rc)
                    after = os.stat(dec)
                    assert after.st_size == before.st_size and open(dec, "rb").read() == prefix, (name, mm)
                    assert after.st_blocks <= before.st_blocks, (name, mm, before.st_blocks, after.st_blocks)
                finally:
                    os.environ.pop("SNAPPY_AMD_NO_MMAP", None)
    with pytest.raises(snappy_amd.SnappyError) as ei:
        snappy_amd.decompress(bogus)
    assert ei.value.code == snappy_amd.ERR_TRUNCATED


def test_host_buffer_sizes_to_one_chunk():
    """snappy_compress_buffer / snappy_decompress_buffer at sizes from 8 MiB
    up to one pipeline chunk (64 MiB), incl. odd ones: the one-shot stream
    byte for byte, and the round trip."""
    M = 1 << 20
    for n, seed in ((8 * M - 1, 91), (8 * M, 92), (16 * M + 1, 93), (48 * M + 3, 94), (64 * M, 95)):
        a = datagen.make("T", n, seed)
        got = snappy_amd.compress(a.tobytes())
        want = oracle.compress_parallel(a, threads=16).tobytes()
        assert got == want, n
        assert snappy_amd.decompress(got) == a.tobytes(), n
        progress(f"host buffer {n}: ok")


def test_host_buffer_pipelined_chunks():
    """snappy_compress_buffer of more than one 64 MiB chunk runs as a pipeline
    of chunk lanes (csrc/snappy_device.hip host_compress_pipelined): the
    stream equals the one-shot reference stream for sizes around the chunk
    and lane-reuse boundaries (5 chunks > 4 lanes), and round-trips."""
    M = 1 << 20
    for n, kind, seed in (((64 << 20) + 1, "T", 81), ((128 << 20) + 65536 * 3 + 7, "T", 82),
                          (300 * M + 12345, "T", 83), (70 * M, "R", 84)):
        a = datagen.make(kind, n, seed)
        got = snappy_amd.compress(a.tobytes())
        want = oracle.compress_parallel(a, threads=16).tobytes()
        assert len(got) == len(want) and got == want, (kind, n)
        assert snappy_amd.decompress(got) == a.tobytes(), (kind, n)
        progress(f"pipelined host compress {kind} {n}: ok")


def test_host_decompress_large_foreign():
    """snappy_decompress_buffer of foreign streams of 34 and 115 MB (literals
    of up to 200,000 bytes across K5p chunks and 65,536-byte blocks, copies up
    to 1 MiB back) decodes as the oracle decodes them, and so does a stream of
    ours just over 32 MiB."""
    for seed, n_out in ((311, 112 << 20), (312, (33 << 20) + 200000)):
        stream = build_stream(random_ops(seed, n_out, 1 << 20, max_lit=200000))
        want = oracle.decompress(stream)
        assert len(want) == n_out
        assert snappy_amd.decompress(stream) == want, (seed, len(stream))
        progress(f"host decompress of a foreign stream, seed {seed}: {len(stream)} stream bytes ok")
    a = datagen.make("R", (32 << 20) + 4096, 313)
    comp = snappy_amd.compress(a.tobytes())
    assert len(comp) > (32 << 20)
    assert snappy_amd.decompress(comp) == a.tobytes()


def test_file_decompress_back_to_back_outputs():
    """The FILE* decoder's mapped output is unmapped in the background once
    its bytes and size are final (IoFile::unmap): the output reads back whole
    right after the call, and the same path can be removed, rewritten and
    decoded into again at once, three times in a row."""
    import ctypes
    libc = ctypes.CDLL(None)
    libc.fopen.restype = ctypes.c_void_p
    libc.fopen.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
    libc.fclose.argtypes = [ctypes.c_void_p]
    lib = snappy_amd.lib()
    data = datagen.make("T", (96 << 20) + 777, 91).tobytes()
    comp = snappy_amd.compress(data)
    with tempfile.TemporaryDirectory(dir="/dev/shm" if os.path.isdir("/dev/shm") else None) as d:
        src, dst = os.path.join(d, "in.snp"), os.path.join(d, "out")
        open(src, "wb").write(comp)
        for _ in range(3):
            fi, fo = libc.fopen(src.encode(), b"rb"), libc.fopen(dst.encode(), b"wb")
            assert lib.snappy_decompress(ctypes.c_void_p(fi), ctypes.c_void_p(fo)) == 0
            libc.fclose(fi), libc.fclose(fo)
            assert os.path.getsize(dst) == len(data)
            assert open(dst, "rb").read() == data
            os.unlink(dst)
