#!/usr/bin/env python3
"""Generate tests/golden/ from the COMPILED REFERENCE (oracle/_ref, built by
`make -C oracle ref` from the sources under /root/reference/src).

Runs only in the build container (the reference does not exist on the GPU
box).  Every input is regenerable from a closed-form spec (datagen kinds,
sizes, seeds) so the fixtures hold only hashes, lengths and small outputs.
Entries:
  * Appendix B known-answer vectors of SURVEY.md (including the reference's
    own LICENSE file as data, committed as tests/golden/license.bin);
  * the Appendix A.4 edge matrix (sizes x data kinds);
  * the reference decoder on hand-built streams using elements the reference
    compressor never emits (copy-4, 4-byte literal lengths, overlaps);
  * cross-block decoder vectors (elements straddling 65,536-byte blocks,
    copies into earlier blocks; hand-built and seeded random foreign streams);
  * the reference's own varint KATs (src/test_varint.c:27-35);
  * the 32 KiB-stream layout of BASELINE.json configs[1] on a 32 MiB sample.
`python oracle/gen_golden.py bst` writes tests/golden/golden_bst.json instead:
the reference's -b compressor (snappy_compress_bst,
src/snappy_compression_tree.c:291-306) over the same Appendix A.4 edge matrix,
period sweep and larger pins, each output checked to round-trip through the
reference decoder.
Usage: python oracle/gen_golden.py [bst]
"""
from __future__ import annotations

import hashlib
import json
import os
import shutil
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "lightweight-snappy_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import datagen  # noqa: E402
import golden_inputs  # noqa: E402
import oracle  # noqa: E402

GOLD = os.path.join(ROOT, "tests", "golden")
HEX_LIMIT = 2048


def sha(b: bytes) -> str:
    return hashlib.sha256(b).hexdigest()


def make_input(spec: dict) -> bytes:
    kind = spec["kind"]
    n = spec["size"]
    if kind == "bytes":
        return bytes.fromhex(spec["hex"])
    if kind == "license":
        lic = open(os.path.join(GOLD, "license.bin"), "rb").read()
        return (lic * (n // len(lic) + 1))[:n]
    if kind == "iota64":
        return (bytes(range(64)) * (n // 64 + 1))[:n]
    if kind == "K":
        return datagen.make("K", n, spec["seed"], spec["period"]).tobytes()
    return datagen.make(kind, n, spec.get("seed", 0)).tobytes()


def entry(name: str, spec: dict, data: bytes | None = None) -> dict:
    if data is None:
        data = make_input(spec)
    out = oracle.ref_compress(data)
    dec = oracle.ref_decompress(out, len(data)) if data else b""
    assert dec == data, f"reference round trip failed on {name}"
    e = {"name": name, "spec": spec, "in_len": len(data), "in_sha256": sha(data), "out_len": len(out),
         "out_sha256": sha(out)}
    if len(out) <= HEX_LIMIT:
        e["out_hex"] = out.hex()
    else:
        e["out_prefix_hex"] = out[:64].hex()
    return e


EDGE_SIZES = [1, 2, 3, 4, 5, 15, 16, 17, 18, 31, 32, 33, 59, 60, 61, 63, 64, 65, 255, 256, 257, 511, 512, 1025,
              2048, 2049, 4095, 4096, 4097, 32767, 32768, 32769, 65535, 65536, 65537, 131072, 131073]
EDGE_KINDS = [("T", {"seed": 7}), ("R", {"seed": 3}), ("Z", {}), ("P", {"seed": 2})]
PERIODS = [1, 2, 3, 4, 5, 7, 11, 12, 13, 63, 64, 65, 67, 68, 69, 2047, 2048, 2049, 3000]


def bst_entry(name: str, spec: dict) -> dict:
    data = make_input(spec)
    out = oracle.ref_compress_bst(data)
    dec = oracle.ref_decompress(out, len(data)) if data else b""
    assert dec == data, f"reference -b round trip failed on {name}"
    e = {"name": name, "spec": spec, "in_len": len(data), "in_sha256": sha(data), "out_len": len(out),
         "out_sha256": sha(out)}
    if len(out) <= HEX_LIMIT:
        e["out_hex"] = out.hex()
    else:
        e["out_prefix_hex"] = out[:64].hex()
    return e


def main_bst() -> None:
    entries = []
    for name, spec in [("abc", {"kind": "bytes", "size": 3, "hex": b"abc".hex()}),
                       ("a_x20", {"kind": "bytes", "size": 20, "hex": (b"a" * 20).hex()}),
                       ("hello", {"kind": "bytes", "size": 16, "hex": b"Hello, Snappy!!!".hex()}),
                       ("empty", {"kind": "bytes", "size": 0, "hex": ""}),
                       ("license", {"kind": "license", "size": 1069}),
                       ("license_1MiB", {"kind": "license", "size": 1 << 20}),
                       ("zeros_1MiB", {"kind": "Z", "size": 1 << 20}),
                       ("iota64_1MiB", {"kind": "iota64", "size": 1 << 20})]:
        entries.append(bst_entry(name, spec))
    for k, extra in EDGE_KINDS:
        for n in EDGE_SIZES:
            entries.append(bst_entry(f"edge_{k}_{n}", {"kind": k, "size": n, **extra}))
    for period in PERIODS:
        for n in [200, 5000, 65536, 70000]:
            entries.append(bst_entry(f"period_{period}_{n}", {"kind": "K", "size": n, "seed": 100 + period,
                                                             "period": period}))
    entries.append(bst_entry("text_1000000", {"kind": "T", "size": 1000000, "seed": 1234}))
    entries.append(bst_entry("text_3MiB", {"kind": "T", "size": 3 << 20, "seed": 99}))
    entries.append(bst_entry("random_1MiB", {"kind": "R", "size": 1 << 20, "seed": 1}))
    entries.append(bst_entry("repeat_1MiB", {"kind": "P", "size": 1 << 20, "seed": 2}))
    entries.append(bst_entry("lcg1_1MiB", {"kind": "L", "size": 1 << 20, "seed": 1}))
    gold = {"generator": "oracle/gen_golden.py bst", "reference": "tturturiello/lightweight-snappy (oracle/_ref, "
            "snappy_compress_bst)", "entries": entries}
    with open(os.path.join(GOLD, "golden_bst.json"), "w") as f:
        json.dump(gold, f, indent=1)
    print(f"wrote {len(entries)} -b entries")


def main() -> None:
    os.makedirs(GOLD, exist_ok=True)
    shutil.copyfile("/root/reference/LICENSE", os.path.join(GOLD, "license.bin"))
    entries = []
    # --- SURVEY.md Appendix B known answers --------------------------------
    kat = [
        ("abc", {"kind": "bytes", "size": 3, "hex": b"abc".hex()}),
        ("a_x20", {"kind": "bytes", "size": 20, "hex": (b"a" * 20).hex()}),
        ("hello", {"kind": "bytes", "size": 16, "hex": b"Hello, Snappy!!!".hex()}),
        ("zeros_1MiB", {"kind": "Z", "size": 1 << 20}),
        ("iota64_1MiB", {"kind": "iota64", "size": 1 << 20}),
        ("lcg1_1MiB", {"kind": "L", "size": 1 << 20, "seed": 1}),
        ("license", {"kind": "license", "size": 1069}),
        ("license_1MiB", {"kind": "license", "size": 1 << 20}),
        ("license_65537", {"kind": "license", "size": 65537}),
        ("empty", {"kind": "bytes", "size": 0, "hex": ""}),
    ]
    for name, spec in kat:
        entries.append(entry(name, spec))
    # --- Appendix A.4 edge matrix -------------------------------------------
    for k, extra in EDGE_KINDS:
        for n in EDGE_SIZES:
            spec = {"kind": k, "size": n, **extra}
            entries.append(entry(f"edge_{k}_{n}", spec))
    for period in PERIODS:
        for n in [200, 5000, 65536, 70000]:
            spec = {"kind": "K", "size": n, "seed": 100 + period, "period": period}
            entries.append(entry(f"period_{period}_{n}", spec))
    # --- larger pins ----------------------------------------------------------
    entries.append(entry("text_1000000", {"kind": "T", "size": 1000000, "seed": 1234}))  # configs[0]
    entries.append(entry("text_3MiB", {"kind": "T", "size": 3 << 20, "seed": 99}))
    entries.append(entry("random_1MiB", {"kind": "R", "size": 1 << 20, "seed": 1}))
    entries.append(entry("repeat_1MiB", {"kind": "P", "size": 1 << 20, "seed": 2}))

    # --- STREAMS layout (configs[1] shape): 32 MiB text as 1024 x 32 KiB ------
    n = 32 << 20
    chunk = 32768
    text = datagen.make("T", n, 1234)
    payload = bytearray()
    offsets = [0]
    first = []
    for s in range(n // chunk):
        piece = text[s * chunk:(s + 1) * chunk].tobytes()
        c = oracle.ref_compress(piece)
        if s < 64:
            first.append({"stream": s, "len": len(c), "sha256": sha(c)})
        payload += c
        offsets.append(len(payload))
    streams = {"spec": {"kind": "T", "size": n, "seed": 1234}, "chunk": chunk, "in_sha256": sha(text.tobytes()),
               "out_len": len(payload), "out_sha256": sha(bytes(payload)),
               "offsets_sha256": sha(np.asarray(offsets, dtype=np.uint64).tobytes()), "first_streams": first}

    # --- decoder-only vectors (elements the reference compressor never emits) -
    dec_vectors = []

    def dec(name: str, stream: bytes, n_out: int):
        out = oracle.ref_decompress(stream, n_out)
        dec_vectors.append({"name": name, "stream_hex": stream.hex(), "out_hex": out.hex()})

    dec("copy4_overlap", bytes([16, 0x0C]) + b"abcd" + bytes([(8 - 1) << 2 | 3, 4, 0, 0, 0, (0 << 5) | ((4 - 4) << 2) | 1, 1]), 16)
    dec("lit_4byte_len", bytes([10, 63 << 2, 9, 0, 0, 0]) + b"0123456789", 10)
    dec("lit_3byte_len", bytes([70, 62 << 2, 69, 0, 0]) + bytes(range(70)), 70)
    dec("copy2_rle", bytes([40, 0]) + b"x" + bytes([(39 - 1) << 2 | 2, 1, 0]), 40)
    # 1024-byte literal (2-byte length), copy-1 with offset high bits (off 1000),
    # copy-2 reaching back 1024 bytes; N = 1037 = varint 8d 08
    dec("copy1_hi_offset", bytes([0x8D, 0x08, 61 << 2, 0xFF, 0x03]) + bytes((i * 7) & 0xFF for i in range(1024))
        + bytes([(3 << 5) | ((8 - 4) << 2) | 1, 0xE8]) + bytes([((5 - 1) << 2) | 2, 0x00, 0x04]), 1037)

    # --- cross-block decoder vectors: streams another encoder could write, whose
    # elements straddle 65,536-byte output blocks and whose copies reach into
    # earlier blocks (up to the reference's 131,072 limit,
    # src/snappy_decompression.c:262); the streams are rebuilt from their specs
    # by tests/golden_inputs.py, only hashes are committed
    xblock = []

    def xvec(name: str, ops: list | None = None, rnd: dict | None = None):
        if rnd is not None:
            ops = golden_inputs.random_ops(rnd["seed"], rnd["n_out"], rnd["max_off"])
        stream = golden_inputs.build_stream(ops)
        n_out = golden_inputs.uncompressed_length(stream)
        out = oracle.ref_decompress(stream, n_out)
        assert len(out) == n_out, name
        assert oracle.decompress(stream) == out, f"oracle differs from the reference on {name}"
        e = {"name": name, "stream_len": len(stream), "stream_sha256": sha(stream), "out_len": n_out,
             "out_sha256": sha(out)}
        if rnd is not None:
            e["random"] = rnd
        else:
            e["ops"] = ops
        xblock.append(e)

    for name, ops in golden_inputs.decoder_vector_ops().items():
        xvec(name, ops=ops)
    for seed, n_out, max_off in [(1, 300_000, 131072), (2, 500_000, 131072), (3, 700_000, 65535),
                                 (4, 1_000_000, 131072), (5, 262_144, 131072), (6, 2_000_000, 131072)]:
        xvec(f"foreign_random_{seed}", rnd={"seed": seed, "n_out": n_out, "max_off": max_off})

    varint_kats = [{"n": 127, "hex": "7f"}, {"n": 227, "hex": "e301"}, {"n": 16384, "hex": "808001"},
                   {"n": 1000000, "hex": "c0843d"}, {"n": 1 << 30, "hex": "8080808004"}, {"n": 32768, "hex": "808002"}]

    gold = {"generator": "oracle/gen_golden.py", "reference": "tturturiello/lightweight-snappy (oracle/_ref)",
            "entries": entries, "streams_32k": streams, "decoder_vectors": dec_vectors,
            "xblock_vectors": xblock, "varint": varint_kats}
    with open(os.path.join(GOLD, "golden.json"), "w") as f:
        json.dump(gold, f, indent=1)
    print(f"wrote {len(entries)} entries, {len(dec_vectors)} decoder vectors, {len(xblock)} cross-block vectors")


if __name__ == "__main__":
    main_bst() if sys.argv[1:] == ["bst"] else main()
