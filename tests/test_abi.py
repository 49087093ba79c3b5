"""CPU: the C-ABI library loads and exports every function include/*.h
declares; pure host helpers (varint) behave like src/varint.c.  No kernel is
launched here."""
import ctypes
import os
import re
import subprocess

import pytest

import snappy_amd

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INC = os.path.join(ROOT, "include")


COMPAT_HEADERS = ("buffer_compression.h",)  # exported by libsnappy_amd_compat.so instead


def declared_functions(compat=False):
    names = set()
    for h in os.listdir(INC):
        if not h.endswith(".h") or (h in COMPAT_HEADERS) != compat:
            continue
        src = open(os.path.join(INC, h)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        for m in re.finditer(r"^[A-Za-z_][\w \*]*?\b(\w+)\s*\([^;{]*\)\s*;", src, flags=re.M):
            names.add(m.group(1))
    return names


def test_headers_declare_the_reference_entry_points():
    names = declared_functions()
    for must in ("snappy_compress", "snappy_decompress", "snappy_compress_bst"):
        assert must in names
    assert len(names) >= 25


def test_library_exports_every_declared_symbol():
    lib = snappy_amd.lib()
    missing = [n for n in sorted(declared_functions()) if not hasattr(lib, n)]
    assert not missing, missing
    out = subprocess.run(["nm", "-D", "--defined-only", snappy_amd.LIB_PATH], capture_output=True, text=True).stdout
    for n in declared_functions():
        assert re.search(rf"\bT {n}$", out, flags=re.M), n


def test_python_binding_covers_header():
    assert declared_functions() <= set(snappy_amd._SIGS)
    assert declared_functions(compat=True) <= set(snappy_amd._COMPAT_SIGS)


def test_compat_library_holds_the_generic_names():
    # init_Buffer / move_current / reset: in libsnappy_amd_compat.so only, so
    # linking the codec cannot interpose on an application's own `reset`
    names = declared_functions(compat=True)
    assert names == {"init_Buffer", "move_current", "reset"}
    main = subprocess.run(["nm", "-D", "--defined-only", snappy_amd.LIB_PATH], capture_output=True, text=True).stdout
    comp = subprocess.run(["nm", "-D", "--defined-only", snappy_amd.COMPAT_PATH], capture_output=True, text=True).stdout
    for n in names:
        assert not re.search(rf"\b{n}$", main, flags=re.M), n
        assert re.search(rf"\bT {n}$", comp, flags=re.M), n


def test_varint_host(golden):
    for k in golden["varint"]:
        assert snappy_amd.varint_encode(k["n"]).hex() == k["hex"]
        v, used = snappy_amd.varint_decode(bytes.fromhex(k["hex"]))
        assert (v, used) == (k["n"], len(k["hex"]) // 2)
    # 64-bit lengths (varint.c:28-42 overflows its int at 2^31)
    for n in (2**31, 5 * 2**30, 64 * 2**30, 2**63):
        v, used = snappy_amd.varint_decode(snappy_amd.varint_encode(n))
        assert v == n
    assert snappy_amd.varint_decode(b"\x80\x80")[1] == 0


def test_cli_usage_without_args():
    exe = os.path.join(ROOT, "lightweight-snappy_amd", "snappy")
    r = subprocess.run([exe], capture_output=True)
    assert r.returncode == 1 and b"snappy [-c|-d|-b]" in r.stderr


def test_no_oracle_in_product():
    # the product package must never load the checker
    pkg = os.path.join(ROOT, "lightweight-snappy_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".c", ".cpp", ".cc", ".hip", ".h", ".hpp", "Makefile")):
                src = open(os.path.join(dirpath, f), errors="ignore").read()
                assert "liboracle" not in src and "import oracle" not in src, f
    out = subprocess.run(["ldd", snappy_amd.LIB_PATH], capture_output=True, text=True).stdout
    assert "oracle" not in out and "snappy_ref" not in out
    # nor may the host code open another library or program at run time
    for f in os.listdir(os.path.join(pkg, "csrc")):
        src = open(os.path.join(pkg, "csrc", f), errors="ignore").read()
        for bad in ("dlopen", "execv", "execl", "system(", "popen("):
            assert bad not in src, (f, bad)


def assert_product_config(cfg: str):
    """A shipped library: both kernel halves built without measurement knobs
    (the wrong-output ones cannot even compile without SNAPPY_MEASUREMENT_BUILD)."""
    assert cfg.startswith("compress{") and " decode{" in cfg, cfg
    for must in ("compress{measurement=0", "decode{measurement=0", "k2_nolit=0", "k4_nofar=0", "k1r_asm=1"):
        assert must in cfg, (must, cfg)


def test_shipped_library_is_a_product_build():
    assert_product_config(snappy_amd.build_config())


def test_wrong_output_knobs_refuse_to_compile(tmp_path):
    # -DSNAPPY_K4_NOFAR / -DSNAPPY_K2_NOLIT=1 without SNAPPY_MEASUREMENT_BUILD: #error
    src = os.path.join(ROOT, "lightweight-snappy_amd", "csrc", "snappy_kernels.hip")
    for knob in ("-DSNAPPY_K4_NOFAR", "-DSNAPPY_K2_NOLIT=1"):
        r = subprocess.run(["/opt/rocm/bin/hipcc", "-E", "--offload-arch=gfx950", "-std=c++17", "-I", INC,
                            "-I", os.path.dirname(src), knob, "--cuda-host-only", src, "-o", str(tmp_path / "x.i")],
                           capture_output=True, text=True)
        assert r.returncode != 0 and "measurement builds only" in r.stderr, (knob, r.stderr[-2000:])


@pytest.mark.skipif(not os.path.isdir("/root/reference/src"), reason="reference sources only in the build container")
def test_reference_cli_links_against_library(tmp_path):
    # the reference's own src/cmd.c, unchanged, links against libsnappy_amd.so
    src = "/root/reference/src"
    exe = tmp_path / "snappy_dropin"
    r = subprocess.run(["gcc", "-O2", "-w", "-I", INC, "-o", str(exe), f"{src}/cmd.c", f"{src}/IO_utils.c",
                        f"{src}/result.c", "-L", os.path.dirname(snappy_amd.LIB_PATH), "-lsnappy_amd"],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_buffer_cursor_helpers():
    # src/buffer_compression.c:10-34 semantics, host-only (no GPU call)
    import ctypes

    class Buffer(ctypes.Structure):
        _fields_ = [("current", ctypes.c_void_p), ("beginning", ctypes.c_void_p), ("bytes_left", ctypes.c_uint)]

    lib = snappy_amd.compat_lib()
    b = Buffer()
    lib.init_Buffer(ctypes.byref(b), 100)
    assert b.current == b.beginning and b.current and b.bytes_left == 100
    assert ctypes.string_at(b.beginning, 100) == bytes(100)  # calloc'd
    lib.move_current(ctypes.byref(b), 30)
    assert b.current - b.beginning == 30 and b.bytes_left == 70
    lib.reset(ctypes.byref(b))
    assert b.current == b.beginning and b.bytes_left == 70  # reset leaves bytes_left alone
    ctypes.CDLL(None).free(ctypes.c_void_p(b.beginning))


def test_kernel_register_budget(tmp_path):
    """The gfx950 code object of the built library: the K1r kernels keep the
    unit in v2..v129 untouched between their register-indexed accesses (the
    65,536-byte kernel writes its ring only through gpr_idx DST moves), fit
    3 waves per SIMD (<= 168 VGPRs) and spill nothing (tools/check_ring.py)."""
    import re
    import shutil
    import subprocess
    import sys
    llvm = "/opt/rocm/lib/llvm/bin"
    obj = os.path.join(ROOT, "lightweight-snappy_amd", "build", "snappy_kernels_c.o")  # the compress kernels
    if not (os.path.exists(obj) and os.path.exists(f"{llvm}/llvm-objdump") and shutil.which("objcopy")):
        pytest.skip("needs the in-tree build object and the ROCm LLVM tools")
    fat, co = tmp_path / "fat.bin", tmp_path / "k.co"
    # (an output file: with none, objcopy rewrites the build object in place)
    subprocess.run(["objcopy", f"--dump-section=.hip_fatbin={fat}", obj, str(tmp_path / "copy.o")], check=True)
    subprocess.run([f"{llvm}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
    notes = subprocess.run([f"{llvm}/llvm-readobj", "--notes", str(co)], check=True, capture_output=True,
                           text=True).stdout
    found = 0
    for blk in notes.split("- .agpr_count")[1:]:
        name = re.search(r"\.name:\s+(\S+)", blk).group(1)
        if "k1r_match_units" not in name:
            continue
        found += 1
        vg = int(re.search(r"\.vgpr_count:\s+(\d+)", blk).group(1))
        sp = int(re.search(r"\.vgpr_spill_count:\s+(\d+)", blk).group(1))
        assert vg <= 168 and sp == 0, (name, vg, sp)
    assert found == 2
    dis = subprocess.run([f"{llvm}/llvm-objdump", "-d", str(co)], check=True, capture_output=True, text=True).stdout
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import check_ring
    assert check_ring.check(dis) == []


@pytest.mark.parametrize("obj", ["snappy_kernels_c.o", "snappy_kernels_d.o"])
def test_asm_memory_ops_drained(tmp_path, obj):
    """Inline-asm memory operations (the round-2 hang class):
    every asm load into a register waits inside its own asm block, and every
    LDS-DMA (global_load_lds) is drained by s_waitcnt vmcnt(0) on every path
    to s_endpgm of the built code object (tools/check_asm_waits.py)."""
    import shutil
    import sys
    llvm = "/opt/rocm/lib/llvm/bin"
    path = os.path.join(ROOT, "lightweight-snappy_amd", "build", obj)
    if not (os.path.exists(path) and os.path.exists(f"{llvm}/llvm-objdump") and shutil.which("objcopy")):
        pytest.skip("needs the in-tree build object and the ROCm LLVM tools")
    fat, co = tmp_path / "fat.bin", tmp_path / "k.co"
    subprocess.run(["objcopy", f"--dump-section=.hip_fatbin={fat}", path, str(tmp_path / "copy.o")], check=True)
    subprocess.run([f"{llvm}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
    dis = subprocess.run([f"{llvm}/llvm-objdump", "-d", str(co)], check=True, capture_output=True, text=True).stdout
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import check_asm_waits
    assert "global_load_lds" in dis or obj.endswith("_d.o")  # the checker sees the compress kernels' DMA
    assert check_asm_waits.check(dis) == []
    if obj.endswith("_d.o"):  # K4's element-start bitmap: clear, or, read in that order
        assert check_asm_waits.check_k4_bitmap(dis) == []
    else:  # the register-index asm leaves m0 holding its index: nothing reads it after
        assert check_asm_waits.check_m0(dis) == []
    csrc = os.path.join(ROOT, "lightweight-snappy_amd", "csrc")
    for f in sorted(os.listdir(csrc)):
        if f.endswith(".hip"):
            assert check_asm_waits.lint_source(os.path.join(csrc, f)) == [], f
            assert check_asm_waits.lint_scc(os.path.join(csrc, f)) == [], f


def test_asm_wait_checker_catches_undrained_dma():
    """The checker itself: a synthetic kernel whose LDS-DMA can reach s_endpgm
    through a branch that skips the wait is flagged; the drained one is not."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import check_asm_waits
    k = ("0000000000001000 <kern>:\n"
         "\tglobal_load_lds_dword v1, s[2:3]      // 000000001000: 0\n"
         "\ts_cbranch_scc1 2                      // 000000001008: 0 <kern+0x14>\n"
         "\ts_waitcnt vmcnt(0)                    // 00000000100C: 0\n"
         "\ts_nop 0                               // 000000001010: 0\n"
         "\ts_endpgm                              // 000000001014: 0\n")
    assert len(check_asm_waits.check(k)) == 1
    assert check_asm_waits.check(k.replace("s_cbranch_scc1 2", "s_nop 1")) == []


def test_m0_and_scc_checkers_catch_their_cases(tmp_path):
    """The checkers themselves: a writelane that reads m0 right after a
    register-index region is flagged, one after m0 is set again is not; an asm
    statement with an SCC-writing SALU and no "scc" clobber is flagged."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import check_asm_waits
    k = ("0000000000001000 <k1r_match_units_x>:\n"
         "\ts_mov_b32 m0, s4                      // 000000001000: 0\n"
         "\ts_set_gpr_idx_on s2, gpr_idx(SRC0)    // 000000001004: 0\n"
         "\tv_mov_b32 v1, v2                      // 00000000100C: 0\n"
         "\ts_set_gpr_idx_off                     // 000000001010: 0\n"
         "\tv_writelane_b32 v3, s5, m0            // 000000001014: 0\n"
         "\ts_endpgm                              // 00000000101C: 0\n")
    assert len(check_asm_waits.check_m0(k)) == 1
    fixed = k.replace("\tv_writelane_b32 v3, s5, m0            // 000000001014: 0\n",
                      "\ts_mov_b32 m0, s4                      // 000000001014: 0\n"
                      "\tv_writelane_b32 v3, s5, m0            // 000000001018: 0\n")
    assert check_asm_waits.check_m0(fixed) == []
    src = tmp_path / "k.hip"
    src.write_text('asm("s_max_u32 %0, %1, 59" : "=s"(a) : "s"(b));\n'
                   'asm("s_max_u32 %0, %1, 59" : "=s"(a) : "s"(b) : "scc");\n'
                   'asm volatile("s_mov_b32 %0, m0\\nL%=_x:" : "=s"(a));\n')
    assert [b[0].rsplit(":", 1)[1] for b in check_asm_waits.lint_scc(str(src))] == ["1"]
