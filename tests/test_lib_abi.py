"""CPU-side checks of the C-ABI boundary: the library loads and exports every entry
point declared in include/*.h, and the ctypes table matches the header (no GPU calls)."""
import ctypes
import glob
import os
import re

from avsr_amd import _lib as L

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    names = set()
    for h in glob.glob(os.path.join(ROOT, "include", "*.h")):
        src = open(h).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        names |= set(re.findall(r"\b(avsr_[a-z0-9_]+)\s*\(", src))
    return names


def test_header_symbols_exported():
    lib = L.load()
    names = _declared()
    assert len(names) >= 5
    for n in sorted(names):
        assert hasattr(lib, n), f"{n} declared in include/ but not exported"


def test_ctypes_table_covers_header():
    assert _declared() <= set(L.SYMBOLS), sorted(_declared() - set(L.SYMBOLS))


def test_version_string():
    assert L.load().avsr_version().decode().startswith("avsr_hip")


def test_struct_sizes_match_c_layout():
    # int fields then 8-byte aligned pointers/int64: ctypes follows the C ABI
    assert ctypes.sizeof(L.GemmParams) % 8 == 0
    assert ctypes.sizeof(L.ConvParams) % 8 == 0


def test_conv_stat_tiles_per_dtype():
    """regression of the round-2 s3h fault: the BN partial-statistics buffer of a conv forward
    is sized by avsr_conv_stat_tiles, whose tile height must be the one the dtype's path
    launches — 192-row tiles on the bf16 LDS-DMA path where they pay (ResNet stage 2 at C2,
    M = 6000 x 11 x 11), the 128-row register-staged tile for fp32. Host-side query, no GPU."""
    from avsr_amd import ops
    g = ops.ConvGeom(6000, 11, 11, 128, 128, 3, 3, (1, 1), (1, 1))
    M = 6000 * 11 * 11
    assert ops.conv_stat_tiles(g, L.AVSR_BF16) == -(-M // 192)
    assert ops.conv_stat_tiles(g, L.AVSR_F32) == -(-M // 128)
    # a shape below the 192 rule stays on 128 rows for both
    g2 = ops.ConvGeom(8, 11, 11, 128, 128, 3, 3, (1, 1), (1, 1))
    assert ops.conv_stat_tiles(g2, L.AVSR_BF16) == ops.conv_stat_tiles(g2, L.AVSR_F32) == -(-8 * 121 // 128)
    # N <= 64 (stage 1): 256-row tiles on both paths
    g3 = ops.ConvGeom(6000, 22, 22, 64, 64, 3, 3, (1, 1), (1, 1))
    assert ops.conv_stat_tiles(g3, L.AVSR_BF16) == ops.conv_stat_tiles(g3, L.AVSR_F32) == -(-6000 * 484 // 256)


def _header_option_defaults():
    """{AVSR_OPT_name: default} from the bracketed defaults in avsr_hip.h's option table"""
    src = open(os.path.join(ROOT, "include", "avsr_hip.h")).read()
    return {m.group(1): int(m.group(2)) for m in re.finditer(r"\*\s+(AVSR_OPT_[A-Z0-9_]+)\s+\[(-?\d+)\]", src)}


def test_kernel_options_declared_and_defaulted():
    """every kernel-selection knob is a declared option (avsr_set_option / avsr_get_option) with
    the default the header documents; Python's name table covers them all"""
    lib = L.load()
    doc = _header_option_defaults()
    src = open(os.path.join(ROOT, "include", "avsr_hip.h")).read()
    ids = {m.group(1): int(m.group(2)) for m in re.finditer(r"\b(AVSR_OPT_[A-Z0-9_]+)\s*=\s*(\d+)", src)}
    count = ids.pop("AVSR_OPT_COUNT")
    assert set(doc) == set(ids) and len(ids) == count == len(L.OPTIONS)
    for name, i in ids.items():
        assert lib.avsr_get_option(i) == doc[name], name
        assert L.OPTIONS[name[len("AVSR_OPT_"):].lower()] == i
    assert lib.avsr_get_option(count) == -1 and lib.avsr_get_option(-1) == -1


def test_set_option_roundtrip_and_range():
    lib = L.load()
    assert lib.avsr_set_option(L.OPTIONS["attn_sq_bwd"], 2) == 1004          # AVSR_E_ARG: out of range
    assert lib.avsr_set_option(99, 0) == 1004                                  # unknown option
    prev = L.set_option("gemm_tile", "192")
    try:
        assert L.get_option("gemm_tile") == L.TILES.index("192") + 1
        assert lib.avsr_set_option(L.OPTIONS["gemm_tile"], len(L.TILES) + 1) == 1004
    finally:
        L.set_option("gemm_tile", prev)
    assert L.get_option("gemm_tile") == 0


def test_library_reads_no_environment():
    """kernel selection does not depend on process environment: no getenv in the sources, and
    the built library imports no getenv"""
    for f in glob.glob(os.path.join(ROOT, "avsr_amd", "csrc", "*")):
        assert "getenv" not in open(f).read(), f
    import subprocess
    out = subprocess.run(["nm", "-D", "--undefined-only", L.LIB_PATH], capture_output=True, text=True).stdout
    assert "getenv" not in out
