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
