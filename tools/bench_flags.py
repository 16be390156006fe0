"""bench.py with engine module constants overridden (A/B runs of a Python-side switch):
  python tools/bench_flags.py _ATTN_DB=0 [NAME=VALUE | opt:OPTION=VALUE ...] -- <bench.py arguments>"""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from avsr_amd import engine  # noqa: E402

i = sys.argv.index("--")
for kv in sys.argv[1:i]:
    k, v = kv.split("=")
    if k.startswith("opt:"):                 # a library option (avsr_set_option)
        from avsr_amd import _lib
        _lib.set_option(k[4:], int(v))
        continue
    assert hasattr(engine, k), k
    setattr(engine, k, type(getattr(engine, k))(int(v)) if isinstance(getattr(engine, k), (bool, int)) else v)
sys.argv = ["bench.py"] + sys.argv[i + 1:]
import bench  # noqa: E402
sys.exit(bench.main())
