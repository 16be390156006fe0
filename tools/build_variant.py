"""Build an A/B variant of libavsr_hip.so with extra preprocessor definitions into ab/NAME/
(git-ignored; travels to the GPU box like the product library). Load it with
AVSR_LIB_PATH_AB=ab/NAME/libavsr_hip.so (avsr_amd/_lib.py). Experiments only.
  python tools/build_variant.py NAME -DMACRO=VALUE [...]"""
import concurrent.futures as cf
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from avsr_amd import build as B  # noqa: E402

name, defs = sys.argv[1], sys.argv[2:]
out = os.path.join(ROOT, "ab", name)
os.makedirs(out, exist_ok=True)


def comp(src):
    obj = os.path.join(out, os.path.basename(src)[:-4] + ".o")
    r = subprocess.run([B.HIPCC] + B.FLAGS + defs + ["-c", src, "-o", obj], capture_output=True, text=True)
    if r.returncode:
        raise RuntimeError(r.stderr[-4000:])
    return obj


with cf.ThreadPoolExecutor(8) as ex:
    objs = list(ex.map(comp, B._sources()))
lib = os.path.join(out, "libavsr_hip.so")
r = subprocess.run([B.HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", lib] + objs, capture_output=True, text=True)
if r.returncode:
    raise RuntimeError(r.stderr[-4000:])
for o in objs:
    os.remove(o)
print("built", lib, defs)
