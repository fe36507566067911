#!/usr/bin/env python3
"""A/B variant of lib/libhmcx.so: the built objects of lib/obj with ONE unit recompiled under extra
flags, linked as lib/<name> (loaded with HMCX_LIB=<name>, tools/gpu_lib_ab.sh).
    python tools/build_variant.py libhmcx_base.so hmcx_persist2.hip -DHMCX_P2_MERGE=0
SRC=<path> compiles that file in place of the unit's source (e.g. `git show HEAD:<path>` saved elsewhere:
the committed version against the working tree)."""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import __graft_entry__ as g  # noqa: E402

name, src, extra = sys.argv[1], sys.argv[2], sys.argv[3:]
objdir = os.path.join(g.PKG, "lib", "obj")
objs = []
for s, objname, ex in g.UNITS:
    obj = os.path.join(objdir, objname)
    if s == src:
        obj = os.path.join(objdir, "variant_" + objname)
        path = os.environ.get("SRC") or os.path.join(g.CSRC, s)
        subprocess.run([g._hipcc()] + g.FLAGS + ex + extra + (["-x", "hip"] if os.environ.get("SRC") else []) + ["-c", path, "-o", obj], check=True)
    objs.append(obj)
out = os.path.join(g.PKG, "lib", name)
subprocess.run([g._hipcc(), "--offload-arch=gfx950", "-shared", "-fPIC", "-o", out] + objs +
               ["-ldl", "-Wl,-rpath," + g.ROCM_LIB], check=True)
print("linked", out)
