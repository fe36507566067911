#!/usr/bin/env python3
"""Recompile the named units of __graft_entry__.UNITS (by source file) and relink lib/libhmcx.so.
    python tools/rebuild_units.py hmcx_mlp.hip [hmcx_wide.hip ...]"""
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import __graft_entry__ as g  # noqa: E402

objdir = os.path.join(g.PKG, "lib", "obj")
units = [u for u in g.UNITS if u[0] in sys.argv[1:]]


def compile_one(u):
    r = subprocess.run([g._hipcc()] + g.FLAGS + u[2] + ["-c", os.path.join(g.CSRC, u[0]), "-o", os.path.join(objdir, u[1])],
                       capture_output=True, text=True)
    errs = [l for l in r.stderr.splitlines() if "error" in l]
    return u[1], r.returncode, "\n".join(errs[:20])


with ThreadPoolExecutor(max(1, len(units))) as ex:
    for name, rc, err in ex.map(compile_one, units):
        print(name, rc, err)
        if rc:
            sys.exit(1)
objs = [os.path.join(objdir, u[1]) for u in g.UNITS]
r = subprocess.run([g._hipcc(), "--offload-arch=gfx950", "-shared", "-fPIC", "-o", g.LIB] + objs +
                   ["-ldl", "-Wl,-rpath," + g.ROCM_LIB], capture_output=True, text=True)
print("link", r.returncode, r.stderr[-2000:])
sys.exit(r.returncode)
