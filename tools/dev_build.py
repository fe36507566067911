#!/usr/bin/env python3
"""Incremental developer build of lib/libhmcx.so: recompiles only sources newer than their objects
(or those named on the command line), with __graft_entry__'s flags, then relinks.  build() in
__graft_entry__.py stays the full, from-scratch build the driver runs."""
import os
import re
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import __graft_entry__ as g  # noqa: E402

objdir = os.path.join(g.PKG, "lib", "obj")
os.makedirs(objdir, exist_ok=True)
force = set(sys.argv[1:])
INC = re.compile(r'^\s*#\s*include\s+"([^"]+)"', re.M)


def deps(path, seen):
    """The source and every local header it includes, transitively."""
    if path in seen or not os.path.exists(path):
        return seen
    seen.add(path)
    with open(path) as fh:
        for name in INC.findall(fh.read()):
            for d in (g.CSRC, os.path.join(REPO, "include")):
                deps(os.path.join(d, name), seen)
    return seen


def stale(unit):
    src, objname, _ = unit
    obj = os.path.join(objdir, objname)
    if src in force or objname in force or not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return any(os.path.getmtime(f) > t for f in deps(os.path.join(g.CSRC, src), set()))


def compile_one(unit):
    src, objname, extra = unit
    obj = os.path.join(objdir, objname)
    r = subprocess.run([g._hipcc()] + g.FLAGS + extra + ["-c", os.path.join(g.CSRC, src), "-o", obj],
                       capture_output=True, text=True)
    if r.returncode != 0:
        sys.exit("hipcc failed for %s:\n%s" % (objname, r.stderr[-6000:]))
    print("compiled", objname, flush=True)


todo = sorted([u for u in g.UNITS if stale(u)], key=lambda u: u[0] != "hmcx_mlp.hip")
with ThreadPoolExecutor(max_workers=8) as ex:
    list(ex.map(compile_one, todo))
objs = [os.path.join(objdir, u[1]) for u in g.UNITS]
r = subprocess.run([g._hipcc(), "--offload-arch=gfx950", "-shared", "-fPIC", "-o", g.LIB] + objs +
                   ["-ldl", "-Wl,-rpath," + g.ROCM_LIB], capture_output=True, text=True)
if r.returncode != 0:
    sys.exit("link failed:\n" + r.stderr[-4000:])
print("linked", os.path.relpath(g.LIB, REPO))
