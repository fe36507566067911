#!/usr/bin/env python3
"""Per-kernel register / scratch figures of the gfx950 code objects inside a built library.

Reads the clang offload bundles of the library's .hip_fatbin section (one per compile unit), extracts
each gfx950 code object and prints, from its AMDHSA metadata note (llvm-readelf --notes), every
kernel's VGPR / AGPR / SGPR counts, spill counts and private segment (scratch) size.  A kernel that
spills to scratch is slow by an order of magnitude (round 5: a k_wgrad edit went from 160 VGPRs to 2,264
spilled ones, 20.6 → 175 µs per step), so `--check` exits non-zero when any kernel has scratch.

    python tools/kernel_resources.py [lib.so] [--check] [--grep REGEX]
"""
import os
import re
import struct
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
READELF = "/opt/rocm/lib/llvm/bin/llvm-readelf"


def fatbin(path):
    """Bytes of the .hip_fatbin section."""
    out = subprocess.run([READELF, "-S", "-W", path], capture_output=True, text=True, check=True).stdout
    for line in out.splitlines():
        if ".hip_fatbin" in line:
            f = line.split("]", 1)[1].split()
            off, size = int(f[3], 16), int(f[4], 16)
            with open(path, "rb") as fh:
                fh.seek(off)
                return fh.read(size)
    raise SystemExit("no .hip_fatbin section in %s" % path)


def code_objects(blob, arch="gfx950"):
    """Every code object for `arch` in the concatenated offload bundles."""
    pos = 0
    while True:
        i = blob.find(MAGIC, pos)
        if i < 0:
            return
        n = struct.unpack_from("<Q", blob, i + 24)[0]
        q = i + 32
        for _ in range(n):
            off, size, tl = struct.unpack_from("<QQQ", blob, q)
            triple = blob[q + 24:q + 24 + tl].decode()
            q += 24 + tl
            if arch in triple and size:
                yield blob[i + off:i + off + size]
        pos = i + len(MAGIC)


def kernels(co):
    """The kernels' metadata maps (amdhsa.kernels of the code object's AMDGPU metadata note)."""
    import yaml
    with tempfile.NamedTemporaryFile(suffix=".co") as fh:
        fh.write(co)
        fh.flush()
        notes = subprocess.run([READELF, "--notes", fh.name], capture_output=True, text=True, check=True).stdout
    i = notes.find("---")
    j = notes.find("\n...", i)
    if i < 0 or j < 0:
        return []
    meta = yaml.safe_load(notes[i:j])
    return [{k.lstrip("."): v for k, v in kd.items() if k != ".args"} for kd in meta.get("amdhsa.kernels", [])]


def demangle(names):
    r = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True)
    return r.stdout.splitlines() if r.returncode == 0 else names


def main():
    argv = sys.argv[1:]
    args = [a for i, a in enumerate(argv) if not a.startswith("--") and (i == 0 or argv[i - 1] != "--grep")]
    lib = args[0] if args else os.path.join(REPO, "dropout_hamiltonian_montecarlo_amd", "lib", "libhmcx.so")
    pat = None
    if "--grep" in sys.argv:
        pat = re.compile(sys.argv[sys.argv.index("--grep") + 1])
    ks = {}
    for co in code_objects(fatbin(lib)):
        for k in kernels(co):
            ks[k["symbol"][:-3]] = k
    names = sorted(ks)
    bad = 0
    for sym, dn in zip(names, demangle(names)):
        k = ks[sym]
        scratch = int(k.get("private_segment_fixed_size", 0))
        if pat and not pat.search(dn):
            continue
        flag = "  SCRATCH" if scratch else ""
        bad += bool(scratch)
        print("%-90s vgpr %4s agpr %3s sgpr %3s spill v%s s%s scratch %5d lds %6s%s" % (
            dn[:90], k.get("vgpr_count"), k.get("agpr_count", "0"), k.get("sgpr_count"), k.get("vgpr_spill_count", "0"),
            k.get("sgpr_spill_count", "0"), scratch, k.get("group_segment_fixed_size", "?"), flag))
    print("%d kernels, %d with scratch" % (len(names), bad))
    if "--check" in sys.argv and bad:
        sys.exit(1)


if __name__ == "__main__":
    main()
