#!/usr/bin/env python3
"""Disassembly of one kernel from a built library or object (gfx950 code objects of its .hip_fatbin).
    python tools/isa_dump.py <lib.so|obj.o> <mangled-name-substring> [out.s]"""
import os
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import kernel_resources as kr  # noqa: E402

OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"


def dump(path, name):
    for co in kr.code_objects(kr.fatbin(path)):
        with tempfile.NamedTemporaryFile(suffix=".co") as fh:
            fh.write(co)
            fh.flush()
            txt = subprocess.run([OBJDUMP, "-d", "--no-show-raw-insn", fh.name], capture_output=True,
                                 text=True).stdout
        out, on = [], False
        for line in txt.splitlines():
            if line.endswith(">:") and "<" in line:
                on = name in line
            if on:
                out.append(line)
        if out:
            return "\n".join(out)
    return ""


if __name__ == "__main__":
    s = dump(sys.argv[1], sys.argv[2])
    if len(sys.argv) > 3:
        open(sys.argv[3], "w").write(s)
    else:
        print(s)
