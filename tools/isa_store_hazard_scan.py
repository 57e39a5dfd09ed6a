"""Scan the gfx950 code of a built library for the store-data hazard of DESIGN §3.4: a 12/16-byte
buffer store followed, within two instructions and no s_nop, by a VALU write of one of its data
registers.  hipcc only spaces the two when the store's soffset is not an SGPR; on gfx950 the store then
read the rewritten register for some lanes (measured, r03_u).

    python tools/isa_store_hazard_scan.py [path/to/libgigapath_hip.so]      # exit 1 on a hit
"""
import os
import re
import shutil
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin/llvm-objdump"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEFAULT = os.path.join(ROOT, "prov-gigapath-replication_amd", "gigapath", "_lib", "libgigapath_hip.so")


def _regs(tok):
    m = re.match(r"v\[(\d+):(\d+)\]", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"v(\d+)$", tok)
    return {int(m.group(1))} if m else set()


def scan_text(text):
    """[(function, store, following instruction)] for every hazard site in disassembly / assembly text."""
    hits, fn, ins = [], None, []
    for line in text.split("\n"):
        m = re.match(r"^(?:[0-9a-f]+ )?<?(_Z\w+)>?:", line)
        if m:
            fn = m.group(1)
            continue
        t = line.split("//")[0].split(";")[0].strip()
        if not t or t.startswith(".") or t.endswith(":"):
            continue
        ins.append((fn, t))
    for i, (fn, t) in enumerate(ins):
        op = t.split()[0]
        if not re.match(r"buffer_store_(dwordx3|dwordx4|b96|b128)$", op):
            continue
        data = _regs(t.split()[1].rstrip(","))
        for j in (1, 2):
            if i + j >= len(ins) or ins[i + j][0] != fn:
                break
            t2 = ins[i + j][1]
            op2 = t2.split()[0]
            if op2.startswith("s_nop"):
                break
            if op2.startswith("v_") and "mfma" not in op2 and len(t2.split()) > 1:
                if _regs(t2.split()[1].rstrip(",")) & data:
                    hits.append((fn, t, t2))
    return hits


def scan_library(path):
    tmp = tempfile.mkdtemp()
    try:
        lib = os.path.join(tmp, os.path.basename(path))
        shutil.copy(path, lib)
        subprocess.run([LLVM, "--offloading", lib], cwd=tmp, check=True, capture_output=True)
        hits = []
        for f in sorted(os.listdir(tmp)):
            if f.endswith("gfx950"):
                dis = subprocess.run([LLVM, "-d", "--mcpu=gfx950", os.path.join(tmp, f)], check=True,
                                     capture_output=True, text=True).stdout
                hits += scan_text(dis)
        return hits
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def main():
    path = sys.argv[1] if len(sys.argv) > 1 else DEFAULT
    hits = scan_library(path)
    for fn, a, b in hits[:20]:
        print(f"{fn[:80]}: {a}  ->  {b}")
    print(f"{len(hits)} store-data hazard sites in {path}")
    return 1 if hits else 0


if __name__ == "__main__":
    sys.exit(main())
