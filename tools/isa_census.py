"""Instruction census of the built library's kernels (gfx950 ISA from llvm-objdump; no GPU needed).

    python tools/isa_census.py                                   # every kernel: size, VGPRs, spills
    python tools/isa_census.py -k 'dilated_attn32_kernel<48, true, 0, false, 8, false, false>' --loops
    python tools/isa_census.py -k 'gemm_kernel<12, 1, 2, false, true>' --ktile-waits
    python tools/isa_census.py --compare /tmp/other.so           # per kernel: same opcode sequence or not

Used in round 5 to check that the key-part instantiation left the product attention kernel's ISA unchanged
(`--compare` against the ABI-9 build), to count the attention loop body (MFMA / exp / cvt / VALU / SALU per
two 64-key tiles) and to compare the LN-fold and plain QKV GEMMs' K-tile LDS waits.
"""
import argparse
import collections
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "prov-gigapath-replication_amd", "gigapath", "_lib", "libgigapath_hip.so")
LLVM = "/opt/rocm/lib/llvm/bin"


def disassemble(lib):
    """(kernel name -> list of instruction strings, kernel symbol -> metadata dict) of the gfx950 code objects."""
    tmp = tempfile.mkdtemp(prefix="isa_census_")
    dst = os.path.join(tmp, "lib.so")
    subprocess.run(["cp", lib, dst], check=True)
    subprocess.run([os.path.join(LLVM, "llvm-objdump"), "--offloading", dst], check=True, cwd=tmp,
                   stdout=subprocess.DEVNULL)
    objs = sorted(f for f in os.listdir(tmp) if f.endswith("gfx950"))
    kernels, meta = {}, {}
    for f in objs:
        p = os.path.join(tmp, f)
        dis = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--mcpu=gfx950", p], check=True,
                             capture_output=True, text=True).stdout
        name, body = None, []
        for line in dis.split("\n"):
            m = re.match(r"^[0-9a-f]+ <(.*)>:$", line)
            if m:
                if name is not None:
                    kernels[name] = body
                name, body = m.group(1), []
                continue
            if name is None:
                continue
            m = re.match(r"\s*(\S.*?)\s*//\s*([0-9A-Fa-f]+):", line)
            if m:
                body.append((int(m.group(2), 16), m.group(1)))
        if name is not None:
            kernels[name] = body
        notes = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", p], check=True, capture_output=True,
                               text=True).stdout
        for blk in notes.split("- .agpr_count")[1:]:
            nm = re.search(r"\.name:\s+(\S+)", blk)
            if not nm:
                continue
            g = {k: (re.search(r"\." + k + r":\s+(\S+)", blk) or [None, None])[1]
                 for k in ("vgpr_count", "sgpr_count", "vgpr_spill_count", "sgpr_spill_count",
                           "group_segment_fixed_size")}
            meta[nm.group(1)] = g
    # mangled -> demangled names (the metadata is keyed by the mangled symbol)
    mangled = sorted(kernels)
    dem = subprocess.run(["c++filt"], input="\n".join(mangled), capture_output=True,
                         text=True, check=True).stdout.split("\n")
    kernels = {d: (kernels[m], meta.get(m, {})) for m, d in zip(mangled, dem)}
    return kernels


def short(name):
    """'void (anonymous namespace)::k<...>(Args)' -> 'k<...>'."""
    m = re.search(r"(\w+<[^()]*>|\w+)\(", name)
    return m.group(1) if m else name


def klass(ins):
    op = ins.split()[0]
    if "mfma" in op:
        return "mfma"
    if op.startswith("v_exp"):
        return "exp"
    if op.startswith("v_cvt"):
        return "cvt"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("buffer_", "global_", "scratch_")):
        return "vmem"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith("s_barrier"):
        return "barrier"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("s_"):
        return "salu"
    return "other"


def census(body):
    return dict(collections.Counter(klass(x) for x in body))


def loops(body):
    """(first, last) instruction indices of every backward branch's loop body (branch offsets are in dwords
    from the next instruction; the disassembly's address comments locate the target)."""
    at = {a: i for i, (a, _) in enumerate(body)}
    out = []
    for i, (a, x) in enumerate(body):
        m = re.match(r"s_c?branch\w*\s+(\d+)", x)
        if not m:
            continue
        off = int(m.group(1))
        off = off - 65536 if off > 32767 else off
        tgt = a + 4 + 4 * off
        if off < 0 and tgt in at:
            out.append((at[tgt], i))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib", nargs="?", default=LIB)
    ap.add_argument("-k", "--kernel", default="", help="substring of the kernel name (default: all)")
    ap.add_argument("--loops", action="store_true", help="census of each backward-branch loop body")
    ap.add_argument("--ktile-waits", action="store_true", help="LDS waits per 64 MFMAs (GEMM K-tiles)")
    ap.add_argument("--compare", default="", help="another build: same opcode sequence per kernel?")
    args = ap.parse_args()
    kernels = disassemble(args.lib)
    other = {short(k): v[0] for k, v in disassemble(args.compare).items()} if args.compare else None
    for name in sorted(kernels):
        s = short(name)
        if args.kernel and args.kernel not in s:
            continue
        insns, md = kernels[name]
        body = [x for _, x in insns]
        line = "%-70s %5d instrs vgpr %s spill %s sspill %s lds %s %s" % (
            s[:70], len(body), md.get("vgpr_count"), md.get("vgpr_spill_count"), md.get("sgpr_spill_count"),
            md.get("group_segment_fixed_size"), census(body))
        if other is not None:
            # (a template parameter appended since: the old build's name lacks a trailing ", false")
            ob = other.get(s, other.get(s[:-len(", false>")] + ">" if s.endswith(", false>") else "", None))
            ob = [x for _, x in ob] if ob is not None else None
            same = ob is not None and [x.split()[0] for x in ob] == [x.split()[0] for x in body]
            line += "  vs other: %s" % ("same opcodes" if same else ("absent" if ob is None else
                                                                      "differs (%d)" % len(ob)))
        print(line)
        if args.loops:
            for j, i in loops(insns):
                print("    loop [%d, %d] %d instrs %s" % (j, i, i - j + 1, census(body[j:i + 1])))
        if args.ktile_waits:
            n, hist = 0, collections.Counter()
            for x in body:
                if "mfma" in x.split()[0]:
                    n += 1
                elif x.startswith("s_waitcnt lgkm"):
                    hist[n // 64] += 1
            print("    lgkm waits per 64 MFMAs:", [hist[k] for k in sorted(hist)])
    return 0


if __name__ == "__main__":
    sys.exit(main())
