"""Per-kernel instruction counts of a built library (llvm-objdump --offloading): MFMAs, buffer stores /
loads, LDS reads, v_exp -- to check an ablation build for dead-code elimination or a schedule change.

    python tools/isa_count.py <lib.so> [kernel-name-substring]
"""
import os
import re
import shutil
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin/llvm-objdump"
PATS = {"mfma": r"v_mfma", "bstore": r"buffer_store", "bload": r"buffer_load", "ds_read": r"ds_read",
        "exp": r"v_exp_f32", "cvt_pk": r"v_cvt_pk_bf16", "waitcnt": r"s_waitcnt", "barrier": r"s_barrier",
        "valu": r"^\s*v_"}


def counts(lib):
    with tempfile.TemporaryDirectory() as tmp:
        src = os.path.join(tmp, "lib.so")
        shutil.copy(lib, src)                       # (the bundles are extracted next to the input file)
        subprocess.run([LLVM, "--offloading", src], cwd=tmp, check=True, capture_output=True)
        out = {}
        for f in sorted(x for x in os.listdir(tmp) if "amdgcn" in x):
            dis = subprocess.run([LLVM, "-d", "-C", "--mcpu=gfx950", os.path.join(tmp, f)], check=True,
                                 capture_output=True, text=True).stdout
            cur = None
            for line in dis.splitlines():
                m = re.match(r"^[0-9a-f]+ <(.*)>:", line)
                if m:
                    cur = m.group(1)
                    out[cur] = {k: 0 for k in PATS}
                    continue
                if cur is None:
                    continue
                ins = line.split("//")[0].strip()
                for k, p in PATS.items():
                    if re.search(p, ins if k != "valu" else ins):
                        out[cur][k] += 1
        return out


if __name__ == "__main__":
    sub = sys.argv[2] if len(sys.argv) > 2 else ""
    for k, v in counts(sys.argv[1]).items():
        if sub in k:
            print(" ".join("%s=%d" % kv for kv in v.items()), k[:110])
