"""Product library vs the round-1 lab library (tools/attn_lab/liblab_r01.so), bit for bit, on one GPU.

    make -C tools/attn_lab && python tools/lab_check.py [--out gpurun_out/lab_check.json]

The product .so has every kernel variant fixed at compile time; the lab .so is the round-1 source
with its run-time variant switches.  Each case runs the same inputs through the product launch and
through the lab variant the product launch replaced, and requires identical bytes:
  * attention, D = 48 pre-scaled (no-max kernel + fixup pass) on the kernel-test schedules and the
    full 70,001-token C3 schedule, and on an input that overflows the no-max kernel (fixup path);
  * attention through the register-staged exact kernel (q not pre-scaled, D = 48 and 64; D = 64
    pre-scaled) and D = 96 (16x16x32 kernel);
  * the varlen (packed slides) launch;
  * GELU+LN: the product's table-copy kernel vs the lab's self-filling table kernel (GP_GELU_IMPL=4)
    and the per-element v2 kernel (GP_GELU_IMPL=3), F = 3072 and 4096; F = 6144 vs v2.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "prov-gigapath-replication_amd"))
import torch  # noqa: E402

from gigapath import _hip, runtime  # noqa: E402

LAB = os.path.join(ROOT, "tools", "attn_lab", "liblab_r01.so")
SEGS, RATIOS = [1024, 5792, 32768, 185363, 1048576], [1, 2, 4, 8, 16]


class use_lib:
    def __init__(self, lib, env=None):
        self.lib, self.env = lib, env or {}

    def __enter__(self):
        self.old = _hip._lib
        _hip._lib = self.lib
        self.saved = {k: os.environ.get(k) for k in self.env}
        os.environ.update(self.env)

    def __exit__(self, *exc):
        _hip._lib = self.old
        for k, v in self.saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
        return False


def qkv_rand(L, E, seed, qscale):
    g = torch.Generator(device="cuda").manual_seed(seed)
    qkv = torch.randn(L, 3 * E, device="cuda", generator=g)
    qkv[:, :E] *= qscale
    return qkv.to(torch.bfloat16)


def run_attn(qkv, L, H, D, segs, ratios, pre):
    E = H * D
    sc = runtime.AttentionScratch(torch.device("cuda"), 1, L, H, D, segs, ratios)
    for t in sc.outs + sc.lses:
        t.fill_(7.0)
    _hip.dilated_attn_fwd(qkv, qkv[:, E:], qkv[:, 2 * E:], 3 * E, 1, L, H, D, segs, ratios, sc.outs, sc.lses, 0.0, pre)
    torch.cuda.synchronize()
    return [t.clone() for t in sc.outs + sc.lses]


def same(a, b):
    return all(torch.equal(x.view(torch.uint8), y.view(torch.uint8)) for x, y in zip(a, b))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    prod = _hip.load_library()
    lab = _hip.load_library(LAB)
    res = {}
    H = 16
    cases = [("default_1025", 1025, SEGS, RATIOS), ("misaligned_200", 200, [32, 60, 90, 120, 1000], RATIOS),
             ("wsi250k_700", 700, [64, 130, 250, 333, 1000], RATIOS), ("tiny_5", 5, [1024, 5792], [1, 16]),
             ("c2_16385", 16385, SEGS, RATIOS), ("c3_70001", 70001, SEGS, RATIOS)]
    # D = 48 pre-scaled: product fast + fixup vs lab VAR 1390594 (its default)
    for name, L, segs, ratios in cases:
        qkv = qkv_rand(L, H * 48, L, 0.35)
        with use_lib(prod):
            a = run_attn(qkv, L, H, 48, segs, ratios, True)
        with use_lib(lab, {"GP_ATTN_IMPL": "2", "GP_ATTN_VAR": "1390594"}):
            b = run_attn(qkv, L, H, 48, segs, ratios, True)
        res["attn48_pre_" + name] = same(a, b)
    # overflow -> fixup pass
    L, E = 300, H * 48
    qkv = (torch.randn(L, 3 * E, device="cuda") * 0.3)
    qkv[:, 0:96] = 0.0
    qkv[:, 0] = 8.0
    qkv[:, 48] = 8.0
    qkv[:, E:E + 96] = 0.0
    qkv[150, E] = 25.0
    qkv[:, E + 48] = (torch.arange(L, device="cuda") // 64).float() * 3.75
    qkv = qkv.to(torch.bfloat16)
    with use_lib(prod):
        a = run_attn(qkv, L, H, 48, [300], [1], True)
    with use_lib(lab, {"GP_ATTN_IMPL": "2", "GP_ATTN_VAR": "1390594"}):
        b = run_attn(qkv, L, H, 48, [300], [1], True)
    res["attn48_overflow_fixup"] = same(a, b)
    # register-staged exact kernel (lab: impl 2, VAR 0 -- the run-time default when unset)
    for D, pre in ((48, False), (64, False), (64, True)):
        L = 5000
        qkv = qkv_rand(L, H * D, D, 0.35 if pre else 1.0)
        with use_lib(prod):
            a = run_attn(qkv, L, H, D, SEGS, RATIOS, pre)
        with use_lib(lab, {"GP_ATTN_IMPL": "2", "GP_ATTN_VAR": "0"}):
            b = run_attn(qkv, L, H, D, SEGS, RATIOS, pre)
        res["attn%d_%s_gen" % (D, "pre" if pre else "plain")] = same(a, b)
    qkv = qkv_rand(3000, H * 96, 96, 1.0)
    with use_lib(prod):
        a = run_attn(qkv, 3000, H, 96, SEGS, RATIOS, False)
    with use_lib(lab, {"GP_ATTN_IMPL": "1", "GP_ATTN_VAR": "0"}):
        b = run_attn(qkv, 3000, H, 96, SEGS, RATIOS, False)
    res["attn96"] = same(a, b)
    # varlen
    Ls = [1025, 2897, 700, 6001, 12000]
    qkv = qkv_rand(sum(Ls), 768, 5, 0.35)
    outs = {}
    for nm, lib, env in (("prod", prod, None), ("lab", lab, {"GP_ATTN_IMPL": "2", "GP_ATTN_VAR": "1390594"})):
        with use_lib(lib, env):
            vs = runtime.VarlenScratch(torch.device("cuda"), Ls, H, 48, SEGS, RATIOS, qkv)
            for t in vs.outs + vs.lses:
                t.zero_()
            _hip.dilated_attn_fwd_varlen(vs.plan, True)
            torch.cuda.synchronize()
            outs[nm] = [t.clone() for t in vs.outs + vs.lses]
    res["attn48_varlen"] = same(outs["prod"], outs["lab"])
    # GELU + LN
    for F in (3072, 4096, 6144):
        g = torch.Generator(device="cuda").manual_seed(F)
        M = 4099
        f = (torch.randn(M, F, device="cuda", generator=g) * 3).to(torch.bfloat16)
        f[0, :1024] = (torch.arange(-512, 512, device="cuda").float() * 0.03).to(torch.bfloat16)
        fw = 1 + 0.1 * torch.randn(F, device="cuda", generator=g)
        fb = 0.1 * torch.randn(F, device="cuda", generator=g)
        got = {}
        for nm, lib, env in (("prod", prod, None), ("lab_self_fill", lab, {"GP_GELU_IMPL": "4"}),
                             ("lab_v2", lab, {"GP_GELU_IMPL": "3"})):
            if F == 6144 and nm == "lab_self_fill":
                continue
            with use_lib(lib, env):
                o = torch.empty(M, F, dtype=torch.bfloat16, device="cuda")
                _hip.gelu_layernorm(f, fw, fb, 1e-5, o, M, F)
                torch.cuda.synchronize()
                got[nm] = o
        for nm in got:
            if nm != "prod":
                res["gelu_ln_F%d_vs_%s" % (F, nm)] = bool(torch.equal(got["prod"].view(torch.int16),
                                                                    got[nm].view(torch.int16)))
    line = json.dumps({"bit_identical": res, "all": all(res.values())})
    print(line)
    if args.out:
        with open(args.out, "w") as fh:
            fh.write(line + "\n")
    return 0 if all(res.values()) else 1


if __name__ == "__main__":
    sys.exit(main())
