"""Probe: does the VALU-bound attention kernel overlap with an MFMA-bound GEMM on another stream?
Times N attention launches and N fc1-shaped GEMMs sequentially and on two streams concurrently.
Only one GEMM stream (two concurrent stream-K GEMMs can wait on each other's workgroups)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "prov-gigapath-replication_amd"))
import torch  # noqa: E402

from gigapath import _hip, runtime  # noqa: E402

H, D, E, F = 16, 48, 768, 3072
L = 70001
segs, ratios = [1024, 5792, 32768, 185363, 1048576], [1, 2, 4, 8, 16]
g = torch.Generator(device="cuda").manual_seed(0)
qkv = torch.randn(L, 3 * E, device="cuda", generator=g)
qkv[:, :E] *= 0.35
qkv = qkv.bfloat16()
sc = runtime.AttentionScratch(torch.device("cuda"), 1, L, H, D, segs, ratios)
a = torch.randn(L, E, device="cuda", generator=g).bfloat16()
w = torch.randn(F, E, device="cuda", generator=g).bfloat16()
b = torch.randn(F, device="cuda", generator=g).bfloat16()
f = torch.empty(L, F, device="cuda", dtype=torch.bfloat16)


def attn():
    _hip.dilated_attn_fwd(qkv, qkv[:, E:], qkv[:, 2 * E:], 3 * E, 1, L, H, D, segs, ratios, sc.outs, sc.lses, 0.0, True)


def gemm():
    torch.addmm(b, a, w.t(), out=f)


def timed(fn):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1)


N = 6
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
for _ in range(2):
    attn(); gemm()
ta = timed(lambda: [attn() for _ in range(N)])
tg = timed(lambda: [gemm() for _ in range(N * 4)])


def both():
    cur = torch.cuda.current_stream()
    s1.wait_stream(cur); s2.wait_stream(cur)
    with torch.cuda.stream(s1):
        for _ in range(N):
            attn()
    with torch.cuda.stream(s2):
        for _ in range(N * 4):
            gemm()
    cur.wait_stream(s1); cur.wait_stream(s2)


tb = timed(both)
print("attention x%d: %.2f ms; fc1 GEMM x%d: %.2f ms; sum %.2f ms; concurrent %.2f ms (%.0f%% of the sum)"
      % (N, ta, 4 * N, tg, ta + tg, tb, 100 * tb / (ta + tg)), flush=True)
