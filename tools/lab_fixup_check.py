"""Run the fixup-pass GPU tests (rows past the no-max kernel's range) against a lab build of the library:
the product tests call gigapath._hip.load_library(), which returns the build loaded here first.

    python tools/lab_fixup_check.py tools/attn_lab/liblab_x.so
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "prov-gigapath-replication_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)

from gigapath import _hip  # noqa: E402

_hip._lib = _hip.load_library(os.path.join(ROOT, sys.argv[1]))
import test_gpu_kernels as t  # noqa: E402

t.test_attention_no_max_overflow_fixup()
print("no_max_overflow_fixup ok", flush=True)
t.test_attention_fp16_qk_bf16_v_overflow_fixup()
print("fp16_qk_bf16_v_overflow_fixup ok", flush=True)
for case in t.KEY_PART_CASES:
    t.test_key_parts_combine_to_the_branch_softmax(*case)
    print("key parts", case[0], "ok", flush=True)
