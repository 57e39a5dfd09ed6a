"""The built library's gfx950 code has no b96/b128 buffer store whose data registers a VALU instruction
rewrites within two instructions (a hazard hipcc does not model when soffset is an SGPR;
measured to corrupt GEMM output rows).  CPU only: disassembles the in-tree .so."""
import importlib.util
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _scanner():
    spec = importlib.util.spec_from_file_location("isa_store_hazard_scan",
                                                  os.path.join(ROOT, "tools", "isa_store_hazard_scan.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_scanner_finds_the_pattern():
    s = _scanner()
    text = "\n".join(["_Zk:", "\tbuffer_store_dwordx4 v[40:43], v231, s[24:27], s78 offen",
                      "\tv_mov_b32_e32 v40, v121", "\tbuffer_store_dwordx4 v[8:11], v2, s[24:27], 0 offen",
                      "\ts_nop 1", "\tv_mov_b32_e32 v8, v1"])
    hits = s.scan_text(text)
    assert len(hits) == 1 and "v40" in hits[0][2]


def test_library_has_no_store_data_hazard():
    s = _scanner()
    if not (os.path.exists(s.LLVM) and os.path.exists(s.DEFAULT)):
        pytest.skip("llvm-objdump or the built library missing")
    hits = s.scan_library(s.DEFAULT)
    assert not hits, hits[:5]
