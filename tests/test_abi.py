"""The C-ABI library loads and exports every symbol include/mpcqp.h declares (no compute
calls: this runs without a GPU)."""
import ctypes as C
import os
import re
import subprocess

import pytest

from conftest import ROOT


def declared_symbols():
    txt = open(os.path.join(ROOT, "include", "mpcqp.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(mpcqp_\w+)\s*\(", txt)))


def test_header_declares_expected_entry_points():
    import mpcqp
    syms = declared_symbols()
    assert set(mpcqp.EXPORTS) == set(syms), set(mpcqp.EXPORTS) ^ set(syms)


def test_library_exports_every_declared_symbol():
    import mpcqp
    L = mpcqp.lib()
    for s in declared_symbols():
        assert hasattr(L, s), s
    out = subprocess.run(["nm", "-D", "--defined-only", mpcqp.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r"\bT (mpcqp_\w+)", out))
    assert set(declared_symbols()) <= exported


def test_library_is_gfx950_code_object():
    import mpcqp
    data = open(mpcqp.LIB_PATH, "rb").read()  # the embedded code-object bundle names its target
    assert b"amdgcn-amd-amdhsa--gfx950" in data


def test_status_strings_without_device():
    import mpcqp
    L = mpcqp.lib()
    for code, name in ((0, b"OK"), (2, b"infeasible"), (7, b"no HIP device")):
        assert L.mpcqp_status_string(code) == name


def test_header_compiles_as_c_and_cpp(tmp_path):
    src = tmp_path / "t.c"
    src.write_text('#include "mpcqp.h"\nint main(void){ mpcqp_model m; (void)m; return 0; }\n')
    inc = os.path.join(ROOT, "include")
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-I", inc, "-c", str(src), "-o",
                    str(tmp_path / "t.o")], check=True)
    subprocess.run(["g++", "-std=c++17", "-Wall", "-Werror", "-x", "c++", "-I", inc, "-c",
                    str(src), "-o", str(tmp_path / "t2.o")], check=True)


def test_model_struct_layout_matches_header(tmp_path):
    """ctypes mirror of mpcqp_model has the C size/offsets"""
    import mpcqp._lib as ml
    src = tmp_path / "s.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "mpcqp.h"\n'
                   'int main(void){printf("%zu %zu %zu %zu\\n", sizeof(mpcqp_model),'
                   ' offsetof(mpcqp_model, Q), offsetof(mpcqp_model, max_free),'
                   ' offsetof(mpcqp_model, Ib)); return 0;}\n')
    exe = tmp_path / "s"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)],
                   check=True)
    size, offQ, offmf, offIb = map(int, subprocess.run([str(exe)], capture_output=True,
                                                        text=True).stdout.split())
    M = ml.Model
    assert C.sizeof(M) == size
    assert M.Q.offset == offQ and M.max_free.offset == offmf and M.Ib.offset == offIb


def test_host_register_refuses_unaligned_start():
    """mpcqp_host_register (include/mpcqp.h) takes page-aligned starts only, checked before any
    device call: two registrations never share a page"""
    import ctypes as C
    import numpy as np
    import mpcqp
    from mpcqp._lib import lib
    a = mpcqp.page_aligned(np.arange(1000.0))
    assert a.ctypes.data % 4096 == 0 and np.array_equal(a, np.arange(1000.0))
    assert lib().mpcqp_host_register(C.c_void_p(a.ctypes.data + 8), C.c_size_t(64)) == 6
