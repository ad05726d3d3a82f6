"""INTEGRATION.md §2's ctypes stub (a reference maintainer's `movierec/ncf_native.py`): its
structs are the header's, field for field (checked against the binding movierec/_native.py,
whose layouts test_native_abi.py pins to include/movierec_ncf.h).  The GPU half,
test_integration_doc_gpu.py, runs the whole block."""

import ctypes
import os
import re

from movierec import _native as N

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def stub_code():
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    sec = text[text.index("## 2."):text.index("## 3.")]
    return re.search(r"```python\n(.*?)```", sec, re.S).group(1)


def test_stub_structs_match_the_binding():
    code = stub_code()
    ns = {}
    exec(compile(code[:code.index("def _ok")].replace('_lib = ctypes.CDLL("libmovierec_ncf.so")', ""),
                 "INTEGRATION.md", "exec"), ns)
    for name, ref in (("NcfShape", N.NcfShape), ("NcfModel", N.NcfModel), ("NcfOptim", N.NcfOptim),
                      ("NcfHyper", N.NcfHyper)):
        got = ns[name]
        assert ctypes.sizeof(got) == ctypes.sizeof(ref), name
        assert [f[0] for f in got._fields_] == [f[0] for f in ref._fields_], name
        for f, _ in ref._fields_:
            assert getattr(got, f).offset == getattr(ref, f).offset, (name, f)
            assert ctypes.sizeof(dict(got._fields_)[f]) == ctypes.sizeof(dict(ref._fields_)[f]), (name, f)


def test_stub_names_every_symbol_it_uses():
    """Every function the stub calls is exported by the library and declared in the header."""
    code = stub_code()
    header = open(os.path.join(ROOT, "include", "movierec_ncf.h")).read()
    for sym in set(re.findall(r"_lib\.(ncf_\w+)", code)):
        assert re.search(r"\b%s\s*\(" % sym, header), sym
        assert sym in N._SIGNATURES, sym
    assert "ABI_VERSION" in dir(N) and "_lib.ncf_abi_version() == %d" % N.ABI_VERSION in code
