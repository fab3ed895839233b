"""Generated native launch bindings (csrc/gen_fastcall.py): the METH_FASTCALL wrappers built from the
ctypes signature table must call the same C functions with the same argument conversions as ctypes.

1. A stub C library with every argument kind (pointer / int / long / float / u64, None pointers,
   ctypes instances, int return and long return) is bound both ways and the results compared.
2. The real kernel library (loadable without a GPU) is bound through hip.lib(): the generated entry
   points agree with the ctypes handle on the host-only workspace-size functions, and both resolve
   the same mapping of the library (hip._load_fast's address check)."""
import ctypes
import importlib.util
import os
import subprocess
import sys
import sysconfig

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(ROOT, "csrc"))

STUB = r"""
#include <stdint.h>
extern "C" {
int ssamd_t_mix(void* p, int i, long l, float f, unsigned long long u, void* q) {
  // fold every argument into the result so a dropped / reordered / truncated one shows
  unsigned long long h = (unsigned long long)(uintptr_t)p * 3u + (unsigned long long)(uintptr_t)q * 5u;
  h ^= (unsigned long long)(long long)i * 7u + (unsigned long long)l * 11u + u * 13u;
  h += (unsigned long long)(long long)(f * 1000.0f);
  return (int)(h % 1000003u);
}
long ssamd_t_big(long a, int b) { return a * 4 + b; }
int ssamd_t_noargs(void) { return 42; }
}
"""


def _build_stub(tmp_path):
    import gen_fastcall as G

    P, I, L_, F, U64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_long, ctypes.c_float, ctypes.c_ulonglong
    sigs = {"ssamd_t_mix": [P, I, L_, F, U64, P], "ssamd_t_big": [L_, I], "ssamd_t_noargs": []}
    rest = {"ssamd_t_big": L_}
    so = tmp_path / "libstub.so"
    (tmp_path / "stub.cpp").write_text(STUB)
    subprocess.check_call(["g++", "-O2", "-shared", "-fPIC", "-Wl,-soname,libstub.so", "-o", str(so),
                           str(tmp_path / "stub.cpp")])
    (tmp_path / "fast.cpp").write_text(G.generate(sigs, rest, module="stubfast"))
    ext = tmp_path / ("stubfast" + sysconfig.get_config_var("EXT_SUFFIX"))
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-I", sysconfig.get_paths()["include"],
                           "-o", str(ext), str(tmp_path / "fast.cpp"), "-L", str(tmp_path), "-l:libstub.so",
                           "-Wl,-rpath,$ORIGIN"])
    h = ctypes.CDLL(str(so))
    for k, v in sigs.items():
        getattr(h, k).argtypes = v
        getattr(h, k).restype = rest.get(k, I)
    spec = importlib.util.spec_from_file_location("stubfast", str(ext))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return h, m


def test_generated_bindings_match_ctypes(tmp_path):
    h, m = _build_stub(tmp_path)
    cases = [
        (0x7F00DEAD0000, 3, 1 << 40, 0.25, 2 ** 63 + 5, None),
        (None, -7, -3, -1.5, 0, 0x1234),
        (ctypes.c_void_p(0x5000), True, 9, 2, ctypes.c_ulonglong(77), ctypes.c_void_p(None)),
    ]
    for args in cases:
        assert m.ssamd_t_mix(*args) == h.ssamd_t_mix(*args), args
    assert m.ssamd_t_big(1 << 40, 3) == h.ssamd_t_big(1 << 40, 3) == (1 << 42) + 3
    assert m.ssamd_t_noargs() == 42
    assert m.ssamd_t_big(ctypes.c_long(5), 1) == 21
    with pytest.raises(TypeError):
        m.ssamd_t_big(1)
    with pytest.raises(TypeError):
        m.ssamd_t_mix("x", 1, 2, 3.0, 4, None)
    # one mapping: the entry address the extension resolved is the ctypes handle's
    assert m._entry_addr() == ctypes.cast(getattr(h, m.entry_name), ctypes.c_void_p).value


def test_kernel_library_bindings_agree():
    from speakingstyle_amd.ops import hip

    if not os.path.exists(hip._LIB_PATH):
        pytest.skip("kernel library not built")
    L = hip.lib()
    assert hip.fast_bindings(), "generated bindings missing (csrc/build.py builds them with the library)"
    h = L._handle
    for fn, args in (("ssamd_colsum_ws", (100000, 256)), ("ssamd_addln_bwd_ws", (200, 1000, 256, 1)),
                     ("ssamd_l1pair_ws", (200, 1000, 80)), ("ssamd_head_bwd_ws", (12345, 256))):
        assert getattr(L, fn)(*args) == getattr(h, fn)(*args)
        assert not isinstance(getattr(L, fn), ctypes._CFuncPtr)  # the generated wrapper, not ctypes
    # struct-by-value entry points stay on ctypes
    assert isinstance(L.ssamd_var_loss_fwd, ctypes._CFuncPtr)


def test_sig_hash_tracks_argument_types():
    """A signature edited without a rebuild changes the digest that hip._load_fast compares, so stale
    bindings fall back to ctypes instead of converting arguments with the old types."""
    import ctypes
    import os
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "csrc"))
    import gen_fastcall

    P, I, F = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
    a = gen_fastcall.sig_hash({"ssamd_x": [P, I, F]}, {})
    assert a == gen_fastcall.sig_hash({"ssamd_x": [P, I, F]}, {})
    assert a != gen_fastcall.sig_hash({"ssamd_x": [P, F, F]}, {})  # same count, different type
    assert a != gen_fastcall.sig_hash({"ssamd_x": [P, I, F]}, {"ssamd_x": ctypes.c_long})
    assert f'"sig_hash", "{a}"' in gen_fastcall.generate({"ssamd_x": [P, I, F]}, {})
