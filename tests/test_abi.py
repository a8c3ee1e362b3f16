"""C-ABI boundary checks that need no GPU: the library loads, and exports every
symbol include/gfslam/abi.h declares (no compute calls)."""
import ctypes
import os

import pytest

from gf_orb_slam_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_library_loads():
    lib = _lib.lib()
    assert lib.gf_version() >= 1


def test_every_declared_symbol_is_exported():
    lib = _lib.lib()
    syms = _lib.declared_symbols()
    assert len(syms) >= 10
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing


def test_every_declared_symbol_has_ctypes_prototype():
    """Without argtypes ctypes truncates pointers to int: every entry point the
    Python mirror can call must carry a prototype matching the header's arity."""
    import re

    src = re.sub(r"/\*.*?\*/", "", open(_lib.ABI_HEADER).read(), flags=re.S)
    protos = dict(re.findall(r"\bint\s+(gf_[a-z0-9_]+)\s*\(([^)]*)\)", src))
    _lib.lib()
    missing = sorted(set(protos) - set(_lib._PROTOS) - {"gf_version"})
    assert not missing, missing
    for name, args in protos.items():
        if name in _lib._PROTOS:
            n = 0 if args.strip() in ("", "void") else args.count(",") + 1
            assert len(_lib._PROTOS[name]) == n, (name, len(_lib._PROTOS[name]), n)


def test_error_codes_without_device():
    lib = _lib.lib()
    n = ctypes.c_int(-1)
    assert lib.gf_device_count(ctypes.byref(n)) == 0
    assert n.value >= 0
    # null-argument behaviour is checked before any device work
    assert lib.gf_ctx_create(0, None) == -1
    assert lib.gf_extractor_capacity(None, None) == -1


def test_keypoint_layout():
    assert ctypes.sizeof(_lib.KeyPoint) == 28


def test_select_port_matches_libstdcxx():
    """select.h (device port of std::nth_element / std::priority_queue) built
    for the host agrees with libstdc++ on tie-heavy random inputs."""
    h = ctypes.CDLL(os.path.join(ROOT, "tests", "helpers", "libselcheck.so"))
    assert h.select_check(3000, 12345) == 0
