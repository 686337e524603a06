"""CPU: the C-ABI library loads and exports every entry point include/mobheat.h declares."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    src = open(os.path.join(ROOT, "include", "mobheat.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return set(re.findall(r"\b(hm_[a-z0-9_]+)\s*\(", src))


def test_header_and_binding_agree(mobheat_lib):
    from mobheat import _lib
    assert _declared() == set(_lib.SIGNATURES)


def test_library_exports_every_symbol(mobheat_lib):
    for name in _declared():
        assert hasattr(mobheat_lib, name), name


def test_library_is_gfx950_code_object():
    from mobheat import _lib
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


def test_missing_library_fails_loudly(monkeypatch, tmp_path):
    from mobheat import _lib
    monkeypatch.setattr(_lib, "_lib", None)
    monkeypatch.setattr(_lib, "LIB_PATH", str(tmp_path / "nope.so"))
    try:
        _lib.load()
    except RuntimeError as e:
        assert "not built" in str(e)
    else:
        raise AssertionError("load() must raise when the HIP library is missing")
