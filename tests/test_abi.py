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


def test_abi_version_matches_header_and_binding(mobheat_lib):
    from mobheat import _lib
    hdr = re.search(r"#define HM_ABI_VERSION (\d+)", open(os.path.join(ROOT, "include", "mobheat.h")).read())
    assert int(hdr.group(1)) == _lib.HM_ABI_VERSION == mobheat_lib.hm_abi_version()
    # hm_batch_out: every field is 8 bytes wide (int64 or pointer), so the declared field count fixes its size
    import ctypes
    body = re.search(r"typedef struct hm_batch_out \{(.*?)\} hm_batch_out;", open(os.path.join(ROOT, "include", "mobheat.h")).read(),
                     re.S).group(1)
    n_fields = len(re.findall(r";", re.sub(r"/\*.*?\*/", "", body, flags=re.S)))
    assert ctypes.sizeof(_lib.HmBatchOut) == 8 * n_fields
