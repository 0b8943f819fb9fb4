"""CPU-side checks of the drop-in boundary: libmqvs.so loads and exports every
entry point include/mqvs.h declares (no GPU calls)."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    with open(os.path.join(ROOT, "include", "mqvs.h")) as f:
        text = f.read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(mqvs_[a-z_]+)\s*\(", text)))


def test_header_declares_expected_entry_points():
    syms = declared_symbols()
    for s in ("mqvs_search", "mqvs_knn_raw", "mqvs_segment_create", "mqvs_rerank",
              "mqvs_merge_shards", "mqvs_last_error"):
        assert s in syms


def test_library_exports_every_declared_symbol():
    from myscaledb_amd import _lib
    for s in declared_symbols():
        assert hasattr(_lib.lib, s), f"libmqvs.so does not export {s}"
    assert sorted(_lib.SYMBOLS) == declared_symbols()


def test_abi_version():
    from myscaledb_amd import _lib
    assert _lib.lib.mqvs_abi_version() == 4


def test_library_is_gfx950_code_object():
    """The HIP fat binary carries a gfx950 code object."""
    from myscaledb_amd import _lib
    with open(_lib.LIB_PATH, "rb") as f:
        blob = f.read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob
