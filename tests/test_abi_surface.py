"""The C-ABI boundary: both libraries load and export every entry point include/swimhip.h declares.

No compute calls are made here, so the test runs without a GPU. The product library is libswimhip.so (gfx950). The
oracle exports the same ABI for parity tests only.
"""
import re
from pathlib import Path

import pytest

from swimhip import _abi, LIB_PATH

HEADER = Path(__file__).resolve().parent.parent / "include" / "swimhip.h"
SHARD_HEADER = Path(__file__).resolve().parent.parent / "include" / "swimhip_shard.h"
SELFTEST_HEADER = Path(__file__).resolve().parent.parent / "include" / "swimhip_selftest.h"
WIRE_HEADER = Path(__file__).resolve().parent.parent / "include" / "swimhip_wire.h"
DEBUG_HEADER = Path(__file__).resolve().parent.parent / "include" / "swimhip_debug.h"


def declared_symbols(header=HEADER):
    text = header.read_text()
    return sorted(set(re.findall(r"\b(swim_[a-z0-9_]+)\s*\(", text)) - {"swim_exchange_fn"})


def test_header_and_ctypes_agree():
    assert set(declared_symbols()) == set(_abi.SIGNATURES), "ctypes mirror out of sync with include/swimhip.h"


def test_shard_header_and_ctypes_agree():
    assert set(declared_symbols(SHARD_HEADER)) == set(_abi.SHARD_SIGNATURES)


def test_wire_header_and_ctypes_agree():
    assert set(declared_symbols(WIRE_HEADER)) == set(_abi.WIRE_SIGNATURES)


def test_selftest_header_and_ctypes_agree():
    assert set(declared_symbols(SELFTEST_HEADER)) == set(_abi.SELFTEST_SIGNATURES)


def test_debug_header_and_ctypes_agree():
    assert set(declared_symbols(DEBUG_HEADER)) == set(_abi.DEBUG_SIGNATURES)
    text = DEBUG_HEADER.read_text()
    for i, name in enumerate(_abi.FB_NAMES):  # index constants match the Python names
        assert re.search(rf"#define SWIM_FB_{name.upper()}\s+{i}u", text), name


def test_oracle_exports_every_symbol(oracle):
    for name in declared_symbols() + declared_symbols(SELFTEST_HEADER):
        assert hasattr(oracle, name), name


def test_engine_library_exports_every_symbol():
    if not LIB_PATH.exists():
        pytest.skip("libswimhip.so not built (run __graft_entry__.build())")
    lib = _abi.load(LIB_PATH)  # loading initialises no device
    for name in (declared_symbols() + declared_symbols(SHARD_HEADER) + declared_symbols(SELFTEST_HEADER)
                 + declared_symbols(WIRE_HEADER) + declared_symbols(DEBUG_HEADER)):
        assert hasattr(lib, name), name
    assert lib.swim_abi_version() == 1
    # pure helpers run on the host side of the library
    assert lib.swim_ceil_log2(100_000) == 17
    assert lib.swim_is_overrides(_abi.ST_ALIVE, 1, _abi.ST_SUSPECT, 0) == 1
