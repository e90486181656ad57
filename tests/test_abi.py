"""CPU tests of the C-ABI boundary: the library loads, exports every symbol that
include/rf_amd.h declares, refuses to run without a HIP device, and its host-only helpers
match the reference formulas. No GPU compute is issued here."""
import ctypes
import os
import re

import pytest

from conftest import ROOT
from splinterdb_amd import build as B
from splinterdb_amd import engine as E


def header_symbols():
    """every rf_amd_* entry point declared in include/*.h (the product interface rf_amd.h
    and the diagnostics header rf_amd_diag.h)"""
    syms = set()
    for h in sorted(os.listdir(os.path.join(ROOT, "include"))):
        if h.endswith(".h"):
            src = open(os.path.join(ROOT, "include", h)).read()
            src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
            syms |= set(re.findall(r"\b(rf_amd_[a-z0-9_]+)\s*\(", src))
    return sorted(syms)


def test_library_builds_and_loads():
    B.build()
    L = E.load_library()
    assert L is not None


def test_exports_every_declared_symbol():
    L = E.load_library()
    syms = header_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(L, s), f"{s} declared in include/ but not exported"
    assert sorted(E.EXPORTED) == syms


def test_no_cpu_fallback_without_device():
    import torch
    if torch.cuda.device_count() > 0:
        pytest.skip("a HIP device is present")
    with pytest.raises(E.PlatformStatusError) as ei:
        E.Engine(0)
    assert ei.value.code == E.STATUS_NO_DEVICE


def test_max_fingerprints():
    # src/routing_filter.h:120-127 with 4 KiB pages, 32-page extents
    assert E.routing_filter_max_fingerprints(E.routing_config_init(log_index_size=8)) == 8388607
    assert E.routing_filter_max_fingerprints(E.routing_config_init(log_index_size=9)) == 16777215


def test_estimate_unique_keys_from_count_matches_oracle(oracle):
    cfg = E.routing_config_init()
    ocfg = oracle.make_config()
    for u in (0, 1, 17, 1000, 992680, 4254486, 7548068):
        assert E.routing_filter_estimate_unique_keys_from_count(cfg, u) == \
            oracle.estimate_unique_keys_from_count(ocfg, u)


def test_space_use_bytes_formula():
    cfg = E.routing_config_init()
    L = E.load_library()
    # 291 data pages -> 1,445,888 B; 1366 -> 5,771,264 B
    assert L.rf_amd_space_use_bytes(ctypes.byref(cfg.c()), 291) == 1445888
    assert L.rf_amd_space_use_bytes(ctypes.byref(cfg.c()), 1366) == 5771264


def test_get_next_value_and_is_found():
    fv = (1 << 5) | (1 << 3) | 1
    seq, last = [], E.ROUTING_NOT_FOUND
    while True:
        last = E.routing_filter_get_next_value(fv, last)
        if last == E.ROUTING_NOT_FOUND:
            break
        seq.append(last)
    assert seq == [5, 3, 0]
    assert E.routing_filter_is_value_found(fv, 3) and not E.routing_filter_is_value_found(fv, 4)
