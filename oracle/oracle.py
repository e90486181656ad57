"""ctypes binding of the parity oracle (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module,
as the checker or the CPU baseline. The product path (splinterdb_amd) never does.
The C restatement it loads is oracle/rf_oracle.c (reference file:line cited there).
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")
REF_PA_PATH = os.path.join(HERE, "_ref", "libpackedarray_ref.so")

u8p = ctypes.POINTER(ctypes.c_uint8)
u32p = ctypes.POINTER(ctypes.c_uint32)
u64p = ctypes.POINTER(ctypes.c_uint64)


class Config(ctypes.Structure):
    _fields_ = [("fingerprint_size", ctypes.c_uint32), ("log_index_size", ctypes.c_uint32),
                ("seed", ctypes.c_uint32), ("page_size", ctypes.c_uint32),
                ("pages_per_extent", ctypes.c_uint32)]


class Filter(ctypes.Structure):
    _fields_ = [("num_fingerprints", ctypes.c_uint32), ("num_unique", ctypes.c_uint32),
                ("value_size", ctypes.c_uint32), ("num_indices", ctypes.c_uint32),
                ("num_pages", ctypes.c_uint32), ("pages_cap", ctypes.c_uint32),
                ("slots", u64p), ("pages", u8p)]


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        L.rfo_xxh32.restype = ctypes.c_uint32
        L.rfo_xxh32.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32]
        L.rfo_hash_fixed.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32,
                                     ctypes.c_uint32, ctypes.c_void_p]
        L.rfo_hash_var.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                   ctypes.c_uint32, ctypes.c_void_p]
        L.rfo_pack.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p,
                               ctypes.c_uint32, ctypes.c_uint32]
        L.rfo_unpack.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p,
                                 ctypes.c_uint32, ctypes.c_uint32]
        L.rfo_get.restype = ctypes.c_uint32
        L.rfo_get.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32]
        L.rfo_filter_new.restype = ctypes.POINTER(Filter)
        L.rfo_filter_delete.argtypes = [ctypes.POINTER(Filter)]
        L.rfo_filter_add.restype = ctypes.c_int
        L.rfo_filter_add.argtypes = [ctypes.POINTER(Config), ctypes.POINTER(Filter),
                                     ctypes.POINTER(Filter), ctypes.c_void_p,
                                     ctypes.c_uint64, ctypes.c_uint16]
        L.rfo_filter_lookup_hashes.argtypes = [ctypes.POINTER(Config), ctypes.POINTER(Filter),
                                               ctypes.c_void_p, ctypes.c_uint64,
                                               ctypes.c_void_p]
        L.rfo_estimate_unique_fp.restype = ctypes.c_int
        L.rfo_estimate_unique_fp.argtypes = [ctypes.POINTER(Config), ctypes.POINTER(Filter),
                                             ctypes.c_uint64, u32p]
        L.rfo_estimate_unique_keys_from_count.restype = ctypes.c_uint32
        L.rfo_estimate_unique_keys_from_count.argtypes = [ctypes.POINTER(Config),
                                                          ctypes.c_uint64]
        L.rfo_space_use_bytes.restype = ctypes.c_uint64
        L.rfo_space_use_bytes.argtypes = [ctypes.POINTER(Config), ctypes.POINTER(Filter)]
        L.rfo_bench_build.restype = ctypes.c_double
        L.rfo_bench_build.argtypes = [ctypes.POINTER(Config), ctypes.c_void_p, ctypes.c_uint32,
                                      ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                      ctypes.c_uint32, ctypes.c_uint16, ctypes.c_int,
                                      ctypes.POINTER(Filter)]
        L.rfo_bench_probe.restype = ctypes.c_double
        L.rfo_bench_probe.argtypes = [ctypes.POINTER(Config), ctypes.POINTER(Filter),
                                      ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p,
                                      ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p]
        L.rfo_bench_build_var.restype = ctypes.c_double
        L.rfo_bench_build_var.argtypes = [ctypes.POINTER(Config), ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                          ctypes.c_uint16, ctypes.c_int, ctypes.POINTER(Filter)]
        L.rfo_bench_probe_var.restype = ctypes.c_double
        L.rfo_bench_probe_var.argtypes = [ctypes.POINTER(Config), ctypes.POINTER(Filter),
                                          ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p]
        _lib = L
    return _lib


def make_config(fingerprint_size=26, log_index_size=8, seed=42, page_size=4096,
                pages_per_extent=32):
    return Config(fingerprint_size, log_index_size, seed, page_size, pages_per_extent)


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def xxh32(data: bytes, seed=42):
    buf = ctypes.create_string_buffer(bytes(data), max(len(data), 1))
    return lib().rfo_xxh32(buf, len(data), seed)


def hash_fixed(keys: np.ndarray, key_len: int, seed=42):
    keys = np.ascontiguousarray(keys, dtype=np.uint8)
    n = keys.size // key_len
    out = np.empty(n, dtype=np.uint32)
    lib().rfo_hash_fixed(_ptr(keys), n, key_len, seed, _ptr(out))
    return out


def hash_var(data: np.ndarray, offs: np.ndarray, seed=42):
    data = np.ascontiguousarray(data, dtype=np.uint8)
    offs = np.ascontiguousarray(offs, dtype=np.uint64)
    n = offs.size - 1
    out = np.empty(n, dtype=np.uint32)
    lib().rfo_hash_var(_ptr(data), _ptr(offs), n, seed, _ptr(out))
    return out


class OracleFilter:
    """A filter built by the oracle, with its relocatable image."""

    def __init__(self, cfg, handle):
        self.cfg = cfg
        self.h = handle

    def __del__(self):
        try:
            if self.h:
                lib().rfo_filter_delete(self.h)
        except Exception:
            pass

    @property
    def f(self):
        return self.h.contents

    @property
    def num_fingerprints(self):
        return self.f.num_fingerprints

    @property
    def num_unique(self):
        return self.f.num_unique

    @property
    def value_size(self):
        return self.f.value_size

    @property
    def num_pages(self):
        return self.f.num_pages

    @property
    def num_indices(self):
        return self.f.num_indices

    def pages(self) -> np.ndarray:
        n = self.f.num_pages * self.cfg.page_size
        return np.ctypeslib.as_array(self.f.pages, shape=(n,)).copy()

    def slots(self) -> np.ndarray:
        n = self.cfg.pages_per_extent * self.cfg.page_size // 8
        return np.ctypeslib.as_array(self.f.slots, shape=(n,)).copy()

    def lookup_hashes(self, hashes: np.ndarray) -> np.ndarray:
        hashes = np.ascontiguousarray(hashes, dtype=np.uint32)
        out = np.empty(hashes.size, dtype=np.uint64)
        lib().rfo_filter_lookup_hashes(ctypes.byref(self.cfg), self.h, _ptr(hashes),
                                       hashes.size, _ptr(out))
        return out

    def space_use_bytes(self):
        return lib().rfo_space_use_bytes(ctypes.byref(self.cfg), self.h)


def filter_add(cfg, hashes: np.ndarray, value=0, old: OracleFilter = None):
    """routing_filter_add on the oracle. `hashes` are full 32-bit XXH32 values (the
    reference shifts them in place; a copy is passed so the caller's array survives)."""
    work = np.array(hashes, dtype=np.uint32, copy=True)
    h = lib().rfo_filter_new()
    rc = lib().rfo_filter_add(ctypes.byref(cfg), old.h if old is not None else None, h,
                              _ptr(work) if work.size else None, work.size, value)
    if rc != 0:
        lib().rfo_filter_delete(h)
        raise ValueError(f"rfo_filter_add failed rc={rc}")
    return OracleFilter(cfg, h)


def estimate_unique_fp(cfg, filters):
    """None entries are NULL_ROUTING_FILTER (addr 0: skipped, :739-742)."""
    arr = (Filter * max(1, len(filters)))(*[(f.f if f is not None else Filter()) for f in filters])
    out = ctypes.c_uint32(0)
    rc = lib().rfo_estimate_unique_fp(ctypes.byref(cfg), arr, len(filters), ctypes.byref(out))
    if rc:
        raise ValueError(rc)
    return out.value


def estimate_unique_keys_from_count(cfg, num_unique):
    return lib().rfo_estimate_unique_keys_from_count(ctypes.byref(cfg), num_unique)


def seq_keys(start, n, key_len=24):
    """filter_test key format (tests/functional/filter_test.c:172-183): a little-endian
    u64 id in bytes 0-7, the rest zero."""
    k = np.zeros((n, key_len), dtype=np.uint8)
    ids = np.arange(start, start + n, dtype=np.uint64)
    k[:, :8] = ids.view(np.uint8).reshape(n, 8)
    return k.reshape(-1)


def ids_keys(ids, key_len=24):
    ids = np.asarray(ids, dtype=np.uint64)
    k = np.zeros((ids.size, key_len), dtype=np.uint8)
    k[:, :8] = ids.view(np.uint8).reshape(ids.size, 8)
    return k.reshape(-1)


# --- the reference's own PackedArray.c, compiled from its sources into _ref/ ---------
_ref_pa = None


def ref_packedarray():
    global _ref_pa
    if _ref_pa is None:
        if not os.path.exists(REF_PA_PATH):
            return None
        L = ctypes.CDLL(REF_PA_PATH)
        L.PackedArray_pack.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p,
                                       ctypes.c_uint32, ctypes.c_size_t]
        L.PackedArray_unpack.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p,
                                         ctypes.c_uint32, ctypes.c_size_t]
        L.PackedArray_get.restype = ctypes.c_uint32
        L.PackedArray_get.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_size_t]
        _ref_pa = L
    return _ref_pa
