"""TEST INFRASTRUCTURE ONLY: the reference's whole key-value store (splinterdb.c, core.c,
trunk.c, ... compiled unmodified, oracle/ref_kvs.c) as the routing filter's caller, once with
the reference's routing_filter.c (KVS_REF) and once with the drop-in shim (KVS_SHIM).

    with Kvs(KVS_REF) as db:
        db.insert(keys, values)          # splinterdb_insert per key (memtable flushes and
                                         # trunk compactions build maplets: routing_filter_add)
        found, val8, secs = db.lookup(keys)            # splinterdb_lookup per key
        found, val8, secs = db.lookup_async(keys, 64)  # core_lookup_async, 64 in flight
        adds, n_lookups, n_async = db.adds()           # every routing_filter_add the trunk made
"""
import ctypes
import os
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
KVS_REF = os.path.join(HERE, "_ref", "libkvs_ref.so")
KVS_SHIM = os.path.join(HERE, "_ref", "libkvs_shim.so")

ADD_FIELDS = ("old_addr", "num_new", "value", "rc", "addr", "meta_head", "num_fingerprints", "num_unique",
              "value_size", "digest")


class AddRec(ctypes.Structure):
    _fields_ = [(f, ctypes.c_uint64) for f in ADD_FIELDS]


def available(path=KVS_REF):
    return os.path.exists(path)


_libs = {}


def lib(path):
    if path not in _libs:
        L = ctypes.CDLL(path)
        vp, u32, u64, i32 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int
        L.rfk_open.argtypes = [u64, u64, u64, u32, u32, i32]
        L.rfk_open.restype = vp
        L.rfk_close.argtypes = [vp]
        L.rfk_close.restype = None
        L.rfk_close_ex.argtypes = [vp, i32]
        L.rfk_close_ex.restype = None
        L.rfk_direct_stats.argtypes = [vp, ctypes.POINTER(u64)]
        L.rfk_direct_stats.restype = None
        L.rfk_add_breakdown.argtypes = [ctypes.POINTER(u64)]
        L.rfk_add_breakdown.restype = None
        L.rfk_attach.argtypes = [vp]
        L.rfk_attach.restype = i32
        L.rfk_insert.argtypes = [vp, vp, u32, vp, u32, u64]
        L.rfk_insert.restype = i32
        L.rfk_lookup.argtypes = [vp, vp, u32, u64, vp, vp]
        L.rfk_lookup.restype = ctypes.c_double
        L.rfk_lookup_async.argtypes = [vp, vp, u32, u64, vp, vp, u32]
        L.rfk_lookup_async.restype = ctypes.c_double
        L.rfk_adds.argtypes = [vp, u64, ctypes.POINTER(u64), ctypes.POINTER(u64), i32]
        L.rfk_adds.restype = u64
        _libs[path] = L
    return _libs[path]


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


class Kvs:
    def __init__(self, path=KVS_REF, cache_mib=1024, disk_mib=8192, memtable_mib=4, filter_hash_size=26,
                 filter_log_index_size=8, record_digest=True, attach=True):
        """attach=True: the shim's cache attach after the store opens (direct placement of the
        images into the cache pages) and its release before the store closes; attach=False: the
        store driven exactly as the unmodified reference does (no shim extension called)"""
        self.L = lib(path)
        self.h = self.L.rfk_open(cache_mib, disk_mib, memtable_mib, filter_hash_size, filter_log_index_size,
                                 int(record_digest))
        if not self.h:
            raise RuntimeError("splinterdb_create failed")
        self.attached = False
        self.attach_s = 0.0
        if attach:
            t = time.perf_counter()
            self.attached = self.L.rfk_attach(self.h) == 0
            self.attach_s = time.perf_counter() - t

    def close(self):
        if self.h:
            self.L.rfk_close_ex(self.h, int(self.attached))
            self.h = None

    def add_breakdown(self):
        """the shim's routing_filter_add time split (ns totals; zeros with the reference)"""
        out = (ctypes.c_uint64 * 11)()
        self.L.rfk_add_breakdown(out)
        keys = ("calls", "batches", "create", "stage", "build", "infos", "readback", "wait", "place",
                "engine_create", "register")
        return dict(zip(keys, [int(x) for x in out]))

    def direct_stats(self):
        """(caches registered, registrations found stale, adds placing now, this store's
        page-buffer address)"""
        out = (ctypes.c_uint64 * 4)()
        self.L.rfk_direct_stats(self.h, out)
        return tuple(out)

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def insert(self, keys, values):
        k = np.ascontiguousarray(keys, dtype=np.uint8)
        v = np.ascontiguousarray(values, dtype=np.uint8)
        n = k.shape[0]
        rc = self.L.rfk_insert(self.h, _p(k), k.shape[1], _p(v), v.shape[1], n)
        if rc:
            raise RuntimeError(f"splinterdb_insert: {rc}")

    def lookup(self, keys):
        k = np.ascontiguousarray(keys, dtype=np.uint8)
        n = k.shape[0]
        found = np.zeros(n, dtype=np.uint8)
        val = np.zeros(n, dtype=np.uint64)
        t = self.L.rfk_lookup(self.h, _p(k), k.shape[1], n, _p(found), _p(val))
        if t < 0:
            raise RuntimeError("splinterdb_lookup failed")
        return found.astype(bool), val, t

    def lookup_async(self, keys, max_inflight=64):
        k = np.ascontiguousarray(keys, dtype=np.uint8)
        n = k.shape[0]
        found = np.zeros(n, dtype=np.uint8)
        val = np.zeros(n, dtype=np.uint64)
        t = self.L.rfk_lookup_async(self.h, _p(k), k.shape[1], n, _p(found), _p(val), max_inflight)
        if t < 0:
            raise RuntimeError("core_lookup_async failed")
        return found.astype(bool), val, t

    def adds(self, reset=False):
        """(records of every routing_filter_add so far as a structured array, filter lookups,
        async filter lookups started)"""
        nl, na = ctypes.c_uint64(0), ctypes.c_uint64(0)
        n = self.L.rfk_adds(None, 0, ctypes.byref(nl), ctypes.byref(na), 0)
        arr = (AddRec * max(1, n))()
        n = self.L.rfk_adds(ctypes.addressof(arr), n, ctypes.byref(nl), ctypes.byref(na), int(reset))
        recs = np.array([tuple(getattr(arr[i], f) for f in ADD_FIELDS) for i in range(n)],
                        dtype=[(f, np.uint64) for f in ADD_FIELDS])
        return recs, nl.value, na.value
