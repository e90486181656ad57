"""ctypes binding of the reference's OWN routing filter (TEST INFRASTRUCTURE ONLY).

oracle/_ref/libref_rf.so is vmware/splinterdb's src/routing_filter.c and the page stack it
runs on (clockcache, mini_allocator, rc_allocator, PackedArray), compiled unmodified from
/root/reference by oracle/Makefile, with ref_harness.c's in-memory device behind the
reference's io_ops interface. Only tests/, oracle/gen_ref_golden.py and bench.py's
cpu_baseline leg use it, as the checker / the CPU baseline. The library is built in this
container and travels to the GPU box as a built file; where it is absent, `available()`
is False and its users skip or fall back to the restatement.
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_ref", "libref_rf.so")
# the same harness and page stack with shim/routing_filter_amd.c (the MI355X drop-in) in
# place of routing_filter.c
SHIM_PATH = os.path.join(HERE, "_ref", "libshim_rf.so")
# each of the two stacks with the reference's tests/functional/filter_test.c test bodies
# (oracle/ref_filter_test.c #includes it unmodified)
FT_REF_PATH = os.path.join(HERE, "_ref", "libfilter_test_ref.so")
FT_SHIM_PATH = os.path.join(HERE, "_ref", "libfilter_test_shim.so")


class RoutingFilter(ctypes.Structure):
    """routing_filter (src/routing_filter.h:66-72), ONDISK = packed: 28 bytes."""
    _pack_ = 1
    _fields_ = [("addr", ctypes.c_uint64), ("meta_head", ctypes.c_uint64),
                ("num_fingerprints", ctypes.c_uint32), ("num_unique", ctypes.c_uint32),
                ("value_size", ctypes.c_uint32)]


assert ctypes.sizeof(RoutingFilter) == 28

_libs = {}


def available(path=LIB_PATH):
    return os.path.exists(path)


def lib(path=LIB_PATH):
    if path not in _libs:
        L = ctypes.CDLL(path)
        vp, u16, u32, u64, i32 = ctypes.c_void_p, ctypes.c_uint16, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int
        RF = ctypes.POINTER(RoutingFilter)
        L.rfr_create.restype = vp
        L.rfr_create.argtypes = [u32, u32, u64, u64]
        L.rfr_destroy.argtypes = [vp]
        L.rfr_destroy.restype = None
        L.rfr_device_io_count.restype = u64
        L.rfr_device_io_count.argtypes = [vp, i32]
        L.rfr_max_fingerprints.restype = u64
        L.rfr_max_fingerprints.argtypes = [vp]
        L.rfr_filter_add.restype = i32
        L.rfr_filter_add.argtypes = [vp, RF, RF, vp, u64, u16]
        L.rfr_filter_image.restype = u32
        L.rfr_filter_image.argtypes = [vp, RF, vp, u32, vp, ctypes.POINTER(u32)]
        L.rfr_lookup_keys.argtypes = [vp, RF, vp, u32, u64, vp]
        L.rfr_lookup_keys.restype = None
        L.rfr_lookup_keys_async.argtypes = [vp, RF, vp, u32, u64, vp]
        L.rfr_lookup_keys_async.restype = u64
        L.rfr_estimate_unique_fp.restype = i32
        L.rfr_estimate_unique_fp.argtypes = [vp, vp, u64, ctypes.POINTER(u32)]
        L.rfr_estimate_unique_keys_from_count.restype = u32
        L.rfr_estimate_unique_keys_from_count.argtypes = [vp, u64]
        L.rfr_estimate_unique_keys.restype = u32
        L.rfr_estimate_unique_keys.argtypes = [vp, RF]
        L.rfr_space_use_bytes.restype = u64
        L.rfr_space_use_bytes.argtypes = [vp, RF]
        L.rfr_dec_ref.argtypes = [vp, RF]
        L.rfr_dec_ref.restype = None
        L.rfr_get_next_value.restype = u16
        L.rfr_get_next_value.argtypes = [u64, u16]
        L.rfr_is_value_found.restype = i32
        L.rfr_is_value_found.argtypes = [u64, u16]
        L.rfr_hash_keys.argtypes = [vp, vp, u32, u64, vp]
        L.rfr_hash_keys.restype = None
        L.rfr_lookup_var_keys.argtypes = [vp, RF, vp, vp, u64, vp]
        L.rfr_lookup_var_keys.restype = None
        L.rfr_hash_var_keys.argtypes = [vp, vp, vp, u64, vp]
        L.rfr_hash_var_keys.restype = None
        L.rfr_bench_build.argtypes = [vp, vp, vp, u32, i32, vp, vp, u32, u16, i32, RF]
        L.rfr_bench_build.restype = ctypes.c_double
        L.rfr_bench_chain.argtypes = [vp, u32, u32, u32, i32, RF]
        L.rfr_bench_chain.restype = ctypes.c_double
        L.rfr_bench_probe.restype = ctypes.c_double
        L.rfr_bench_probe.argtypes = [vp, RF, vp, vp, u32, vp, u64, i32, vp]
        L.rfr_lookup_keys_async_many.restype = u64
        L.rfr_lookup_keys_async_many.argtypes = [vp, vp, vp, vp, u32, u64, vp, ctypes.POINTER(u64)]
        L.rfr_async_stats.restype = i32
        L.rfr_lookup_batch.restype = i32
        L.rfr_lookup_batch.argtypes = [vp, vp, vp, vp, u32, u64, vp]
        L.rfr_async_stats.argtypes = [ctypes.POINTER(u64), ctypes.POINTER(u64)]
        L.rfr_print.argtypes = [vp, RF]
        L.rfr_print.restype = None
        L.rfr_read_page.argtypes = [vp, u64, vp]
        L.rfr_read_page.restype = None
        L.rfr_lookup_keys_async_driven.argtypes = [vp, vp, vp, vp, u32, u64, vp, u32, vp, ctypes.c_double]
        L.rfr_lookup_keys_async_driven.restype = i32
        L.rfr_mt_chains.argtypes = [vp, vp, u32, u32, u32, u64, vp, u64, vp, vp, vp, vp]
        L.rfr_mt_chains.restype = i32
        L.rfr_async_many_phases.argtypes = [vp]
        L.rfr_async_many_phases.restype = None
        L.rfr_shim_stats.argtypes = [vp]
        L.rfr_shim_stats.restype = i32
        L.rfr_registry_set_limit.argtypes = [u64]
        L.rfr_registry_set_limit.restype = i32
        L.rfr_lookup_keys_async_flush.argtypes = [vp, vp, vp, vp, u32, u64, vp]
        L.rfr_lookup_keys_async_flush.restype = u64
        L.rfr_lookup_keys_async_flush_multi.argtypes = [vp, vp, vp, vp, vp, u32, u64, vp]
        L.rfr_lookup_keys_async_flush_multi.restype = u64
        L.rfr_add_breakdown.argtypes = [vp]
        L.rfr_add_breakdown.restype = ctypes.c_int
        L.rfr_async_breakdown.argtypes = [vp]
        L.rfr_async_breakdown.restype = ctypes.c_int
        if hasattr(L, "rfr_filter_test_basic"):  # the filter_test libraries only
            L.rfr_filter_test_basic.argtypes = [vp, u64, u64, u64, ctypes.c_char_p]
            L.rfr_filter_test_basic.restype = i32
            L.rfr_filter_test_perf.argtypes = [vp, u64, u64, u64, u64, ctypes.c_char_p]
            L.rfr_filter_test_perf.restype = i32
        _libs[path] = L
    return _libs[path]


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


class Image:
    """A reference-built filter read back as a relocatable image (this repo's form)."""

    def __init__(self, desc, pages, slots):
        self.desc = desc
        self.num_fingerprints = desc.num_fingerprints
        self.num_unique = desc.num_unique
        self.value_size = desc.value_size
        self.pages = pages
        self.slots = slots
        self.num_pages = pages.size // 4096
        self.num_indices = slots.size


class Stack:
    """One reference filter stack (heap, in-memory device, rc_allocator, clockcache,
    routing_config with seed 42 and the default data_config)."""

    def __init__(self, fingerprint_size=26, log_index_size=8, cache_mib=2048, disk_mib=16384, path=LIB_PATH):
        """path: LIB_PATH (the reference's routing_filter.c) or SHIM_PATH (the drop-in)"""
        self.lis = log_index_size
        self.fps = fingerprint_size
        self.L = lib(path)
        self.h = self.L.rfr_create(fingerprint_size, log_index_size, cache_mib, disk_mib)
        if not self.h:
            raise RuntimeError("rfr_create failed")

    def close(self):
        if self.h:
            self.L.rfr_destroy(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def device_writes(self):
        """pages the cache wrote to the device: 0 while every page stays cached, so every
        filter page is a fresh cache page (unwritten bytes zero, SURVEY finding 4)"""
        return int(self.L.rfr_device_io_count(self.h, 1))

    def device_reads(self):
        return int(self.L.rfr_device_io_count(self.h, 0))

    def max_fingerprints(self):
        return int(self.L.rfr_max_fingerprints(self.h))

    def add(self, hashes, value=0, old=None):
        """routing_filter_add over a COPY of hashes (the reference mutates its input)."""
        fps = np.array(hashes, dtype=np.uint32, copy=True)
        out = RoutingFilter()
        rc = self.L.rfr_filter_add(self.h, ctypes.byref(old) if old is not None else None,
                                  ctypes.byref(out), _p(fps) if fps.size else None, fps.size, value)
        if rc:
            raise RuntimeError(f"routing_filter_add: platform_status {rc}")
        return out

    def image(self, desc):
        if desc.addr == 0:
            return None
        lnb = max(int(desc.num_fingerprints).bit_length() - 1, self.lis)
        ni = 1 << (lnb - self.lis)
        cap = ni  # at most one data page per index
        pages = np.zeros(cap * 4096, dtype=np.uint8)
        slots = np.zeros(ni, dtype=np.uint64)
        np_ = ctypes.c_uint32(0)
        got = self.L.rfr_filter_image(self.h, ctypes.byref(desc), _p(pages), cap, _p(slots), ctypes.byref(np_))
        if got != ni:
            raise RuntimeError("rfr_filter_image failed")
        return Image(desc, pages[: np_.value * 4096].copy(), slots)

    def lookup_keys(self, desc, keys, key_len=24, use_async=False):
        k = np.ascontiguousarray(keys, dtype=np.uint8).reshape(-1)
        n = k.size // key_len
        out = np.zeros(n, dtype=np.uint64)
        if use_async:
            self.L.rfr_lookup_keys_async(self.h, ctypes.byref(desc), _p(k), key_len, n, _p(out))
        else:
            self.L.rfr_lookup_keys(self.h, ctypes.byref(desc), _p(k), key_len, n, _p(out))
        return out

    def lookup_var_keys(self, desc, data, offs):
        d = np.ascontiguousarray(data, dtype=np.uint8)
        o = np.ascontiguousarray(offs, dtype=np.uint64)
        out = np.zeros(o.size - 1, dtype=np.uint64)
        self.L.rfr_lookup_var_keys(self.h, ctypes.byref(desc), _p(d), _p(o), o.size - 1, _p(out))
        return out

    def hash_var_keys(self, data, offs):
        d = np.ascontiguousarray(data, dtype=np.uint8)
        o = np.ascontiguousarray(offs, dtype=np.uint64)
        out = np.zeros(o.size - 1, dtype=np.uint32)
        self.L.rfr_hash_var_keys(self.h, _p(d), _p(o), o.size - 1, _p(out))
        return out

    def hash_keys(self, keys, key_len=24):
        k = np.ascontiguousarray(keys, dtype=np.uint8).reshape(-1)
        n = k.size // key_len
        out = np.zeros(n, dtype=np.uint32)
        self.L.rfr_hash_keys(self.h, _p(k), key_len, n, _p(out))
        return out

    def estimate_unique_fp(self, descs):
        arr = (RoutingFilter * max(1, len(descs)))()
        for i, d in enumerate(descs):
            arr[i] = d if d is not None else RoutingFilter()
        out = ctypes.c_uint32(0)
        rc = self.L.rfr_estimate_unique_fp(self.h, ctypes.addressof(arr), len(descs), ctypes.byref(out))
        if rc:
            raise RuntimeError(f"estimate_unique_fp: platform_status {rc}")
        return out.value

    def estimate_unique_keys_from_count(self, num_unique):
        return int(self.L.rfr_estimate_unique_keys_from_count(self.h, num_unique))

    def space_use_bytes(self, desc):
        return int(self.L.rfr_space_use_bytes(self.h, ctypes.byref(desc)))

    def lookup_keys_async_many(self, descs, keys, filter_id=None, key_len=24):
        """len(keys) lookups as concurrent routing_filter_lookup_async states (each started
        once, then all polled): (found, callbacks fired, states that first returned RUNNING)"""
        k = np.ascontiguousarray(keys, dtype=np.uint8).reshape(-1)
        n = k.size // key_len
        arr = (RoutingFilter * max(1, len(descs)))(*descs)
        fid = None if filter_id is None else np.ascontiguousarray(filter_id, dtype=np.uint32)
        out = np.zeros(n, dtype=np.uint64)
        running = ctypes.c_uint64(0)
        cb = self.L.rfr_lookup_keys_async_many(self.h, ctypes.addressof(arr), None if fid is None else _p(fid),
                                               _p(k), key_len, n, _p(out), ctypes.byref(running))
        return out, int(cb), int(running.value)

    def lookup_batch(self, descs, keys, filter_id, key_len=24):
        """len(keys) lookups (descs[filter_id[i]], key i): one routing_filter_amd_lookup_batch
        call in the shim's stack, one routing_filter_lookup per key in the reference's.
        Returns (found, batched)."""
        k = np.ascontiguousarray(keys, dtype=np.uint8).reshape(-1)
        n = k.size // key_len
        arr = (RoutingFilter * max(1, len(descs)))(*descs)
        fid = np.ascontiguousarray(filter_id, dtype=np.uint32)
        out = np.zeros(n, dtype=np.uint64)
        r = self.L.rfr_lookup_batch(self.h, ctypes.addressof(arr), _p(fid), _p(k), key_len, n, _p(out))
        if r < 0:
            raise RuntimeError("routing_filter_amd_lookup_batch failed")
        return out, bool(r)

    def async_stats(self):
        b, p = ctypes.c_uint64(0), ctypes.c_uint64(0)
        self.L.rfr_async_stats(ctypes.byref(b), ctypes.byref(p))
        return int(b.value), int(p.value)

    def print_text(self, desc):
        """routing_filter_print's output (C stdout captured through a temporary file)"""
        import sys
        import tempfile
        sys.stdout.flush()
        fd = os.dup(1)
        with tempfile.TemporaryFile() as tmp:
            os.dup2(tmp.fileno(), 1)
            try:
                self.L.rfr_print(self.h, ctypes.byref(desc))
            finally:
                os.dup2(fd, 1)
                os.close(fd)
            tmp.seek(0)
            return tmp.read().decode()

    def read_page(self, addr):
        out = np.zeros(4096, dtype=np.uint8)
        self.L.rfr_read_page(self.h, addr, _p(out))
        return out

    def bench_build(self, data, key_len, starts, counts, threads, hash_keys=True, offs=None, value=0):
        """routing_filter_add of len(counts) filters (filter f = keys starts[f] ..
        starts[f] + counts[f] - 1) on `threads` registered threads, one filter per task as the
        trunk's TASK_TYPE_NORMAL workers run them. data = keys (hash_keys=True: each filter's
        keys are hashed first, trunk semantics) or u32 hashes (hash_keys=False, filter_test
        semantics). Returns (seconds, descriptors)."""
        d = np.ascontiguousarray(data)
        st = np.ascontiguousarray(starts, dtype=np.uint64)
        ct = np.ascontiguousarray(counts, dtype=np.uint32)
        keep = (RoutingFilter * max(1, ct.size))()
        o = None if offs is None else np.ascontiguousarray(offs, dtype=np.uint64)
        t = self.L.rfr_bench_build(self.h, _p(d), None if o is None else _p(o), key_len, 1 if hash_keys else 0,
                                   _p(st), _p(ct), ct.size, value, threads, keep)
        if t < 0:
            raise RuntimeError("routing_filter_add failed in the bench")
        return t, keep

    def bench_probe(self, keep, data, key_len, filter_id, threads, offs=None):
        """routing_filter_lookup of every key (key i in filter filter_id[i]) on `threads`
        threads. Returns (seconds, found_values)."""
        d = np.ascontiguousarray(data)
        fid = np.ascontiguousarray(filter_id, dtype=np.uint32)
        o = None if offs is None else np.ascontiguousarray(offs, dtype=np.uint64)
        found = np.zeros(fid.size, dtype=np.uint64)
        t = self.L.rfr_bench_probe(self.h, keep, _p(d), None if o is None else _p(o), key_len, _p(fid), fid.size,
                                   threads, _p(found))
        return t, found

    def bench_chain(self, num_filters, rounds, n, threads):
        """num_filters compaction chains on `threads` threads: round v of filter f hashes n
        24 B keys of ids (f << 32) + (v + 1) * j and routing_filter_adds them (value v) to
        the filter of round v-1, dropping the superseded one (oracle/ref_harness.c
        chain_worker). Returns (seconds, each chain's last filter)."""
        keep = (RoutingFilter * max(1, num_filters))()
        t = self.L.rfr_bench_chain(self.h, num_filters, rounds, n, threads, keep)
        if t < 0:
            raise RuntimeError("routing_filter_add failed in the chain bench")
        return t, keep

    def dec_ref(self, desc):
        self.L.rfr_dec_ref(self.h, ctypes.byref(desc))

    def lookup_keys_async_driven(self, descs, keys, filter_id=None, key_len=24, max_inflight=64, timeout_s=30.0):
        """len(keys) routing_filter_lookup_async lookups driven by callbacks as
        tests/functional/test_async.c drives them (a state is called again only after its
        callback fired; oracle/ref_harness.c rfr_lookup_keys_async_driven). Returns (found,
        stats) with stats = {running, callbacks, done, violations}; raises on a stall."""
        k = np.ascontiguousarray(keys, dtype=np.uint8).reshape(-1)
        n = k.size // key_len
        arr = (RoutingFilter * max(1, len(descs)))(*descs)
        fid = None if filter_id is None else np.ascontiguousarray(filter_id, dtype=np.uint32)
        out = np.zeros(n, dtype=np.uint64)
        st = np.zeros(4, dtype=np.uint64)
        r = self.L.rfr_lookup_keys_async_driven(self.h, ctypes.addressof(arr), None if fid is None else _p(fid),
                                                _p(k), key_len, n, _p(out), max_inflight, _p(st), timeout_s)
        stats = dict(zip(("running", "callbacks", "done", "violations"), (int(x) for x in st)))
        if r:
            raise RuntimeError(f"async lookups stalled: {stats}")
        return out, stats

    def lookup_keys_async_flush(self, descs, keys, filter_id=None, key_len=24):
        """every state started once, then one routing_filter_amd_flush(); returns (found,
        callbacks) -- callbacks None if a state was not done after the flush"""
        k = np.ascontiguousarray(keys, dtype=np.uint8).reshape(-1)
        n = k.size // key_len
        arr = (RoutingFilter * max(1, len(descs)))(*descs)
        fid = None if filter_id is None else np.ascontiguousarray(filter_id, dtype=np.uint32)
        out = np.zeros(n, dtype=np.uint64)
        cb = self.L.rfr_lookup_keys_async_flush(self.h, ctypes.addressof(arr), None if fid is None else _p(fid),
                                                _p(k), key_len, n, _p(out))
        return out, (None if cb == (1 << 64) - 1 else int(cb))

    def lookup_keys_async_flush_multi(self, stacks, descs, filter_stack, keys, filter_id, key_len=24):
        """async states over filters of several stacks of this library (descs[f] belongs to
        stacks[filter_stack[f]]), all queued, then ONE routing_filter_amd_flush()"""
        k = np.ascontiguousarray(keys, dtype=np.uint8).reshape(-1)
        n = k.size // key_len
        arr = (RoutingFilter * max(1, len(descs)))(*descs)
        hs = (ctypes.c_void_p * len(stacks))(*[st.h for st in stacks])
        fs = np.ascontiguousarray(filter_stack, dtype=np.uint32)
        fid = np.ascontiguousarray(filter_id, dtype=np.uint32)
        out = np.zeros(n, dtype=np.uint64)
        cb = self.L.rfr_lookup_keys_async_flush_multi(ctypes.addressof(hs), ctypes.addressof(arr), _p(fs), _p(fid),
                                                      _p(k), key_len, n, _p(out))
        return out, (None if cb == (1 << 64) - 1 else int(cb))

    def mt_chains(self, keys, threads, rounds, n, probe, nprobe, key_len=24):
        """threads x rounds incremental chains built by `threads` concurrent threads
        (oracle/ref_harness.c rfr_mt_chains), then each thread's nprobe lookups of its probe
        keys, synchronous and async. Returns (filters [threads][rounds], found_sync,
        found_async, per-thread add seconds)."""
        k = np.ascontiguousarray(keys, dtype=np.uint8).reshape(-1)
        p = np.ascontiguousarray(probe, dtype=np.uint8).reshape(-1)
        out = (RoutingFilter * (threads * rounds))()
        fs = np.zeros(threads * nprobe, dtype=np.uint64)
        fa = np.zeros(threads * nprobe, dtype=np.uint64)
        add_s = np.zeros(threads, dtype=np.float64)
        rc = self.L.rfr_mt_chains(self.h, _p(k), key_len, threads, rounds, n, _p(p), nprobe, out, _p(fs), _p(fa),
                                  _p(add_s))
        if rc:
            raise RuntimeError(f"concurrent routing_filter_add: platform_status {rc}")
        return [[out[t * rounds + r] for r in range(rounds)] for t in range(threads)], fs, fa, add_s

    def shim_stats(self):
        """the shim's add batches / filters, registry bytes / evictions / trims (None for
        the reference's library)"""
        out = np.zeros(6, dtype=np.uint64)
        if not self.L.rfr_shim_stats(_p(out)):
            return None
        return dict(zip(("add_batches", "add_filters", "registry_bytes", "evictions", "trims", "async_probe_ns"),
                        (int(x) for x in out)))

    def add_breakdown(self):
        """the shim's routing_filter_add so far: calls, combiner batches, ns per phase (None
        for the reference's library)"""
        out = np.zeros(11, dtype=np.uint64)  # routing_filter_amd_add_breakdown writes 11 words
        if not self.L.rfr_add_breakdown(_p(out)):
            return None
        keys = ("calls", "batches", "create_ns", "stage_ns", "build_ns", "infos_ns", "readback_ns", "wait_ns",
                "place_ns", "engine_create_ns", "register_ns")
        return dict(zip(keys, (int(x) for x in out)))

    def async_breakdown(self):
        """the shim's async path so far: reaps that completed states, states, ns submitting
        (hash, pin, ring) / reaping / in callbacks, and the engine's launch-based lookup round
        trips (calls, prep / launch / wait ns); None for the reference's library"""
        out = np.zeros(10, dtype=np.uint64)
        if not self.L.rfr_async_breakdown(_p(out)):
            return None
        keys = ("batches", "states", "submit_ns", "unused_ns", "reap_ns", "callback_ns",
                "rt_calls", "rt_prep_ns", "rt_launch_ns", "rt_wait_ns")
        return dict(zip(keys, (int(x) for x in out)))

    def async_many_phases(self):
        """(start, poll) nanoseconds of the last lookup_keys_async_many call"""
        out = np.zeros(2, dtype=np.uint64)
        self.L.rfr_async_many_phases(_p(out))
        return int(out[0]), int(out[1])

    def registry_set_limit(self, mib):
        return bool(self.L.rfr_registry_set_limit(mib))

    def filter_test_basic(self, num_fingerprints, num_values, key_size=24):
        """the reference's test_filter_basic (tests/functional/filter_test.c:22-148) on this
        stack; returns (platform_status, its log text)"""
        return self._filter_test(lambda path: self.L.rfr_filter_test_basic(
            self.h, key_size, num_fingerprints, num_values, path))

    def filter_test_perf(self, num_fingerprints, num_values, num_trees, key_size=24):
        """the reference's test_filter_perf (filter_test.c:150-273); (status, log text)"""
        return self._filter_test(lambda path: self.L.rfr_filter_test_perf(
            self.h, key_size, num_fingerprints, num_values, num_trees, path))

    def _filter_test(self, run):
        import tempfile
        with tempfile.NamedTemporaryFile(suffix=".log") as tmp:
            rc = run(tmp.name.encode())
            with open(tmp.name) as f:
                return int(rc), f.read()


def get_next_value(found_values, last_value):
    return int(lib().rfr_get_next_value(found_values, last_value))


def is_value_found(found_values, value):
    return bool(lib().rfr_is_value_found(found_values, value))
