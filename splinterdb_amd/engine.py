"""Python host mirror of SplinterDB's routing_filter.h API over the MI355X engine's C ABI.

Names, argument meaning and errors follow the reference interface
(src/routing_filter.h:32-192): `routing_config_init`, `routing_filter_add`,
`routing_filter_lookup`, `routing_filter_get_next_value`, `routing_filter_is_value_found`,
`routing_filter_max_fingerprints`, `routing_filter_estimate_unique_keys_from_count`,
`routing_filter_space_use_bytes`. Errors raise `PlatformStatusError` carrying the
platform_status code (ENOMEM / EINVAL / ENODEV).

The compute runs only in librf_amd.so (hand-written HIP kernels for gfx950). There is
no CPU fallback: without the library or a HIP device every call raises.
"""
import ctypes
import os
from dataclasses import dataclass

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "librf_amd.so")

STATUS_OK = 0
STATUS_NO_MEMORY = 12
STATUS_NO_DEVICE = 19
STATUS_BAD_PARAM = 22
MAX_FILTERS = 32  # src/routing_filter.h:25
ROUTING_NOT_FOUND = 0xFFFF  # src/routing_filter.h:26

# symbols the C ABI (include/rf_amd.h) exports
EXPORTED = [
    "rf_amd_engine_create", "rf_amd_engine_destroy", "rf_amd_last_error",
    "rf_amd_batch_create", "rf_amd_batch_destroy", "rf_amd_batch_build_keys",
    "rf_amd_batch_build_var_keys", "rf_amd_batch_build_hashes", "rf_amd_batch_probe_keys",
    "rf_amd_batch_probe_var_keys", "rf_amd_batch_probe_hashes", "rf_amd_batch_info",
    "rf_amd_batch_probe_keys_runs", "rf_amd_batch_probe_hashes_runs",
    "rf_amd_batch_read_image", "rf_amd_batch_read_image_async", "rf_amd_batch_image_ptrs", "rf_amd_batch_num_filters",
    "rf_amd_batch_set_timing", "rf_amd_batch_timings", "rf_amd_batch_timings_back", 
    "rf_amd_debug_read_lines", "rf_amd_debug_rebuild_lines", "rf_amd_debug_phase_buffer", "rf_amd_diag_lookup_stats",
    "rf_amd_debug_probe_floor",
    "rf_amd_host_alloc", "rf_amd_host_free", "rf_amd_engine_fence", "rf_amd_engine_fence_wait",
    "rf_amd_host_register", "rf_amd_host_unregister", "rf_amd_batch_place_image", "rf_amd_engine_set_pool_limit",
    "rf_amd_lookup_submit", "rf_amd_lookup_wait", "rf_amd_lookup_reap", "rf_amd_lookup_server_stats",
    "rf_amd_build_id",
    "rf_amd_filter_add", "rf_amd_filter_lookup_hashes", "rf_amd_filter_lookup_keys",
    "rf_amd_image_free",
    "rf_amd_max_fingerprints", "rf_amd_estimate_unique_keys_from_count",
    "rf_amd_space_use_bytes",
    "rf_amd_estimate_unique_fp", "rf_amd_batch_estimate_unique_fp", "rf_amd_estimate_unique_keys",
    "rf_amd_lookup_async", "rf_amd_lookup_async_poll", "rf_amd_lookup_async_wait",
    "rf_amd_lookup_async_free", "rf_amd_filter_verify", "rf_amd_filter_print",
    "rf_amd_hash_keys", "rf_amd_hash_var_keys",
    "rf_amd_batch_export", "rf_amd_batch_import", "rf_amd_route_scratch_bytes", "rf_amd_route_probes", "rf_amd_batch_probe_pairs", "rf_amd_unroute_found",
    "rf_amd_batch_build_hashes_host", "rf_amd_batch_probe_hashes_host", "rf_amd_engine_pool_stats",
    "rf_amd_filter_print_abs", "rf_amd_batch_infos", "rf_amd_batch_destroy_on", "rf_amd_probe_many_hashes_host",
    "rf_amd_probe_filters_host", "rf_amd_engine_pool_trim", "rf_amd_engine_stream", "rf_amd_engine_sync",
    "rf_amd_batch_device_bytes", "rf_amd_batch_trim", "rf_amd_batch_stage_begin", "rf_amd_batch_stage_build",
    "rf_amd_batch_stage_abort", "rf_amd_lookup_server_error", "rf_amd_lookup_server_failed",
    "rf_amd_lookup_server_set_times", "rf_amd_diag_lookup_server_kill", "rf_amd_diag_lookup_ring",
]
ROUTE_MAX_WORLD = 16
ASYNC_STATUS_RUNNING = 0  # src/platform_linux/async.h:137-140
ASYNC_STATUS_DONE = 1
CALLBACK_FN = ctypes.CFUNCTYPE(None, ctypes.c_void_p)


class PlatformStatusError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"platform_status {code}: {msg}")
        self.code = code


class RfConfig(ctypes.Structure):
    _fields_ = [("fingerprint_size", ctypes.c_uint32), ("log_index_size", ctypes.c_uint32),
                ("seed", ctypes.c_uint32), ("page_size", ctypes.c_uint32),
                ("pages_per_extent", ctypes.c_uint32)]


class RfFilterInfo(ctypes.Structure):
    _fields_ = [("num_fingerprints", ctypes.c_uint32), ("num_unique", ctypes.c_uint32),
                ("value_size", ctypes.c_uint32), ("num_indices", ctypes.c_uint32),
                ("num_pages", ctypes.c_uint32), ("error", ctypes.c_uint32)]


class RfImage(ctypes.Structure):
    _fields_ = [("info", RfFilterInfo), ("pages", ctypes.POINTER(ctypes.c_uint8)),
                ("slots", ctypes.POINTER(ctypes.c_uint64))]


_lib = None


def check_build_id(L, path):
    """a library built from other sources than the tree's (a stale prebuilt .so, e.g. the
    diagnostics build left behind by an earlier round) fails loudly instead of running"""
    from . import build as _b
    L.rf_amd_build_id.restype = ctypes.c_char_p
    got = L.rf_amd_build_id().decode()
    try:
        want = _b.source_id()
    except OSError:  # sources absent: nothing to compare with
        return
    if got != want:
        raise RuntimeError(f"{path} was built from other sources (build id {got}, tree {want}): "
                           "rebuild it (python -c 'import __graft_entry__ as g; g.build()')")


def load_library(build_if_missing=True):
    """Load librf_amd.so (building it in-tree with hipcc if absent)."""
    global _lib
    if _lib is not None:
        return _lib
    path = os.environ.get("RF_AMD_LIB", LIB_PATH)  # e.g. the phase-stamp diagnostics build
    if not os.path.exists(path):
        if not build_if_missing or path != LIB_PATH:
            raise PlatformStatusError(STATUS_NO_DEVICE, f"{path} missing (run build)")
        from . import build as _b
        _b.build()
    L = ctypes.CDLL(path)
    check_build_id(L, path)
    vp, u32, u64, i32 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int
    L.rf_amd_last_error.restype = ctypes.c_char_p
    L.rf_amd_engine_create.argtypes = [i32, ctypes.POINTER(vp)]
    L.rf_amd_engine_destroy.argtypes = [vp]
    L.rf_amd_engine_destroy.restype = None
    L.rf_amd_batch_create.argtypes = [vp, ctypes.POINTER(RfConfig), u32, vp, vp, vp, vp,
                                      ctypes.POINTER(vp)]
    L.rf_amd_batch_destroy.argtypes = [vp]
    L.rf_amd_batch_destroy.restype = None
    L.rf_amd_batch_build_keys.argtypes = [vp, vp, u32, vp]
    L.rf_amd_batch_build_var_keys.argtypes = [vp, vp, vp, vp]
    L.rf_amd_batch_build_hashes.argtypes = [vp, vp, vp]
    L.rf_amd_batch_probe_keys.argtypes = [vp, vp, u32, vp, u64, vp, vp]
    L.rf_amd_batch_probe_var_keys.argtypes = [vp, vp, vp, vp, u64, vp, vp]
    L.rf_amd_batch_probe_hashes.argtypes = [vp, vp, vp, u64, vp, vp]
    L.rf_amd_batch_probe_keys_runs.argtypes = [vp, vp, u32, ctypes.POINTER(u64), vp, vp]
    L.rf_amd_batch_probe_hashes_runs.argtypes = [vp, vp, ctypes.POINTER(u64), vp, vp]
    L.rf_amd_batch_info.argtypes = [vp, u32, ctypes.POINTER(RfFilterInfo)]
    L.rf_amd_batch_read_image.argtypes = [vp, u32, vp, u64, vp, u32]
    L.rf_amd_batch_read_image_async.argtypes = [vp, u32, vp, u64, vp, u32, vp]
    L.rf_amd_batch_image_ptrs.argtypes = [vp, u32, ctypes.POINTER(vp), ctypes.POINTER(vp)]
    L.rf_amd_batch_set_timing.argtypes = [vp, i32]
    L.rf_amd_batch_timings.argtypes = [vp, ctypes.POINTER(ctypes.c_float), u32]
    L.rf_amd_batch_timings_back.argtypes = [vp, u32, ctypes.POINTER(ctypes.c_float), u32]
    L.rf_amd_debug_read_lines.argtypes = [vp, vp, u64, ctypes.POINTER(u64)]
    L.rf_amd_debug_rebuild_lines.argtypes = [vp]
    L.rf_amd_debug_phase_buffer.argtypes = [vp, u32]
    L.rf_amd_debug_probe_floor.argtypes = [vp, vp, u32, vp, vp, vp]
    L.rf_amd_diag_lookup_stats.argtypes = [vp, ctypes.c_int]
    L.rf_amd_lookup_submit.argtypes = [vp, vp, u32, u32, vp, ctypes.POINTER(u64)]
    L.rf_amd_lookup_wait.argtypes = [vp, u64, ctypes.POINTER(u64)]
    L.rf_amd_lookup_reap.argtypes = [vp, vp, vp, u64]
    L.rf_amd_lookup_reap.restype = u64
    L.rf_amd_lookup_server_stats.argtypes = [vp, vp]
    L.rf_amd_lookup_server_error.argtypes = [vp]
    L.rf_amd_lookup_server_failed.argtypes = [vp, vp, u64]
    L.rf_amd_lookup_server_failed.restype = u64
    L.rf_amd_lookup_server_set_times.argtypes = [vp, u64, u64]
    L.rf_amd_diag_lookup_server_kill.argtypes = [vp, i32, u32]
    L.rf_amd_diag_lookup_ring.argtypes = [vp]
    L.rf_amd_batch_num_filters.argtypes = [vp]
    L.rf_amd_batch_num_filters.restype = u32
    L.rf_amd_filter_add.argtypes = [vp, ctypes.POINTER(RfConfig), ctypes.POINTER(RfImage),
                                    ctypes.POINTER(RfImage), vp, u64, ctypes.c_uint16]
    L.rf_amd_filter_lookup_hashes.argtypes = [vp, ctypes.POINTER(RfConfig),
                                              ctypes.POINTER(RfImage), vp, u64, vp]
    L.rf_amd_filter_lookup_keys.argtypes = [vp, ctypes.POINTER(RfConfig), ctypes.POINTER(RfImage),
                                            vp, u32, u64, vp]
    L.rf_amd_image_free.argtypes = [ctypes.POINTER(RfImage)]
    L.rf_amd_image_free.restype = None
    L.rf_amd_max_fingerprints.argtypes = [ctypes.POINTER(RfConfig)]
    L.rf_amd_max_fingerprints.restype = u64
    L.rf_amd_estimate_unique_keys_from_count.argtypes = [ctypes.POINTER(RfConfig), u64]
    L.rf_amd_estimate_unique_keys_from_count.restype = u32
    L.rf_amd_space_use_bytes.argtypes = [ctypes.POINTER(RfConfig), u32]
    L.rf_amd_space_use_bytes.restype = u64
    L.rf_amd_estimate_unique_fp.argtypes = [vp, ctypes.POINTER(RfConfig), vp, u64,
                                            ctypes.POINTER(u32)]
    L.rf_amd_batch_estimate_unique_fp.argtypes = [vp, vp, u64, ctypes.POINTER(u32)]
    L.rf_amd_estimate_unique_keys.argtypes = [ctypes.POINTER(RfFilterInfo), ctypes.POINTER(RfConfig)]
    L.rf_amd_estimate_unique_keys.restype = u32
    L.rf_amd_lookup_async.argtypes = [vp, vp, u32, vp, u64, vp, CALLBACK_FN, vp, vp,
                                      ctypes.POINTER(vp)]
    L.rf_amd_lookup_async_poll.argtypes = [vp]
    L.rf_amd_lookup_async_wait.argtypes = [vp]
    L.rf_amd_lookup_async_free.argtypes = [vp]
    L.rf_amd_lookup_async_free.restype = None
    L.rf_amd_filter_verify.argtypes = [vp, ctypes.POINTER(RfConfig), ctypes.POINTER(RfImage), vp, u32,
                                       u64, ctypes.c_uint16, ctypes.POINTER(u64)]
    L.rf_amd_filter_print.argtypes = [ctypes.POINTER(RfConfig), ctypes.POINTER(RfImage), vp]
    L.rf_amd_hash_keys.argtypes = [vp, ctypes.POINTER(RfConfig), vp, u32, u64, vp, vp]
    L.rf_amd_hash_var_keys.argtypes = [vp, ctypes.POINTER(RfConfig), vp, vp, u64, vp, vp]
    L.rf_amd_batch_export.argtypes = [vp, vp, u64, vp, u64, vp]
    L.rf_amd_batch_import.argtypes = [vp, ctypes.POINTER(RfConfig), u32, ctypes.POINTER(RfFilterInfo), vp, vp,
                                      i32, ctypes.POINTER(vp)]
    L.rf_amd_route_scratch_bytes.argtypes = [u64, u32]
    L.rf_amd_route_scratch_bytes.restype = u64
    L.rf_amd_route_probes.argtypes = [vp, vp, vp, u64, vp, u32, u32, vp, vp, vp, ctypes.POINTER(u64), vp]
    L.rf_amd_batch_probe_pairs.argtypes = [vp, vp, u64, vp, vp]
    L.rf_amd_unroute_found.argtypes = [vp, vp, vp, u64, vp, vp]
    L.rf_amd_batch_build_hashes_host.argtypes = [vp, vp]
    L.rf_amd_batch_probe_hashes_host.argtypes = [vp, vp, vp, u64, vp]
    L.rf_amd_engine_pool_stats.argtypes = [vp, ctypes.POINTER(u64), ctypes.POINTER(u64), ctypes.POINTER(u64)]
    L.rf_amd_filter_print_abs.argtypes = [ctypes.POINTER(RfConfig), ctypes.POINTER(RfImage), u64, vp, vp]
    L.rf_amd_batch_infos.argtypes = [vp, ctypes.POINTER(RfFilterInfo), vp]
    L.rf_amd_batch_destroy_on.argtypes = [vp, vp]
    L.rf_amd_probe_many_hashes_host.argtypes = [vp, vp, vp, vp, u32, vp, vp]
    L.rf_amd_probe_filters_host.argtypes = [vp, vp, vp, u32, vp, vp, u64, vp]
    L.rf_amd_engine_pool_trim.argtypes = [vp, u64]
    L.rf_amd_engine_stream.argtypes = [vp]
    L.rf_amd_engine_stream.restype = vp
    L.rf_amd_engine_sync.argtypes = [vp]
    L.rf_amd_batch_device_bytes.argtypes = [vp]
    L.rf_amd_batch_device_bytes.restype = u64
    L.rf_amd_batch_trim.argtypes = [vp, vp]
    L.rf_amd_batch_stage_begin.argtypes = [vp, ctypes.POINTER(vp)]
    L.rf_amd_batch_stage_build.argtypes = [vp]
    L.rf_amd_batch_stage_abort.argtypes = [vp]
    L.rf_amd_batch_stage_abort.restype = None
    _lib = L
    return L


def _check(rc):
    if rc != 0:
        raise PlatformStatusError(rc, load_library().rf_amd_last_error().decode())


# ---- routing_config (src/routing_filter.h:32-58) --------------------------------------
@dataclass
class RoutingConfig:
    fingerprint_size: int = 26
    log_index_size: int = 8
    seed: int = 42
    page_size: int = 4096
    pages_per_extent: int = 32

    @property
    def index_size(self):
        return 1 << self.log_index_size

    def c(self):
        return RfConfig(self.fingerprint_size, self.log_index_size, self.seed, self.page_size,
                        self.pages_per_extent)


def routing_config_init(fingerprint_size=26, log_index_size=8, seed=42, page_size=4096,
                        pages_per_extent=32):
    """routing_config_init (src/routing_filter.h:42-58); the key_hash argument of the
    reference is ignored there too -- hashing is XXH32 with `seed`."""
    return RoutingConfig(fingerprint_size, log_index_size, seed, page_size, pages_per_extent)


class Engine:
    """One HIP device + stream. Raises PlatformStatusError(ENODEV) without a GPU."""

    def __init__(self, device=0):
        L = load_library()
        h = ctypes.c_void_p()
        _check(L.rf_amd_engine_create(device, ctypes.byref(h)))
        self.h = h
        self.device = device

    def pool_stats(self):
        """device-memory pool of the engine's batches: bytes held, hits, misses"""
        v = [ctypes.c_uint64() for _ in range(3)]
        _check(load_library().rf_amd_engine_pool_stats(self.h, *[ctypes.byref(x) for x in v]))
        return dict(zip(("pooled_bytes", "hits", "misses"), (x.value for x in v)))

    def close(self):
        if self.h:
            load_library().rf_amd_engine_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


_default_engine = None


def default_engine():
    global _default_engine
    if _default_engine is None:
        _default_engine = Engine(0)
    return _default_engine


# ---- routing_filter descriptor + image -----------------------------------------------
@dataclass
class RoutingFilter:
    """routing_filter (src/routing_filter.h:66-72) plus its relocatable page image:
    pages = num_pages * page_size bytes, slots[i] = data_page_no * page_size + offset."""
    num_fingerprints: int
    num_unique: int
    value_size: int
    num_indices: int
    num_pages: int
    pages: np.ndarray
    slots: np.ndarray

    def _c(self):
        img = RfImage()
        img.info = RfFilterInfo(self.num_fingerprints, self.num_unique, self.value_size,
                                self.num_indices, self.num_pages, 0)
        self._pages_c = np.ascontiguousarray(self.pages, dtype=np.uint8)
        self._slots_c = np.ascontiguousarray(self.slots, dtype=np.uint64)
        img.pages = self._pages_c.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))
        img.slots = self._slots_c.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))
        return img


NULL_ROUTING_FILTER = None


def routing_filter_add(cfg: RoutingConfig, old_filter, new_fp_arr, value=0, engine=None):
    """routing_filter_add (src/routing_filter.h:78-85): 32-bit key hashes in, new filter
    out. new_fp_arr is not modified (the reference shifts/sorts it in place)."""
    eng = engine or default_engine()
    L = load_library()
    fps = np.ascontiguousarray(new_fp_arr, dtype=np.uint32)
    out = RfImage()
    old_c = old_filter._c() if old_filter is not None else None
    _check(L.rf_amd_filter_add(eng.h, ctypes.byref(cfg.c()),
                               ctypes.byref(old_c) if old_c is not None else None,
                               ctypes.byref(out), fps.ctypes.data if fps.size else None,
                               fps.size, value))
    try:
        info = out.info
        npg = info.num_pages * cfg.page_size
        pages = np.ctypeslib.as_array(out.pages, shape=(npg,)).copy()
        slots = np.ctypeslib.as_array(out.slots, shape=(info.num_indices,)).copy()
    finally:
        L.rf_amd_image_free(ctypes.byref(out))
    return RoutingFilter(info.num_fingerprints, info.num_unique, info.value_size,
                         info.num_indices, info.num_pages, pages, slots)


def routing_filter_lookup_hashes(cfg: RoutingConfig, filt, hashes, engine=None):
    eng = engine or default_engine()
    L = load_library()
    h = np.ascontiguousarray(hashes, dtype=np.uint32)
    out = np.zeros(h.size, dtype=np.uint64)
    fc = filt._c() if filt is not None else None
    _check(L.rf_amd_filter_lookup_hashes(eng.h, ctypes.byref(cfg.c()),
                                         ctypes.byref(fc) if fc is not None else None,
                                         h.ctypes.data, h.size, out.ctypes.data))
    return out


def routing_filter_lookup_keys(cfg: RoutingConfig, filt, keys: np.ndarray, engine=None):
    """Fixed-length keys (n x key_len uint8) hashed and probed on the GPU."""
    eng = engine or default_engine()
    L = load_library()
    k = np.ascontiguousarray(keys, dtype=np.uint8)
    if k.ndim == 1:
        k = k.reshape(1, -1)
    out = np.zeros(k.shape[0], dtype=np.uint64)
    fc = filt._c() if filt is not None else None
    _check(L.rf_amd_filter_lookup_keys(eng.h, ctypes.byref(cfg.c()),
                                       ctypes.byref(fc) if fc is not None else None,
                                       k.ctypes.data, k.shape[1], k.shape[0], out.ctypes.data))
    return out


def routing_filter_lookup(cfg: RoutingConfig, filt, key: bytes, engine=None):
    """routing_filter_lookup (src/routing_filter.h:87-92) for one key; returns found_values."""
    arr = np.frombuffer(bytes(key), dtype=np.uint8)
    return int(routing_filter_lookup_keys(cfg, filt, arr, engine)[0])


def _c_int_shl1(v: int) -> int:
    """`1 << v` on a 32-bit C int as the reference's x86-64 build evaluates it, widened to
    uint64: the shift count is taken mod 32 (`shl %cl`), and 1 << 31 is INT_MIN, which
    sign-extends. (Values >= 31 are UB in C; this is the code gcc emits for them.)"""
    sh = v & 31
    return 0xFFFFFFFF80000000 if sh == 31 else 1 << sh


def routing_filter_get_next_value(found_values: int, last_value: int) -> int:
    """src/routing_filter.h:94-105: `uint64 mask = (1 << last_value) - 1` is int arithmetic
    (INT_MIN - 1 wraps to INT_MAX), so last_value >= 31 does not mask the way a 64-bit
    shift would."""
    if last_value != ROUTING_NOT_FOUND:
        m = _c_int_shl1(last_value)
        mask = 0x7FFFFFFF if m == 0xFFFFFFFF80000000 else m - 1
        found_values &= mask
    if found_values == 0:
        return ROUTING_NOT_FOUND
    return found_values.bit_length() - 1


def routing_filter_is_value_found(found_values: int, value: int) -> bool:
    """src/routing_filter.h:107-111: `found_values & (1 << value)` with an int shift."""
    return (found_values & _c_int_shl1(value)) != 0


def routing_filter_max_fingerprints(cfg: RoutingConfig) -> int:
    return load_library().rf_amd_max_fingerprints(ctypes.byref(cfg.c()))


def routing_filter_estimate_unique_keys_from_count(cfg: RoutingConfig, num_unique: int) -> int:
    return load_library().rf_amd_estimate_unique_keys_from_count(ctypes.byref(cfg.c()), num_unique)


def routing_filter_estimate_unique_keys(filt: RoutingFilter, cfg: RoutingConfig) -> int:
    """src/routing_filter.h:165-167, .c:1141-1146."""
    info = RfFilterInfo(filt.num_fingerprints, filt.num_unique, filt.value_size,
                        filt.num_indices, filt.num_pages, 0)
    return load_library().rf_amd_estimate_unique_keys(ctypes.byref(info), ctypes.byref(cfg.c()))


def routing_filter_estimate_unique_fp(cfg: RoutingConfig, filters, engine=None) -> int:
    """routing_filter_estimate_unique_fp (src/routing_filter.h:169-175, .c:702-848) over
    host images; None entries are NULL_ROUTING_FILTER. Returns num_unique_fp."""
    eng = engine or default_engine()
    arr = (RfImage * max(1, len(filters)))()
    keep = []
    for i, f in enumerate(filters):
        if f is None:
            arr[i] = RfImage()
        else:
            arr[i] = f._c()
            keep.append(f)
    out = ctypes.c_uint32(0)
    _check(load_library().rf_amd_estimate_unique_fp(eng.h, ctypes.byref(cfg.c()), ctypes.addressof(arr),
                                                    len(filters), ctypes.byref(out)))
    return out.value


def batch_estimate_unique_fp(members) -> int:
    """estimate_unique_fp over device-resident filters: members = [(FilterBatch, f) or None]."""
    n = len(members)
    hs = (ctypes.c_void_p * max(1, n))()
    idx = np.zeros(max(1, n), dtype=np.uint32)
    for i, m in enumerate(members):
        if m is not None:
            hs[i] = m[0].h.value
            idx[i] = m[1]
    out = ctypes.c_uint32(0)
    _check(load_library().rf_amd_batch_estimate_unique_fp(ctypes.addressof(hs), idx.ctypes.data, n,
                                                          ctypes.byref(out)))
    return out.value


def routing_filter_verify(cfg: RoutingConfig, filt, keys: np.ndarray, value: int, engine=None) -> int:
    """routing_filter_verify (src/routing_filter.c:1163-1183) over fixed-length keys: raises
    PlatformStatusError(EINVAL) if a key does not find `value` (the reference asserts)."""
    eng = engine or default_engine()
    k = np.ascontiguousarray(keys, dtype=np.uint8)
    if k.ndim == 1:
        k = k.reshape(1, -1)
    missing = ctypes.c_uint64(0)
    fc = filt._c() if filt is not None else None
    rc = load_library().rf_amd_filter_verify(eng.h, ctypes.byref(cfg.c()),
                                             ctypes.byref(fc) if fc is not None else None,
                                             k.ctypes.data, k.shape[1], k.shape[0], value,
                                             ctypes.byref(missing))
    if rc:
        err = PlatformStatusError(rc, load_library().rf_amd_last_error().decode())
        err.num_missing = missing.value
        raise err
    return 0


def routing_filter_print(cfg: RoutingConfig, filt, path=None) -> str:
    """routing_filter_print (src/routing_filter.c:1260-1286); returns the text."""
    import tempfile
    libc = ctypes.CDLL(None)
    libc.fopen.restype = ctypes.c_void_p
    libc.fopen.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
    libc.fclose.argtypes = [ctypes.c_void_p]
    fd, tmp = tempfile.mkstemp(suffix=".txt")
    os.close(fd)
    fh = libc.fopen((path or tmp).encode(), b"w")
    try:
        fc = filt._c()
        _check(load_library().rf_amd_filter_print(ctypes.byref(cfg.c()), ctypes.byref(fc), fh))
    finally:
        libc.fclose(fh)
    with open(path or tmp) as t:
        text = t.read()
    os.unlink(tmp)
    return text


def hash_keys(cfg: RoutingConfig, d_keys, key_len, n, d_hashes, stream=None, engine=None):
    """XXH32 of n device-resident fixed-length keys (data_key_hash) into d_hashes, on the GPU."""
    eng = engine or default_engine()
    _check(load_library().rf_amd_hash_keys(eng.h, ctypes.byref(cfg.c()), _dptr(d_keys), key_len, n,
                                           _dptr(d_hashes), _stream(stream)))


def hash_var_keys(cfg: RoutingConfig, d_bytes, d_offsets, n, d_hashes, stream=None, engine=None):
    eng = engine or default_engine()
    _check(load_library().rf_amd_hash_var_keys(eng.h, ctypes.byref(cfg.c()), _dptr(d_bytes), _dptr(d_offsets), n,
                                               _dptr(d_hashes), _stream(stream)))


def route_scratch_bytes(n, world):
    return int(load_library().rf_amd_route_scratch_bytes(n, world))


def route_probes(d_hashes, d_filter_id, n, d_route, num_filters, world, d_pairs, d_perm, d_scratch,
                 stream=None, engine=None):
    """Stable partition of n probes by owning rank (rf_amd_route_probes); returns the
    per-rank pair counts (list of `world` ints)."""
    eng = engine or default_engine()
    counts = (ctypes.c_uint64 * max(1, world))()
    _check(load_library().rf_amd_route_probes(eng.h, _dptr(d_hashes), _dptr(d_filter_id), n, _dptr(d_route),
                                              num_filters, world, _dptr(d_pairs), _dptr(d_perm),
                                              _dptr(d_scratch), counts, _stream(stream)))
    return [int(c) for c in counts[:world]]


def unroute_found(d_back, d_perm, n, d_found, stream=None, engine=None):
    eng = engine or default_engine()
    _check(load_library().rf_amd_unroute_found(eng.h, _dptr(d_back), _dptr(d_perm), n, _dptr(d_found),
                                               _stream(stream)))


class LookupAsync:
    """routing_filter_lookup_async (src/routing_filter.h:130-155) for a batch of host keys
    against a built FilterBatch: poll() returns ASYNC_STATUS_RUNNING / ASYNC_STATUS_DONE;
    callback() (optional, no arguments) runs once the results are in `found`."""

    def __init__(self, batch, keys: np.ndarray, filter_id=None, callback=None, stream=None):
        k = np.ascontiguousarray(keys, dtype=np.uint8)
        if k.ndim == 1:
            k = k.reshape(1, -1)
        self.found = np.zeros(k.shape[0], dtype=np.uint64)
        self._fid = None if filter_id is None else np.ascontiguousarray(filter_id, dtype=np.uint32)
        self._cb = CALLBACK_FN(lambda _arg: callback()) if callback else CALLBACK_FN()
        self.batch = batch
        self.h = ctypes.c_void_p()
        _check(load_library().rf_amd_lookup_async(
            batch.h, k.ctypes.data, k.shape[1], None if self._fid is None else self._fid.ctypes.data,
            k.shape[0], self.found.ctypes.data, self._cb, None, stream, ctypes.byref(self.h)))

    def poll(self) -> int:
        return load_library().rf_amd_lookup_async_poll(self.h)

    def wait(self) -> np.ndarray:
        _check(load_library().rf_amd_lookup_async_wait(self.h))
        return self.found

    def close(self):
        if self.h:
            load_library().rf_amd_lookup_async_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def routing_filter_space_use_bytes(cfg: RoutingConfig, filt: RoutingFilter) -> int:
    if filt is None:
        return 0
    return load_library().rf_amd_space_use_bytes(ctypes.byref(cfg.c()), filt.num_pages)


# ---- batched device-resident engine -----------------------------------------------------
def _stream(stream):
    """The caller's stream: explicit handle, else torch's current stream when torch has a
    live HIP context and uses a non-default stream, else None (the engine's blocking
    stream, which is ordered with the legacy null stream)."""
    if stream is not None:
        return stream
    import sys
    t = sys.modules.get("torch")
    if t is not None and t.cuda.is_initialized():
        h = t.cuda.current_stream().cuda_stream
        return h or None
    return None


def _hptr(x):
    """Address of a numpy array, torch tensor or int."""
    if isinstance(x, np.ndarray):
        return x.ctypes.data
    return _dptr(x)


def _dptr(x):
    """Device pointer of a torch tensor (or an int address)."""
    if x is None:
        return None
    if isinstance(x, int):
        return x
    return x.data_ptr()


class FilterBatch:
    """F independent filters built in one launch sequence on the device.

    num_new[f] inputs feed filter f (runs concatenated in filter order); old=[(batch, i)
    or None] merges a previously built filter (incremental routing_filter_add)."""

    def __init__(self, cfg: RoutingConfig, num_new, values=None, old=None, engine=None):
        self.engine = engine or default_engine()
        self.cfg = cfg
        L = load_library()
        nn = np.ascontiguousarray(num_new, dtype=np.uint32)
        self.F = nn.size
        vals = np.ascontiguousarray(values if values is not None else np.zeros(self.F),
                                    dtype=np.uint16)
        self.num_new = nn
        self.values = vals
        self._keep = [nn, vals]
        ob_arr = oi_arr = None
        if old is not None:
            ob_arr = (ctypes.c_void_p * self.F)(*[(o[0].h.value if o else None) for o in old])
            oi_arr = np.ascontiguousarray([(o[1] if o else 0) for o in old], dtype=np.uint32)
            self._keep += [ob_arr, oi_arr, [o[0] for o in old if o]]
        h = ctypes.c_void_p()
        _check(L.rf_amd_batch_create(self.engine.h, ctypes.byref(cfg.c()), self.F,
                                     nn.ctypes.data, vals.ctypes.data,
                                     ctypes.cast(ob_arr, ctypes.c_void_p) if ob_arr is not None else None,
                                     oi_arr.ctypes.data if oi_arr is not None else None,
                                     ctypes.byref(h)))
        self.h = h

    @classmethod
    def imported(cls, cfg: RoutingConfig, infos, d_pages, d_slots, device_resident=True, engine=None):
        """A built, probe-only batch from packed images (rf_amd_batch_import); infos: one
        RfFilterInfo per filter."""
        self = cls.__new__(cls)
        self.engine = engine or default_engine()
        self.cfg = cfg
        self.F = len(infos)
        arr = (RfFilterInfo * max(1, self.F))(*infos)
        self._keep = [arr]
        h = ctypes.c_void_p()
        _check(load_library().rf_amd_batch_import(self.engine.h, ctypes.byref(cfg.c()), self.F, arr,
                                                  _hptr(d_pages), _hptr(d_slots), 1 if device_resident else 0,
                                                  ctypes.byref(h)))
        self.h = h
        return self

    def export(self, d_pages, d_slots, stream=None):
        """Pack every filter's pages and slots (device tensors sized by export_sizes())."""
        _check(load_library().rf_amd_batch_export(self.h, _dptr(d_pages), d_pages.numel() * d_pages.element_size(),
                                                  _dptr(d_slots), d_slots.numel(), _stream(stream)))

    def export_sizes(self):
        """(infos, total page bytes, total index slots) of the packed export."""
        infos = [self.info(f) for f in range(self.F)]
        return infos, sum(i.num_pages for i in infos) * self.cfg.page_size, sum(i.num_indices for i in infos)

    def close(self, stream=None):
        """release the batch; with `stream`, stream-ordered (rf_amd_batch_destroy_on: every
        use of the batch must be ordered before the stream's current end), else after a
        device synchronisation"""
        if getattr(self, "h", None):
            if stream is not None:
                _check(load_library().rf_amd_batch_destroy_on(self.h, _stream(stream)))
            else:
                load_library().rf_amd_batch_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def build_keys(self, d_keys, key_len, stream=None):
        _check(load_library().rf_amd_batch_build_keys(self.h, _dptr(d_keys), key_len, _stream(stream)))

    def build_var_keys(self, d_bytes, d_offsets, stream=None):
        _check(load_library().rf_amd_batch_build_var_keys(self.h, _dptr(d_bytes), _dptr(d_offsets),
                                                          _stream(stream)))

    def build_hashes(self, d_hashes, stream=None):
        _check(load_library().rf_amd_batch_build_hashes(self.h, _dptr(d_hashes), _stream(stream)))

    def probe_keys(self, d_keys, key_len, d_filter_id, n, d_found, stream=None):
        _check(load_library().rf_amd_batch_probe_keys(self.h, _dptr(d_keys), key_len,
                                                      _dptr(d_filter_id), n, _dptr(d_found), _stream(stream)))

    def probe_var_keys(self, d_bytes, d_offsets, d_filter_id, n, d_found, stream=None):
        _check(load_library().rf_amd_batch_probe_var_keys(self.h, _dptr(d_bytes), _dptr(d_offsets),
                                                          _dptr(d_filter_id), n, _dptr(d_found),
                                                          _stream(stream)))

    def probe_hashes(self, d_hashes, d_filter_id, n, d_found, stream=None):
        _check(load_library().rf_amd_batch_probe_hashes(self.h, _dptr(d_hashes), _dptr(d_filter_id),
                                                        n, _dptr(d_found), _stream(stream)))

    def probe_keys_runs(self, d_keys, key_len, counts, d_found, stream=None):
        """Probes grouped by filter: counts[f] probes of filter f, in filter order."""
        c = (ctypes.c_uint64 * self.F)(*[int(x) for x in counts])
        _check(load_library().rf_amd_batch_probe_keys_runs(self.h, _dptr(d_keys), key_len, c, _dptr(d_found),
                                                           _stream(stream)))

    def probe_hashes_runs(self, d_hashes, counts, d_found, stream=None):
        c = (ctypes.c_uint64 * self.F)(*[int(x) for x in counts])
        _check(load_library().rf_amd_batch_probe_hashes_runs(self.h, _dptr(d_hashes), c, _dptr(d_found),
                                                             _stream(stream)))

    def probe_floor(self, d_in, key_len, counts, d_out, stream=None):
        """The probe's memory floor (rf_amd_debug_probe_floor): the fast path's traffic over the
        same runs with the arithmetic removed; d_out gets no lookup results."""
        c = (ctypes.c_uint64 * self.F)(*[int(x) for x in counts])
        _check(load_library().rf_amd_debug_probe_floor(self.h, _dptr(d_in), key_len, c, _dptr(d_out),
                                                       _stream(stream)))

    def probe_pairs(self, d_pairs, n, d_found, stream=None):
        """Probes given as (local filter id << 32 | hash) u64 pairs (routed probes, route.py)."""
        _check(load_library().rf_amd_batch_probe_pairs(self.h, _dptr(d_pairs), n, _dptr(d_found),
                                                       _stream(stream)))

    # fresh builds: partition = fused hash + coarse-bucket partition (K1+K3); count_scan and
    # scatter = the spill fallback (near zero unless a coarse bucket overflowed); incremental
    # builds: partition = K1 count, count_scan = K2, scatter = K3. assemble includes the
    # probe lines.
    STAGES = ["partition", "count_scan", "scatter", "cb_sort", "cb_sort_big", "layout",
              "assemble", "build_total", "probe"]

    def set_timing(self, enable=True, sets=1, probe_only=False):
        """Per-stage HIP-event timing; `sets` rounds (build + probe) kept in a ring.
        probe_only: record only the probe's two events (the build stages read -1)."""
        n = sets if enable else 0
        _check(load_library().rf_amd_batch_set_timing(self.h, -n if probe_only else n))

    def debug_lines(self) -> np.ndarray:
        """The batch's device-only probe lines (diagnostics), as an (N, 64) uint8 array."""
        L, n = load_library(), ctypes.c_uint64(0)
        _check(L.rf_amd_debug_read_lines(self.h, None, 0, ctypes.byref(n)))
        out = np.zeros((n.value, 64), dtype=np.uint8)
        _check(L.rf_amd_debug_read_lines(self.h, out.ctypes.data, out.nbytes, ctypes.byref(n)))
        return out

    def debug_rebuild_lines(self):
        """Re-cut the probe lines from the images with the image-upload kernel (diagnostics)."""
        _check(load_library().rf_amd_debug_rebuild_lines(self.h))

    def timings(self, back=0):
        """Per-stage milliseconds of a build / probe round (HIP events on the launch stream);
        back = 0 is the latest round, up to sets - 1 (set_timing)."""
        arr = (ctypes.c_float * len(self.STAGES))()
        _check(load_library().rf_amd_batch_timings_back(self.h, back, arr, len(self.STAGES)))
        return dict(zip(self.STAGES, [float(x) for x in arr]))

    def info(self, f):
        out = RfFilterInfo()
        _check(load_library().rf_amd_batch_info(self.h, f, ctypes.byref(out)))
        return out

    def infos(self, stream=None):
        """every filter's RfFilterInfo (one synchronisation: with `stream`, the build's
        stream, or the whole device)"""
        arr = (RfFilterInfo * self.F)()
        _check(load_library().rf_amd_batch_infos(self.h, arr, _stream(stream)))
        return list(arr)

    def read_image_async(self, f, h_pages, h_slots, stream=None):
        """D2H of filter f's pages/slots into (pinned) host tensors sized by the caller."""
        _check(load_library().rf_amd_batch_read_image_async(
            self.h, f, h_pages.data_ptr(), h_pages.numel(), h_slots.data_ptr(), h_slots.numel(),
            _stream(stream)))

    def image(self, f) -> RoutingFilter:
        inf = self.info(f)
        if inf.error:
            raise PlatformStatusError(STATUS_BAD_PARAM, f"filter {f} error bits {inf.error:#x}")
        pages = np.zeros(inf.num_pages * self.cfg.page_size, dtype=np.uint8)
        slots = np.zeros(inf.num_indices, dtype=np.uint64)
        _check(load_library().rf_amd_batch_read_image(self.h, f, pages.ctypes.data, pages.size,
                                                      slots.ctypes.data, slots.size))
        return RoutingFilter(inf.num_fingerprints, inf.num_unique, inf.value_size,
                             inf.num_indices, inf.num_pages, pages, slots)
