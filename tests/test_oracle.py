"""CPU tests: the parity oracle against the reference's own facts and the golden vectors.

Pinning (see oracle/rf_oracle.h): reference-run known answers (known_answers.json), the
reference's own PackedArray.c (packedarray.npz / oracle/_ref), XXH32 from the image's
libxxhash (xxh32.json). filters.npz / sha256.json are oracle outputs kept as regression
fixtures and as the GPU parity targets.
"""
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import GOLD
from splinterdb_amd import keys as K


def test_xxh32_vectors(oracle):
    with open(os.path.join(GOLD, "xxh32.json")) as fh:
        vecs = json.load(fh)["vectors"]
    for v in vecs:
        assert oracle.xxh32(bytes.fromhex(v["hex"]), v["seed"]) == v["xxh32"]


def test_xxh32_matches_system_libxxhash(oracle):
    import ctypes
    path = "/lib/x86_64-linux-gnu/libxxhash.so.0"
    if not os.path.exists(path):
        pytest.skip("system libxxhash absent")
    L = ctypes.CDLL(path)
    L.XXH32.restype = ctypes.c_uint32
    L.XXH32.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32]
    d, o = K.var_keys(500)
    h = oracle.hash_var(d, o)
    for i in range(500):
        b = bytes(d[o[i]:o[i + 1]])
        buf = ctypes.create_string_buffer(b, len(b))
        assert L.XXH32(buf, len(b), 42) == h[i]


def test_packedarray_vs_reference_vectors(oracle):
    import ctypes
    z = np.load(os.path.join(GOLD, "packedarray.npz"))
    L = oracle.lib()
    keys = sorted(k[:-3] for k in z.files if k.endswith("_in"))
    assert len(keys) == 1024
    for key in keys:
        bits = int(key.split("_")[0][1:])
        off = int(key.split("_")[1][1:])
        fill = int(key.split("_")[3][1:], 16)
        items = z[key + "_in"]
        want = z[key + "_out"]
        buf = np.full(want.size, fill, dtype=np.uint32)
        L.rfo_pack(buf.ctypes.data, off, items.ctypes.data, items.size, bits)
        assert (buf == want).all(), key
        got = np.zeros(items.size, dtype=np.uint32)
        L.rfo_unpack(want.ctypes.data, off, got.ctypes.data, items.size, bits)
        assert (got == items).all(), key
        for i in (0, items.size - 1):
            assert L.rfo_get(want.ctypes.data, off + i, bits) == items[i]


def test_packedarray_fuzz_vs_compiled_reference(oracle):
    ref = oracle.ref_packedarray()
    if ref is None:
        pytest.skip("oracle/_ref not built (reference tree absent)")
    L = oracle.lib()
    rng = np.random.default_rng(3)
    for _ in range(300):
        bits = int(rng.integers(1, 33))
        off = int(rng.integers(0, 70))
        cnt = int(rng.integers(1, 300))
        items = (rng.integers(0, 1 << 32, size=cnt, dtype=np.uint64) & ((1 << bits) - 1)).astype(np.uint32)
        n = ((off + cnt) * bits + 31) // 32 + 2
        a = rng.integers(0, 1 << 32, size=n, dtype=np.uint64).astype(np.uint32)
        b = a.copy()
        ref.PackedArray_pack(a.ctypes.data, off, items.ctypes.data, cnt, bits)
        L.rfo_pack(b.ctypes.data, off, items.ctypes.data, cnt, bits)
        assert (a == b).all()


def test_known_answers_1M(oracle):
    """Reference-run facts for 1M sequential keys."""
    with open(os.path.join(GOLD, "known_answers.json")) as fh:
        ka = json.load(fh)
    cfg = oracle.make_config()
    h = oracle.hash_fixed(K.seq_keys(0, 1000000).reshape(-1), 24)
    f = oracle.filter_add(cfg, h)
    g = ka["geometry"][0]
    assert (f.num_unique, f.num_pages, f.space_use_bytes()) == (g["num_unique"], g["data_pages"],
                                                              g["space_use_bytes"])
    pages, slots = f.pages(), f.slots()
    for fact in ka["index_facts_1M_lis8"]:
        s = int(slots[fact["index"]])
        assert int(pages[s]) | (int(pages[s + 1]) << 8) == fact["count"]
        if "page" in fact:
            assert divmod(s, 4096) == (fact["page"], fact["offset"])
    neg = oracle.hash_fixed(K.seq_keys(1000000, 100000).reshape(-1), 24)
    assert round(float((f.lookup_hashes(neg) != 0).mean()) * 100, 2) == ka["fp_rate"][0]["rate_pct"]
    # no false negatives (tests/functional/filter_test.c:100-116)
    assert (f.lookup_hashes(h[:200000]) & np.uint64(1)).all()


@pytest.mark.slow
def test_known_answers_geometry(oracle):
    with open(os.path.join(GOLD, "known_answers.json")) as fh:
        ka = json.load(fh)
    for g in ka["geometry"][1:]:
        cfg = oracle.make_config(log_index_size=g["lis"])
        f = oracle.filter_add(cfg, oracle.hash_fixed(K.seq_keys(0, g["keys"]).reshape(-1), 24))
        assert f.num_unique == g["num_unique"]
        assert f.space_use_bytes() == g["space_use_bytes"]
        if "data_pages" in g:
            assert f.num_pages == g["data_pages"]


@pytest.mark.slow
def test_known_answers_filter_test_chain(oracle):
    """tests/functional/filter_test.c basic mode: 8 incremental values of 1,048,575 fps."""
    with open(os.path.join(GOLD, "known_answers.json")) as fh:
        ch = json.load(fh)["filter_test_basic_chain"]
    cfg = oracle.make_config()
    nf, nv = ch["fps_per_value"], ch["values"]
    filt = None
    for i in range(nv):
        h = oracle.hash_fixed(K.ids_keys((i + 1) * np.arange(nf, dtype=np.uint64)).reshape(-1), 24)
        filt = oracle.filter_add(cfg, h, value=i, old=filt)
        if i == 0:
            assert filt.num_unique == ch["num_unique_first"]
        assert (filt.lookup_hashes(h[:50000]) >> np.uint64(i) & np.uint64(1)).all()
    assert filt.num_unique == ch["num_unique_last"]
    unused = (nv + 1) * nf
    neg = oracle.hash_fixed(K.ids_keys(np.arange(unused, unused + nf, dtype=np.uint64)).reshape(-1), 24)
    assert round((filt.lookup_hashes(neg) != 0).sum() / nf, 4) == ch["fp_rate_4dp"]


def _golden_cases(z):
    return sorted({k.split("/")[0] for k in z.files if k.endswith("/meta")})


def test_oracle_reproduces_golden_filters(oracle, golden_filters):
    from oracle.gen_golden import filter_cases, case_hashes
    z = golden_filters
    for name, ckw, kind, n, value in filter_cases():
        cfg = oracle.make_config(**ckw)
        h, _ = case_hashes(kind, n)
        assert (h == z[name + "/hashes"]).all(), name
        f = oracle.filter_add(cfg, h, value=value)
        meta = z[name + "/meta"]
        assert [f.num_fingerprints, f.num_unique, f.value_size, f.num_indices, f.num_pages] == \
            list(meta[:5]), name
        assert (f.pages() == z[name + "/pages"]).all(), name
        assert (f.slots()[: f.num_indices] == z[name + "/slots"]).all(), name
        assert (f.lookup_hashes(z[name + "/probe_hashes"]) == z[name + "/probe_found"]).all(), name


def test_oracle_chain_golden(oracle, golden_filters):
    z = golden_filters
    cfg = oracle.make_config()
    filt = None
    chain = []
    for i in range(4):
        h = z[f"chain_v{i}/hashes"]
        filt = oracle.filter_add(cfg, h, value=i, old=filt)
        chain.append(filt)
        assert (filt.pages() == z[f"chain_v{i}/pages"]).all()
        assert (filt.slots()[: filt.num_indices] == z[f"chain_v{i}/slots"]).all()
    assert oracle.estimate_unique_fp(cfg, chain) == int(z["chain/estimate_unique_fp"][0])


@pytest.mark.slow
def test_oracle_sha256_goldens(oracle):
    with open(os.path.join(GOLD, "sha256.json")) as fh:
        sh = json.load(fh)
    cfg = oracle.make_config()
    f = oracle.filter_add(cfg, oracle.hash_fixed(K.seq_keys(0, 1000000).reshape(-1), 24))
    assert hashlib.sha256(f.pages().tobytes()).hexdigest() == sh["seq_n1000000_lis8"]["pages_sha256"]


def test_oracle_rejects_reference_ub(oracle):
    cfg = oracle.make_config()
    with pytest.raises(ValueError):
        oracle.filter_add(cfg, np.zeros(0, dtype=np.uint32))  # clz(0): UB in the reference
    with pytest.raises(ValueError):
        oracle.filter_add(cfg, np.arange(10, dtype=np.uint32), value=200)  # 26 + 8 > 32


def test_estimate_unique_keys_from_count(oracle):
    cfg = oracle.make_config()
    for u in (0, 1, 1000, 992680, 4254486):
        v = oracle.estimate_unique_keys_from_count(cfg, u)
        assert abs(v - u) <= max(2, u * 0.1)
