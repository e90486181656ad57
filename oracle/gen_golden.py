"""Generate the committed golden fixtures under tests/golden/ (TEST INFRASTRUCTURE ONLY).

Run in the build container:  python oracle/gen_golden.py
Sources of truth, in order of strength:
  * known_answers.json -- facts recorded from runs of the REFERENCE itself (SURVEY.md §6,
    §8c); checked here against the oracle before anything is written;
  * packedarray.npz    -- outputs of the reference's own src/PackedArray.c, compiled from
    its sources into oracle/_ref/ (this script refuses to run without it);
  * xxh32.json         -- XXH32 from the image's libxxhash.so.0 (the library the reference
    links, Makefile:94), cross-checked against python-xxhash;
  * filters.npz        -- filter images / lookup vectors produced by the oracle
    (rf_oracle.c), whose correctness rests on the three items above.
"""
import ctypes
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402
from splinterdb_amd import keys as K  # noqa: E402

GOLD = os.path.join(ROOT, "tests", "golden")

# Reference-run facts (SURVEY.md §6 table "Filter geometry" and §8(c) "Known-answer facts").
KNOWN_ANSWERS = {
    "source": "SURVEY.md §6 and §8(c): outputs of the reference's routing_filter_add/"
              "lookup run in the survey container (sequential-id 24 B keys, seed 42, "
              "fp_size 26, 4 KiB pages, 32-page extents)",
    "geometry": [
        {"keys": 1000000, "lis": 8, "num_unique": 992680, "data_pages": 291, "space_use_bytes": 1445888},
        {"keys": 1000000, "lis": 9, "num_unique": 992680, "data_pages": 328, "space_use_bytes": 1576960},
        {"keys": 1048576, "lis": 8, "num_unique": 1040504, "data_pages": 273, "space_use_bytes": 1314816},
        {"keys": 8000000, "lis": 8, "num_unique": 7548068, "data_pages": 1366, "space_use_bytes": 5771264},
        {"keys": 8388607, "lis": 8, "num_unique": 7892883, "space_use_bytes": 6033408},
    ],
    "index_facts_1M_lis8": [
        {"index": 0, "count": 509}, {"index": 1, "count": 516}, {"index": 2, "count": 472},
        {"index": 2047, "count": 486, "page": 290, "offset": 1573},
    ],
    "fp_rate": [
        {"keys": 1000000, "lis": 8, "negatives": "ids N..N+99999", "rate_pct": 1.44},
    ],
    "filter_test_basic_chain": {
        "fps_per_value": 1048575, "values": 8, "keys": "(i+1)*j",
        "num_unique_first": 1040503, "num_unique_last": 4254486,
        "fp_rate_4dp": 0.0625,
    },
    "xxh32_seq_ids_0_3": ["b7684d5d", "be25666a", "166202fa", "d024e88e"],
}


def check_known_answers():
    for g in KNOWN_ANSWERS["geometry"]:
        cfg = O.make_config(log_index_size=g["lis"])
        f = O.filter_add(cfg, O.hash_fixed(K.seq_keys(0, g["keys"]).reshape(-1), 24))
        assert f.num_unique == g["num_unique"], (g, f.num_unique)
        assert f.space_use_bytes() == g["space_use_bytes"], (g, f.space_use_bytes())
        if "data_pages" in g:
            assert f.num_pages == g["data_pages"], (g, f.num_pages)
    cfg = O.make_config()
    h = O.hash_fixed(K.seq_keys(0, 1000000).reshape(-1), 24)
    f = O.filter_add(cfg, h)
    pages, slots = f.pages(), f.slots()
    for fact in KNOWN_ANSWERS["index_facts_1M_lis8"]:
        s = int(slots[fact["index"]])
        assert int(pages[s]) | (int(pages[s + 1]) << 8) == fact["count"], fact
        if "page" in fact:
            assert divmod(s, 4096) == (fact["page"], fact["offset"]), fact
    neg = O.hash_fixed(K.seq_keys(1000000, 100000).reshape(-1), 24)
    rate = float((f.lookup_hashes(neg) != 0).mean()) * 100
    assert round(rate, 2) == 1.44, rate
    ch = KNOWN_ANSWERS["filter_test_basic_chain"]
    nf, nv = ch["fps_per_value"], ch["values"]
    filt = None
    for i in range(nv):
        hh = O.hash_fixed(K.ids_keys((i + 1) * np.arange(nf, dtype=np.uint64)).reshape(-1), 24)
        filt = O.filter_add(cfg, hh, value=i, old=filt)
        if i == 0:
            assert filt.num_unique == ch["num_unique_first"]
    assert filt.num_unique == ch["num_unique_last"]
    unused = (nv + 1) * nf
    neg = O.hash_fixed(K.ids_keys(np.arange(unused, unused + nf, dtype=np.uint64)).reshape(-1), 24)
    fp = (filt.lookup_hashes(neg) != 0).sum() / nf
    assert round(fp, 4) == ch["fp_rate_4dp"], fp
    got = [format(O.xxh32(K.ids_keys([i]).tobytes()), "08x") for i in range(4)]
    assert got == KNOWN_ANSWERS["xxh32_seq_ids_0_3"], got
    print("oracle agrees with every reference known-answer fact")


def gen_xxh32():
    sys_lib = ctypes.CDLL("/lib/x86_64-linux-gnu/libxxhash.so.0")
    sys_lib.XXH32.restype = ctypes.c_uint32
    sys_lib.XXH32.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32]
    import xxhash
    rng = np.random.default_rng(7)
    vecs = []
    for ln in list(range(0, 130)) + [255, 256, 1000, 4096]:
        for seed in (0, 42, 0xDEADBEEF):
            data = rng.integers(0, 256, size=ln, dtype=np.uint8).tobytes()
            buf = ctypes.create_string_buffer(data, max(ln, 1))
            a = sys_lib.XXH32(buf, ln, seed)
            b = xxhash.xxh32(data, seed=seed).intdigest()
            assert a == b
            vecs.append({"hex": data.hex(), "seed": seed, "xxh32": a})
    with open(os.path.join(GOLD, "xxh32.json"), "w") as fh:
        json.dump({"source": "libxxhash.so.0 (image) == python-xxhash", "vectors": vecs}, fh)
    print("xxh32.json:", len(vecs), "vectors")


def gen_packedarray():
    ref = O.ref_packedarray()
    if ref is None:
        raise SystemExit("oracle/_ref/libpackedarray_ref.so missing: run make -C oracle")
    rng = np.random.default_rng(11)
    out = {}
    for bits in range(1, 33):
        for offset in (0, 3, 31, 37):
            for count in (1, 7, 32, 100):
                mask = (1 << bits) - 1
                items = (rng.integers(0, 1 << 32, size=count, dtype=np.uint64) & mask).astype(np.uint32)
                nwords = ((offset + count) * bits + 31) // 32 + 2
                for fill in (0x00000000, 0xA5A5A5A5):
                    buf = np.full(nwords, fill, dtype=np.uint32)
                    ref.PackedArray_pack(buf.ctypes.data, offset, items.ctypes.data, count, bits)
                    key = f"b{bits}_o{offset}_c{count}_f{fill:x}"
                    out[key + "_in"] = items
                    out[key + "_out"] = buf
                    got = np.array([ref.PackedArray_get(buf.ctypes.data, offset + i, bits)
                                    for i in range(count)], dtype=np.uint32)
                    assert (got == items).all()
                    un = np.zeros(count, dtype=np.uint32)
                    ref.PackedArray_unpack(buf.ctypes.data, offset, un.ctypes.data, count, bits)
                    assert (un == items).all()
    np.savez_compressed(os.path.join(GOLD, "packedarray.npz"), **out)
    print("packedarray.npz:", len(out) // 2, "cases")


def filter_cases():
    """(name, cfg kwargs, key kind, n, value) -- SURVEY.md §8(c) 'Goldens to commit'."""
    cases = []
    for lis in (8, 9):
        for n in (1, 2, 100, 1000, 10000, 100000):
            cases.append((f"seq_lis{lis}_n{n}_v0", dict(log_index_size=lis), "seq", n, 0))
    cases += [
        ("seq_lis8_n1000_v5", dict(), "seq", 1000, 5),
        ("seq_lis8_n100000_v31", dict(), "seq", 100000, 31),
        ("rand24_lis8_n50000_v0", dict(), "rand24", 50000, 0),
        ("var8_100_lis8_n30000_v0", dict(), "var", 30000, 0),
        ("dups_lis8_n20000_v2", dict(), "dups", 20000, 2),
        ("fp20_lis8_n50000_v0", dict(fingerprint_size=20), "seq", 50000, 0),
        ("fp28_lis8_n3000_v7", dict(fingerprint_size=28), "seq", 3000, 7),
        ("fp32_lis8_n5000_v0", dict(fingerprint_size=32), "seq", 5000, 0),
        ("lis6_n40000_v1", dict(log_index_size=6), "seq", 40000, 1),
    ]
    return cases


def case_hashes(kind, n, seed=42):
    if kind == "seq":
        return O.hash_fixed(K.seq_keys(0, n).reshape(-1), 24, seed), None
    if kind == "rand24":
        return O.hash_fixed(K.random_keys(n).reshape(-1), 24, seed), None
    if kind == "dups":
        return O.hash_fixed(K.ids_keys(np.arange(n, dtype=np.uint64) % 1500).reshape(-1), 24, seed), None
    if kind == "var":
        d, o = K.var_keys(n)
        return O.hash_var(d, o, seed), None
    raise ValueError(kind)


def probe_hashes(kind, n, seed=42):
    pos, _ = case_hashes(kind, n, seed)
    pos = pos[: min(n, 2000)]
    neg = O.hash_fixed(K.random_keys(2000, seed=0xBAD).reshape(-1), 24, seed)
    return np.concatenate([pos, neg])


def image_dict(prefix, f, cfg):
    ni = f.num_indices
    return {
        prefix + "meta": np.array([f.num_fingerprints, f.num_unique, f.value_size, ni,
                                   f.num_pages, f.space_use_bytes()], dtype=np.uint64),
        prefix + "pages": f.pages(),
        prefix + "slots": f.slots()[:ni],
    }


def gen_filters():
    out = {}
    for name, ckw, kind, n, value in filter_cases():
        cfg = O.make_config(**ckw)
        h, _ = case_hashes(kind, n)
        f = O.filter_add(cfg, h, value=value)
        out.update(image_dict(name + "/", f, cfg))
        ph = probe_hashes(kind, n)
        out[name + "/probe_hashes"] = ph
        out[name + "/probe_found"] = f.lookup_hashes(ph)
        out[name + "/hashes"] = h
    # incremental chain, filter_test basic pattern (keys (i+1)*j, values 0..3)
    cfg = O.make_config()
    filt = None
    chain = []
    for i in range(4):
        h = O.hash_fixed(K.ids_keys((i + 1) * np.arange(20000, dtype=np.uint64)).reshape(-1), 24)
        filt = O.filter_add(cfg, h, value=i, old=filt)
        chain.append(filt)
        out.update(image_dict(f"chain_v{i}/", filt, cfg))
        out[f"chain_v{i}/hashes"] = h
        ph = np.concatenate([h[:1000], probe_hashes("seq", 10)[10:]])
        out[f"chain_v{i}/probe_hashes"] = ph
        out[f"chain_v{i}/probe_found"] = filt.lookup_hashes(ph)
    out["chain/estimate_unique_fp"] = np.array([O.estimate_unique_fp(cfg, chain)], dtype=np.uint64)
    np.savez_compressed(os.path.join(GOLD, "filters.npz"), **out)
    print("filters.npz:", len(out), "arrays")


SHARD_SAMPLE = (0, 1, 77, 255, 256, 511, 768, 1023)  # filters of C3 (0-255) and C4 (0-1023)


def gen_sha():
    res = {}
    for n, lis in ((1000000, 8), (8000000, 8), (1048576, 8)):
        cfg = O.make_config(log_index_size=lis)
        f = O.filter_add(cfg, O.hash_fixed(K.seq_keys(0, n).reshape(-1), 24))
        res[f"seq_n{n}_lis{lis}"] = {
            "pages_sha256": hashlib.sha256(f.pages().tobytes()).hexdigest(),
            "slots_sha256": hashlib.sha256(f.slots()[: f.num_indices].tobytes()).hexdigest(),
            "num_unique": f.num_unique, "num_pages": f.num_pages}
    for n in (1 << 20,):
        cfg = O.make_config()
        f = O.filter_add(cfg, O.hash_fixed(K.random_keys(n).reshape(-1), 24))
        res[f"rand24_n{n}_lis8"] = {
            "pages_sha256": hashlib.sha256(f.pages().tobytes()).hexdigest(),
            "slots_sha256": hashlib.sha256(f.slots()[: f.num_indices].tobytes()).hexdigest(),
            "num_unique": f.num_unique, "num_pages": f.num_pages}
    # C3 / C4 filters: filter k of the 2^20-key layout holds sequential ids [k 2^20, (k+1) 2^20)
    cfg = O.make_config()
    for k in SHARD_SAMPLE:
        n = 1 << 20
        f = O.filter_add(cfg, O.hash_fixed(K.seq_keys(k * n, n).reshape(-1), 24))
        res[f"seq_n{n}_lis8_k{k}"] = {
            "pages_sha256": hashlib.sha256(f.pages().tobytes()).hexdigest(),
            "slots_sha256": hashlib.sha256(f.slots()[: f.num_indices].tobytes()).hexdigest(),
            "num_unique": f.num_unique, "num_pages": f.num_pages}
    with open(os.path.join(GOLD, "sha256.json"), "w") as fh:
        json.dump(res, fh, indent=1)
    print("sha256.json:", list(res))


CHAIN_SAMPLE = (0, 1, 63)
CHAIN_ROUNDS, CHAIN_N = 8, (1 << 20) - 1


def gen_chain_sha():
    """Compaction chains (bench.py --workload compaction): filter f after CHAIN_ROUNDS
    incremental routing_filter_adds of CHAIN_N keys of ids (f << 32) + (v + 1) * j, value v,
    built by the REFERENCE itself (oracle/_ref/libref_rf.so, oracle/ref_harness.c
    chain_worker). Merged into sha256.json."""
    from oracle import refimpl as R
    path = os.path.join(GOLD, "sha256.json")
    with open(path) as fh:
        res = json.load(fh)
    with R.Stack(log_index_size=8, cache_mib=4096, disk_mib=65536) as s:
        _, keep = s.bench_chain(max(CHAIN_SAMPLE) + 1, CHAIN_ROUNDS, CHAIN_N, 8)
        for f in CHAIN_SAMPLE:
            img = s.image(keep[f])
            res[f"chain_f{f}_v{CHAIN_ROUNDS}_n{CHAIN_N}_lis8"] = {
                "pages_sha256": hashlib.sha256(img.pages.tobytes()).hexdigest(),
                "slots_sha256": hashlib.sha256(img.slots.tobytes()).hexdigest(),
                "num_fingerprints": int(keep[f].num_fingerprints), "num_unique": int(keep[f].num_unique),
                "num_pages": int(img.pages.size // 4096), "source": "reference"}
    with open(path, "w") as fh:
        json.dump(res, fh, indent=1)
    print("sha256.json chains:", CHAIN_SAMPLE)


if __name__ == "__main__":
    os.makedirs(GOLD, exist_ok=True)
    O.build()
    check_known_answers()
    with open(os.path.join(GOLD, "known_answers.json"), "w") as fh:
        json.dump(KNOWN_ANSWERS, fh, indent=1)
    gen_xxh32()
    gen_packedarray()
    gen_filters()
    gen_sha()
    gen_chain_sha()
