"""GPU parity tests: the HIP engine (through the C ABI) against the oracle and the
committed golden fixtures. Bit-exact on every page byte and slot, num_unique, num_pages,
and every probe's found_values bit-vector."""
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import GOLD
from splinterdb_amd import engine as E
from splinterdb_amd import keys as K

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to("cuda:0")


def cfg_of(ckw):
    return E.routing_config_init(**ckw)


def case_input(kind, n):
    """device tensors for a golden case: ('keys', tensor, key_len) or ('var', bytes, offs)"""
    if kind == "seq":
        return "keys", dev(K.seq_keys(0, n)), 24
    if kind == "rand24":
        return "keys", dev(K.random_keys(n)), 24
    if kind == "dups":
        return "keys", dev(K.ids_keys(np.arange(n, dtype=np.uint64) % 1500)), 24
    if kind == "var":
        d, o = K.var_keys(n)
        return "var", dev(d), dev(o)
    raise ValueError(kind)


def assert_image_eq(img, z, name):
    meta = z[name + "/meta"]
    got = [img.num_fingerprints, img.num_unique, img.value_size, img.num_indices, img.num_pages]
    assert got == [int(x) for x in meta[:5]], (name, got, list(meta[:5]))
    want = z[name + "/pages"]
    if not (img.pages == want).all():
        bad = np.nonzero(img.pages != want)[0]
        raise AssertionError(f"{name}: {bad.size} page bytes differ, first at {bad[0]} "
                             f"(page {bad[0] // 4096} off {bad[0] % 4096})")
    assert (img.slots == z[name + "/slots"]).all(), name


def test_golden_filters_from_keys(golden_filters):
    from oracle.gen_golden import filter_cases
    z = golden_filters
    for name, ckw, kind, n, value in filter_cases():
        cfg = cfg_of(ckw)
        b = E.FilterBatch(cfg, [n], [value])
        inp = case_input(kind, n)
        if inp[0] == "keys":
            b.build_keys(inp[1], inp[2])
        else:
            b.build_var_keys(inp[1], inp[2])
        img = b.image(0)
        assert_image_eq(img, z, name)
        ph = dev(z[name + "/probe_hashes"])
        fid = torch.zeros(ph.numel(), dtype=torch.int32, device="cuda:0")
        found = torch.zeros(ph.numel(), dtype=torch.int64, device="cuda:0")
        b.probe_hashes(ph, fid, ph.numel(), found)
        torch.cuda.synchronize()
        assert (found.cpu().numpy().view(np.uint64) == z[name + "/probe_found"]).all(), name


def test_golden_filters_from_hashes_one_batch(golden_filters):
    """every lis-8 / fp-26 golden case as ONE multi-filter batch from hashes"""
    from oracle.gen_golden import filter_cases
    z = golden_filters
    cases = [c for c in filter_cases() if not c[1]]
    cfg = E.routing_config_init()
    hs = [z[c[0] + "/hashes"] for c in cases]
    b = E.FilterBatch(cfg, [h.size for h in hs], [c[4] for c in cases])
    b.build_hashes(dev(np.concatenate(hs)))
    for f, c in enumerate(cases):
        assert_image_eq(b.image(f), z, c[0])
    # batched probe: every case's probes, each tagged with its filter
    ph = np.concatenate([z[c[0] + "/probe_hashes"] for c in cases])
    fid = np.concatenate([np.full(z[c[0] + "/probe_hashes"].size, f, dtype=np.uint32)
                          for f, c in enumerate(cases)])
    want = np.concatenate([z[c[0] + "/probe_found"] for c in cases])
    found = torch.zeros(ph.size, dtype=torch.int64, device="cuda:0")
    b.probe_hashes(dev(ph), dev(fid), ph.size, found)
    torch.cuda.synchronize()
    assert (found.cpu().numpy().view(np.uint64) == want).all()


def test_dropin_routing_filter_add_and_lookup(golden_filters):
    z = golden_filters
    cfg = E.routing_config_init()
    for name, value in (("seq_lis8_n100000_v31", 31), ("rand24_lis8_n50000_v0", 0),
                        ("seq_lis8_n1_v0", 0)):
        f = E.routing_filter_add(cfg, None, z[name + "/hashes"], value)
        assert_image_eq(f, z, name)
        got = E.routing_filter_lookup_hashes(cfg, f, z[name + "/probe_hashes"])
        assert (got == z[name + "/probe_found"]).all()
    # keys-in single lookup (hash on the GPU)
    f = E.routing_filter_add(cfg, None, z["seq_lis8_n1000_v5/hashes"], 5)
    for i in (0, 1, 999):
        fv = E.routing_filter_lookup(cfg, f, K.seq_keys(i, 1).tobytes())
        assert E.routing_filter_is_value_found(fv, 5)


def test_incremental_chain_dropin(golden_filters):
    """routing_filter_add with old_filter (src/routing_filter.c:496-597), filter_test pattern"""
    z = golden_filters
    cfg = E.routing_config_init()
    filt = None
    for i in range(4):
        filt = E.routing_filter_add(cfg, filt, z[f"chain_v{i}/hashes"], i)
        assert_image_eq(filt, z, f"chain_v{i}")
        got = E.routing_filter_lookup_hashes(cfg, filt, z[f"chain_v{i}/probe_hashes"])
        assert (got == z[f"chain_v{i}/probe_found"]).all()


def test_incremental_chain_batch(golden_filters):
    """the same chain through the device-resident batch API (old = previous batch)"""
    z = golden_filters
    cfg = E.routing_config_init()
    prev = None
    keep = []
    for i in range(4):
        h = z[f"chain_v{i}/hashes"]
        b = E.FilterBatch(cfg, [h.size], [i], old=[(prev, 0)] if prev is not None else None)
        b.build_hashes(dev(h))
        assert_image_eq(b.image(0), z, f"chain_v{i}")
        keep.append(b)
        prev = b


def test_sha256_full_size_filters():
    with open(os.path.join(GOLD, "sha256.json")) as fh:
        sh = json.load(fh)
    cfg = E.routing_config_init()
    for key, gen in (("seq_n1000000_lis8", lambda: K.seq_keys(0, 1000000)),
                     ("seq_n8000000_lis8", lambda: K.seq_keys(0, 8000000)),
                     ("rand24_n1048576_lis8", lambda: K.random_keys(1 << 20))):
        keys = gen()
        b = E.FilterBatch(cfg, [keys.shape[0]])
        b.build_keys(dev(keys), 24)
        img = b.image(0)
        assert img.num_unique == sh[key]["num_unique"] and img.num_pages == sh[key]["num_pages"]
        assert hashlib.sha256(img.pages.tobytes()).hexdigest() == sh[key]["pages_sha256"], key
        assert hashlib.sha256(img.slots.tobytes()).hexdigest() == sh[key]["slots_sha256"], key


def test_c2_64M_eight_filters_vs_oracle(oracle):
    """BASELINE config 2: 64M x 24 B keys as 8 filters x 8,000,000 (per-filter cap), device
    resident; per-filter SHA-256 of pages/slots equals the oracle's; full 64M probe has no
    false negatives and agrees with the oracle on a sample."""
    cfg = E.routing_config_init()
    ocfg = oracle.make_config()
    F, n = 8, 8_000_000
    keys = K.seq_keys_torch(0, F * n, 24, "cuda:0")
    b = E.FilterBatch(cfg, [n] * F)
    b.build_keys(keys, 24)
    for f in range(F):
        img = b.image(f)
        assert img.num_fingerprints == n
        if f in (0, 5, 7):
            h = oracle.hash_fixed(K.seq_keys(f * n, n).reshape(-1), 24)
            of = oracle.filter_add(ocfg, h)
            assert (img.num_unique, img.num_pages) == (of.num_unique, of.num_pages)
            assert hashlib.sha256(img.pages.tobytes()).digest() == \
                hashlib.sha256(of.pages().tobytes()).digest(), f
            assert (img.slots == of.slots()[: of.num_indices]).all()
    fid = torch.arange(F * n, device="cuda:0", dtype=torch.int64).div(n, rounding_mode="floor").to(torch.int32)
    found = torch.zeros(F * n, dtype=torch.int64, device="cuda:0")
    b.probe_keys(keys, 24, fid, F * n, found)
    torch.cuda.synchronize()
    assert bool(((found & 1) == 1).all())  # value 0 found for every inserted key
    # sample vs oracle (filter 5)
    h = oracle.hash_fixed(K.seq_keys(5 * n, 20000).reshape(-1), 24)
    of = oracle.filter_add(ocfg, oracle.hash_fixed(K.seq_keys(5 * n, n).reshape(-1), 24))
    want = of.lookup_hashes(h)
    got = found[5 * n: 5 * n + 20000].cpu().numpy().view(np.uint64)
    assert (got == want).all()
    # negatives (ids never inserted): FP rate close to the reference's 10.97% at 8M keys
    neg = K.seq_keys_torch(F * n, 200000, 24, "cuda:0")
    nf = torch.zeros(200000, dtype=torch.int64, device="cuda:0")
    b.probe_keys(neg, 24, torch.zeros(200000, dtype=torch.int32, device="cuda:0"), 200000, nf)
    torch.cuda.synchronize()
    rate = float((nf != 0).float().mean())
    assert 0.09 < rate < 0.13


def test_duplicate_heavy_overflow_path(oracle):
    """all-identical keys overflow the LDS coarse bucket -> k_cb_sort_big"""
    cfg = E.routing_config_init()
    ocfg = oracle.make_config()
    for n, mod in ((100000, 1), (300000, 3), (60000, 20000)):
        keys = K.ids_keys(np.arange(n, dtype=np.uint64) % mod)
        b = E.FilterBatch(cfg, [n], [3])
        b.build_keys(dev(keys), 24)
        img = b.image(0)
        of = oracle.filter_add(ocfg, oracle.hash_fixed(keys.reshape(-1), 24), value=3)
        assert (img.num_unique, img.num_pages) == (of.num_unique, of.num_pages)
        assert (img.pages == of.pages()).all()
        assert (img.slots == of.slots()[: of.num_indices]).all()


def test_repeated_fingerprint_bins(oracle):
    """Buckets of 9-64 entries (ranked by a whole wave in K4) and over 64 (insertion sort),
    in LDS-resident coarse buckets, fresh and incremental (64-bit entries)."""
    cfg = E.routing_config_init()
    ocfg = oracle.make_config()
    rng = np.random.default_rng(3)
    for rep in (10, 30, 70, 200):
        base = rng.integers(0, 1 << 32, size=200_000 // rep, dtype=np.uint64).astype(np.uint32)
        h = rng.permutation(np.repeat(base, rep)).astype(np.uint32)
        b = E.FilterBatch(cfg, [h.size], [1])
        b.build_hashes(dev(h))
        img = b.image(0)
        of = oracle.filter_add(ocfg, h, value=1)
        assert (img.num_unique, img.num_pages) == (of.num_unique, of.num_pages), rep
        assert (img.pages == of.pages()).all(), rep
        assert (img.slots == of.slots()[: of.num_indices]).all(), rep
        # incremental: the same multiset again with value 2, merged into the old filter
        b2 = E.FilterBatch(cfg, [h.size], [2], old=[(b, 0)])
        b2.build_hashes(dev(h))
        img2 = b2.image(0)
        of2 = oracle.filter_add(ocfg, h, value=2, old=of)
        assert (img2.num_unique, img2.num_pages) == (of2.num_unique, of2.num_pages), rep
        assert (img2.pages == of2.pages()).all(), rep


def test_multi_filter_random_sizes_vs_oracle(oracle):
    """C3-style concurrent builds: mixed sizes/values in one batch, random probe routing"""
    cfg = E.routing_config_init(log_index_size=9)
    ocfg = oracle.make_config(log_index_size=9)
    rng = np.random.default_rng(5)
    sizes = [int(x) for x in rng.integers(1, 300000, size=12)] + [1, 2, 4095, 4096, 4097, 1 << 18]
    vals = [int(x) for x in rng.integers(0, 64, size=len(sizes))]
    total = sum(sizes)
    keys = K.random_keys(total, seed=99)
    b = E.FilterBatch(cfg, sizes, vals)
    b.build_keys(dev(keys), 24)
    ofs = []
    s = 0
    hashes = oracle.hash_fixed(keys.reshape(-1), 24)
    for f, (n, v) in enumerate(zip(sizes, vals)):
        of = oracle.filter_add(ocfg, hashes[s:s + n], value=v)
        img = b.image(f)
        assert (img.num_unique, img.num_pages) == (of.num_unique, of.num_pages), f
        assert (img.pages == of.pages()).all(), f
        assert (img.slots == of.slots()[: of.num_indices]).all(), f
        ofs.append(of)
        s += n
    P = 200000
    pk = K.random_keys(P, seed=7)
    pk[: P // 2] = keys[rng.integers(0, total, size=P // 2)]
    fid = rng.integers(0, len(sizes), size=P).astype(np.uint32)
    found = torch.zeros(P, dtype=torch.int64, device="cuda:0")
    b.probe_keys(dev(pk), 24, dev(fid), P, found)
    torch.cuda.synchronize()
    got = found.cpu().numpy().view(np.uint64)
    ph = oracle.hash_fixed(pk.reshape(-1), 24)
    for f in range(len(sizes)):
        m = fid == f
        assert (got[m] == ofs[f].lookup_hashes(ph[m])).all(), f


def test_var_keys_zipf_probe(oracle):
    """C5: variable-length 8-100 B keys, Zipf(0.99) positive mix + 10% negatives"""
    cfg = E.routing_config_init()
    ocfg = oracle.make_config()
    n = 200000
    d, o = K.var_keys(n)
    b = E.FilterBatch(cfg, [n])
    b.build_var_keys(dev(d), dev(o))
    img = b.image(0)
    of = oracle.filter_add(ocfg, oracle.hash_var(d, o))
    assert (img.pages == of.pages()).all() and (img.slots == of.slots()[: of.num_indices]).all()
    rng = np.random.default_rng(1)
    P = 50000
    ranks = np.arange(1, n + 1, dtype=np.float64)
    p = ranks ** -0.99
    p /= p.sum()
    ids = rng.choice(n, size=P, p=p)
    lens = (o[ids + 1] - o[ids]).astype(np.int64)
    pos_bytes = [d[o[i]:o[i + 1]] for i in ids]
    neg_d, neg_o = K.var_keys(P // 10, seed=0xBADD)
    parts = pos_bytes + [neg_d[neg_o[i]:neg_o[i + 1]] for i in range(P // 10)]
    pb = np.concatenate(parts)
    po = np.zeros(len(parts) + 1, dtype=np.uint64)
    np.cumsum([x.size for x in parts], out=po[1:])
    found = torch.zeros(len(parts), dtype=torch.int64, device="cuda:0")
    b.probe_var_keys(dev(pb), dev(po), torch.zeros(len(parts), dtype=torch.int32, device="cuda:0"),
                     len(parts), found)
    torch.cuda.synchronize()
    got = found.cpu().numpy().view(np.uint64)
    assert (got == of.lookup_hashes(oracle.hash_var(pb, po))).all()
    assert (got[:P] & np.uint64(1)).all() and lens.min() >= 8


def test_probe_line_overflow_falls_back_to_image(oracle):
    """Clustered fingerprints overflow some 64-byte probe lines; those probes take the
    full-scan path on the image. Every probe must still equal the oracle's lookup."""
    rng = np.random.default_rng(11)
    for lis, fps, value, n in ((8, 26, 0, 200000), (10, 28, 5, 150000), (6, 24, 1, 70000)):
        cfg = E.routing_config_init(fingerprint_size=fps, log_index_size=lis)
        ocfg = oracle.make_config(fingerprint_size=fps, log_index_size=lis)
        lnb = max(int(n).bit_length() - 1, lis)
        rem = fps - lnb
        sh = 32 - fps  # hash -> fingerprint shift
        h = rng.integers(0, 1 << 32, size=n, dtype=np.uint64).astype(np.uint32)
        # 8 clusters of 150 distinct fingerprints in 4 adjacent buckets each
        k = 0
        for c in range(8):
            b0 = int(rng.integers(0, (1 << lnb) - 4))
            for j in range(150):
                fp = ((b0 + j % 4) << rem) | (j * 7919 % (1 << rem))
                h[k] = np.uint32((fp << sh) | (j & ((1 << sh) - 1)))
                k += 1
        b = E.FilterBatch(cfg, [n], [value])
        b.build_hashes(dev(h))
        img = b.image(0)
        of = oracle.filter_add(ocfg, h, value=value)
        assert (img.num_unique, img.num_pages) == (of.num_unique, of.num_pages), lis
        assert (img.pages == of.pages()).all(), lis
        P = 300000
        ph = rng.integers(0, 1 << 32, size=P, dtype=np.uint64).astype(np.uint32)
        ph[: P // 3] = h[rng.integers(0, n, size=P // 3)]
        ph[P // 3: P // 3 + k] = h[:k] ^ np.uint32(1 << sh)  # same buckets, other remainders
        found = torch.zeros(P, dtype=torch.int64, device="cuda:0")
        b.probe_hashes(dev(ph), torch.zeros(P, dtype=torch.int32, device="cuda:0"), P, found)
        torch.cuda.synchronize()
        got = found.cpu().numpy().view(np.uint64)
        want = of.lookup_hashes(ph)
        assert (got == want).all(), (lis, int((got != want).sum()))
        assert (got[: P // 3] >> np.uint64(value) & np.uint64(1)).all()


def expected_probe_lines(pages, slots, num_indices, IS, G, rvs):
    """numpy restatement of the device-only probe-line format (rf_kernels.hip, "probe
    lines"), cut from a filter image: per group of G buckets, bits [0,128) the group's slice
    of the unary encoding (zero padded; all ones = overflow), bits [128,512) its packed
    remainders."""
    bits = np.unpackbits(pages, bitorder="little")
    L = IS // G
    out = np.zeros((num_indices * L, 64), dtype=np.uint8)
    for i in range(num_indices):
        h = int(slots[i])
        c = int(pages[h]) | (int(pages[h + 1]) << 8)
        e0 = (h + 2) * 8
        enc = bits[e0: e0 + c + IS]
        ones = np.flatnonzero(enc)
        r0 = (h + 2 + (c + IS - 1) // 8 + 4) * 8
        for g in range(L):
            a = 0 if g == 0 else int(ones[g * G - 1]) + 1
            end = int(ones[g * G + G - 1]) + 1
            ne = end - a
            n, E = ne - G, a - g * G
            line = np.zeros(512, dtype=np.uint8)
            if ne > 128 or n * rvs > 384:
                line[:128] = 1
            else:
                line[:ne] = enc[a:end]
                line[128:128 + n * rvs] = bits[r0 + E * rvs: r0 + (E + n) * rvs]
            out[i * L + g] = np.packbits(line, bitorder="little")
    return out


def _check_lines(b, img, cfg_kw, value):
    lines = b.debug_lines()
    lis = cfg_kw.get("log_index_size", 8)
    fps = cfg_kw.get("fingerprint_size", 26)
    IS = 1 << lis
    lnb = max(int(img.num_fingerprints).bit_length() - 1, lis)
    rvs = fps - lnb + int(value).bit_length()
    G = img.num_indices * IS // lines.shape[0]
    assert G * lines.shape[0] == img.num_indices * IS and G & (G - 1) == 0
    want = expected_probe_lines(img.pages, img.slots, img.num_indices, IS, G, rvs)
    bad = np.nonzero((lines != want).any(axis=1))[0]
    assert bad.size == 0, f"{bad.size} of {lines.shape[0]} lines differ, first {bad[:5]}"
    b.debug_rebuild_lines()  # the image-upload path re-cuts the same lines
    assert (b.debug_lines() == want).all()
    return G, float((want[:, :16] == 0xFF).all(axis=1).mean())


def test_probe_lines_match_numpy_restatement(oracle):
    """The device-only probe lines, byte for byte, against a numpy restatement cut from the
    (oracle-verified) image: fresh build, spill fallback + big buckets, clustered
    fingerprints (overflowed lines), incremental merge (64-bit entries)."""
    kw = {}
    b = E.FilterBatch(E.routing_config_init(), [300_000], [0])
    b.build_keys(dev(K.random_keys(300_000, seed=3)), 24)
    G, ovf = _check_lines(b, b.image(0), kw, 0)
    assert G >= 8 and ovf < 1e-3
    keys = K.ids_keys(np.arange(200_000, dtype=np.uint64) % 3)  # spill -> k_cb_sort_big
    b = E.FilterBatch(E.routing_config_init(), [200_000], [3])
    b.build_keys(dev(keys), 24)
    _check_lines(b, b.image(0), kw, 3)
    # clustered fingerprints: 150 in 4 adjacent buckets overflow their line
    rng = np.random.default_rng(2)
    n, rem, sh = 100_000, 26 - 16, 6
    h = rng.integers(0, 1 << 32, size=n, dtype=np.uint64).astype(np.uint32)
    for j in range(150):
        h[j] = np.uint32((((777 + j % 4) << rem) | (j * 7919 % (1 << rem))) << sh)
    b = E.FilterBatch(E.routing_config_init(), [n], [0])
    b.build_hashes(dev(h))
    _, ovf = _check_lines(b, b.image(0), kw, 0)
    assert ovf > 0
    kw9 = dict(log_index_size=9, fingerprint_size=28)
    cfg9 = E.routing_config_init(**kw9)
    b0 = E.FilterBatch(cfg9, [150_000], [1])
    b0.build_keys(dev(K.random_keys(150_000, seed=4)), 24)
    b1 = E.FilterBatch(cfg9, [200_000], [6], old=[(b0, 0)])
    b1.build_keys(dev(K.random_keys(200_000, seed=5)), 24)
    _check_lines(b1, b1.image(0), kw9, 6)


def test_errors_match_reference_contract():
    cfg = E.routing_config_init()
    with pytest.raises(E.PlatformStatusError) as ei:
        E.FilterBatch(cfg, [0])
    assert ei.value.code == E.STATUS_BAD_PARAM
    with pytest.raises(E.PlatformStatusError):
        E.FilterBatch(cfg, [E.routing_filter_max_fingerprints(cfg) + 1])
    with pytest.raises(E.PlatformStatusError):
        E.FilterBatch(cfg, [10], [200])  # fp_size + value_size > 32


@pytest.mark.parametrize("shift", [0, 5])
def test_var_keys_long_and_empty_wave_windows(oracle, shift):
    """Variable-length keys through the wave-staged LDS windows (partition: 8 KiB per wave,
    probe: 4 KiB per wave): empty and 1-15 B keys, and keys longer than either window
    (hashed straight from HBM), from a key buffer at an odd address. Image and every probe
    bit-exact against the oracle."""
    rng = np.random.default_rng(7 + shift)
    n = 40000
    lens = rng.integers(0, 101, size=n)
    lens[rng.random(n) < 0.05] = 0
    short = rng.random(n) < 0.05
    lens[short] = rng.integers(1, 16, size=int(short.sum()))
    long_ix = rng.choice(n, size=300, replace=False)
    lens[long_ix] = rng.integers(3000, 9500, size=300)
    lens[:3] = [9000, 0, 8180]  # the first keys of the first wave: over both windows
    offs = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum(lens, out=offs[1:])
    data = rng.integers(0, 256, size=int(offs[-1]), dtype=np.uint8)
    cfg = E.routing_config_init()
    ocfg = oracle.make_config()
    buf = dev(np.concatenate([np.zeros(shift, np.uint8), data, np.zeros(16, np.uint8)]))
    d_data = buf[shift:shift + data.size]
    b = E.FilterBatch(cfg, [n])
    b.build_var_keys(d_data, dev(offs))
    img = b.image(0)
    hv = oracle.hash_var(data, offs)
    of = oracle.filter_add(ocfg, hv)
    assert (img.pages == of.pages()).all() and (img.slots == of.slots()[: of.num_indices]).all()
    hout = torch.zeros(n, dtype=torch.int32, device="cuda:0")
    E.hash_var_keys(cfg, d_data, dev(offs), n, hout)
    torch.cuda.synchronize()
    assert (hout.cpu().numpy().view(np.uint32) == hv).all()
    found = torch.zeros(n, dtype=torch.int64, device="cuda:0")
    b.probe_var_keys(d_data, dev(offs), torch.zeros(n, dtype=torch.int32, device="cuda:0"), n, found)
    torch.cuda.synchronize()
    got = found.cpu().numpy().view(np.uint64)
    assert (got & np.uint64(1)).all()
    # negatives: the same lengths, other bytes
    data2 = rng.integers(0, 256, size=data.size, dtype=np.uint8)
    b.probe_var_keys(dev(data2), dev(offs), torch.zeros(n, dtype=torch.int32, device="cuda:0"), n, found)
    torch.cuda.synchronize()
    assert (found.cpu().numpy().view(np.uint64) == of.lookup_hashes(oracle.hash_var(data2, offs))).all()


def test_sparse_blocks_at_max_indices(oracle):
    """16,384 indices (8M-fingerprint geometry) holding a few thousand distinct fingerprints:
    nearly every block is an empty ~40 B encoding, ~100 blocks per page, so K5's next() runs
    (17 blocks per thread at this index count) each start inside a page much longer than the
    run and advance their pointer across it."""
    cfg = E.routing_config_init()
    ocfg = oracle.make_config()
    rng = np.random.default_rng(11)
    for distinct in (1, 2000, 60000):
        base = rng.integers(0, 1 << 32, size=distinct, dtype=np.uint64).astype(np.uint32)
        h = base[rng.integers(0, distinct, size=8_000_000)].astype(np.uint32)
        b = E.FilterBatch(cfg, [h.size], [5])
        b.build_hashes(dev(h))
        img = b.image(0)
        of = oracle.filter_add(ocfg, h, value=5)
        assert img.num_indices == 16384
        assert (img.num_unique, img.num_pages) == (of.num_unique, of.num_pages), distinct
        assert (img.pages == of.pages()).all(), distinct
        assert (img.slots == of.slots()[: of.num_indices]).all(), distinct


def _clustered_hashes(rng, n_rand, n_clu, lnb, fp_size=26, distinct=48):
    """n_rand uniform hashes + n_clu whose fingerprints all fall in ONE filter bucket, drawn
    from `distinct` remainders in random order: a bucket of thousands of copies of a few
    dozen entries (duplicates collapse in the dedupe, so the index block still fits a page)"""
    rem = fp_size - lnb
    bucket = int(rng.integers(0, 1 << lnb))
    rems = rng.choice(1 << rem, size=distinct, replace=False).astype(np.uint64)
    fp = (np.uint64(bucket) << np.uint64(rem)) | rems[rng.integers(0, distinct, size=n_clu)]
    low = rng.integers(0, 1 << (32 - fp_size), size=n_clu, dtype=np.uint64)
    clu = ((fp << np.uint64(32 - fp_size)) | low).astype(np.uint32)
    h = np.concatenate([rng.integers(0, 1 << 32, size=n_rand, dtype=np.uint64).astype(np.uint32), clu])
    return rng.permutation(h).astype(np.uint32)


@pytest.mark.parametrize("n_rand,n_clu", [(8000, 12000), (16000, 4000)])
def test_big_bucket_of_distinct_entries_sorts_fast(oracle, n_rand, n_clu):
    """One filter bucket holding 12,000 (resp. 4,000) copies of 48 entries in random order:
    the coarse bucket overflows LDS (K4b, 12,000) or stays in LDS (4,000). Such a bucket used
    to be ordered by a per-bucket insertion sort -- quadratic in the copies out of order,
    seconds at 12K; the whole workgroup now sorts it with an odd-even merge network.
    Bit-exact against the oracle, and fresh plus incremental builds finish in well under a
    second."""
    import time
    rng = np.random.default_rng(n_clu)
    cfg = E.routing_config_init()
    ocfg = oracle.make_config()
    n = n_rand + n_clu  # 20,000: log_num_buckets 14
    h = _clustered_hashes(rng, n_rand, n_clu, 14)
    b = E.FilterBatch(cfg, [n], [2])
    b.build_hashes(dev(h))  # warm: the kernels load once
    torch.cuda.synchronize()
    t = time.perf_counter()
    b.build_hashes(dev(h))
    torch.cuda.synchronize()
    dt = time.perf_counter() - t
    img = b.image(0)
    of = oracle.filter_add(ocfg, h, value=2)
    assert (img.num_unique, img.num_pages) == (of.num_unique, of.num_pages)
    assert (img.pages == of.pages()).all() and (img.slots == of.slots()[: of.num_indices]).all()
    assert dt < 0.2, dt
    # incremental: the new entries cluster in the same kind of bucket (only the new run is sorted)
    h2 = _clustered_hashes(rng, n_rand // 2, n_clu, 15)
    b2 = E.FilterBatch(cfg, [h2.size], [5], old=[(b, 0)])
    t = time.perf_counter()
    b2.build_hashes(dev(h2))
    torch.cuda.synchronize()
    dt2 = time.perf_counter() - t
    img2 = b2.image(0)
    of2 = oracle.filter_add(ocfg, h2, value=5, old=of)
    assert (img2.num_unique, img2.num_pages) == (of2.num_unique, of2.num_pages)
    assert (img2.pages == of2.pages()).all() and (img2.slots == of2.slots()[: of2.num_indices]).all()
    assert dt2 < 0.5, dt2
