"""GPU parity at BASELINE's C3 and C4 shapes, batch reuse with different keys, and the
multi-rank launch path of bench.py.

Checkers, strongest first: the reference's own routing_filter.c (oracle/_ref/libref_rf.so,
built in the build container and shipped with the tree; see tests/test_ref_pinning.py),
the committed golden SHA-256s (tests/golden/sha256.json, equal to the reference's images),
and the oracle restatement where the reference library is absent.
"""
import hashlib
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import GOLD, ROOT
from oracle import refimpl as R
from splinterdb_amd import engine as E
from splinterdb_amd import keys as K

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
N20 = 1 << 20


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to("cuda:0")


@pytest.fixture(scope="module")
def ref():
    if not R.available():
        yield None
        return
    s = R.Stack()
    yield s
    assert s.device_writes() == 0
    s.close()


def gold():
    with open(os.path.join(GOLD, "sha256.json")) as fh:
        return json.load(fh)


def check_filter(b, f, keys_np, ref, oracle, ocfg, value=0, tag=""):
    """filter f of batch b == the reference's (or, without the library, the oracle's) build
    of the same keys, every page byte and slot"""
    img = b.image(f)
    if ref is not None:
        want = ref.image(ref.add(ref.hash_keys(keys_np), value=value))
    else:
        want = oracle.filter_add(ocfg, oracle.hash_fixed(keys_np.reshape(-1), 24), value=value)
        want.pages, want.slots = want.pages(), want.slots()[: want.num_indices]
    assert (img.num_unique, img.num_pages) == (want.num_unique, want.num_pages), tag
    assert img.pages.size == want.pages.size and (img.pages == want.pages).all(), tag
    assert (img.slots == want.slots).all(), tag
    return img


def sha_check(b, F_first, F, n, g):
    """every filter of the batch with a golden SHA (filter k of the n-key layout)"""
    seen = 0
    for f in range(F):
        key = f"seq_n{n}_lis8_k{F_first + f}"
        if key in g:
            img = b.image(f)
            assert hashlib.sha256(img.pages.tobytes()).hexdigest() == g[key]["pages_sha256"], key
            assert hashlib.sha256(img.slots.tobytes()).hexdigest() == g[key]["slots_sha256"], key
            seen += 1
    return seen


def probe_sample_check(b, f, n, keys_dev_all, ref, oracle, ocfg, count=20000):
    """count probes of filter f's own keys plus as many never-inserted keys, against the
    reference's routing_filter_lookup (or the oracle's)"""
    pos = K.seq_keys(f * n, count)
    neg = K.seq_keys(1 << 40, count)
    probe = np.concatenate([pos, neg])
    found = torch.zeros(2 * count, dtype=torch.int64, device="cuda:0")
    b.probe_keys(dev(probe), 24, torch.full((2 * count,), f, dtype=torch.int32, device="cuda:0"), 2 * count, found)
    torch.cuda.synchronize()
    got = found.cpu().numpy().view(np.uint64)
    if ref is not None:
        d = ref.add(ref.hash_keys(K.seq_keys(f * n, n)))
        want = ref.lookup_keys(d, probe)
    else:
        of = oracle.filter_add(ocfg, oracle.hash_fixed(K.seq_keys(f * n, n).reshape(-1), 24))
        want = of.lookup_hashes(oracle.hash_fixed(probe.reshape(-1), 24))
    assert (got == want).all(), f
    assert (got[:count] & np.uint64(1)).all()


def test_c3_256_filters_one_batch(ref, oracle):
    """C3: 256 filters x 2^20 sequential-id keys (268,435,456 keys) in ONE batch: sampled
    images equal the reference's, the golden SHAs of filters 0/1/77/255 hold, every key
    finds its filter (full 2^28 probe grouped by filter), and probe samples of two filters
    equal the reference's lookups"""
    F, n = 256, N20
    cfg = E.routing_config_init()
    ocfg = oracle.make_config()
    keys = K.seq_keys_torch(0, F * n, 24, "cuda:0")
    b = E.FilterBatch(cfg, [n] * F)
    b.build_keys(keys, 24)
    for f in range(F):
        assert b.info(f).error == 0
    assert sha_check(b, 0, F, n, gold()) >= 4
    for f in (3, 200):
        check_filter(b, f, K.seq_keys(f * n, n), ref, oracle, ocfg, tag=f"c3 filter {f}")
    found = torch.zeros(F * n, dtype=torch.int64, device="cuda:0")
    b.probe_keys_runs(keys, 24, [n] * F, found)
    torch.cuda.synchronize()
    assert bool(((found & 1) == 1).all())
    del found
    for f in (5, 254):
        probe_sample_check(b, f, n, keys, ref, oracle, ocfg)


def test_c4_1024_filters_one_gpu(ref, oracle):
    """C4 on one GPU: 1024 filters x 2^20 = 2^30 keys in one batch; the 8 golden-SHA filters
    (0, 1, 77, 255, 256, 511, 768, 1023) and two full images against the reference; the full
    2^30-key probe finds every key"""
    F, n = 1024, N20
    cfg = E.routing_config_init()
    ocfg = oracle.make_config()
    keys = K.seq_keys_torch(0, F * n, 24, "cuda:0")
    b = E.FilterBatch(cfg, [n] * F)
    b.build_keys(keys, 24)
    assert sha_check(b, 0, F, n, gold()) == 8
    for f in (600, 1022):
        check_filter(b, f, K.seq_keys(f * n, n), ref, oracle, ocfg, tag=f"c4 filter {f}")
    found = torch.zeros(F * n, dtype=torch.int64, device="cuda:0")
    b.probe_keys_runs(keys, 24, [n] * F, found)
    torch.cuda.synchronize()
    assert bool(((found & 1) == 1).all())
    del found
    probe_sample_check(b, 1000, n, keys, ref, oracle, ocfg, count=10000)


@pytest.mark.parametrize("poison", [None, "165"])
def test_batch_rebuilt_with_different_keys(ref, oracle, poison, monkeypatch):
    """One batch built twice with different keys of the same sizes (the production reuse
    pattern): the second images carry nothing of the first -- with every work buffer and
    the page images filled with 0xA5 before the first build under RF_AMD_POISON."""
    if poison:
        monkeypatch.setenv("RF_AMD_POISON", poison)
    cfg = E.routing_config_init()
    ocfg = oracle.make_config()
    sizes, values = [300_000, 70_000, 1, 4096], [0, 3, 1, 9]
    total = sum(sizes)
    b = E.FilterBatch(cfg, sizes, values)
    for seed in (0x1111, 0x2222):
        keys = K.random_keys(total, seed=seed)
        b.build_keys(dev(keys), 24)
        s = 0
        for f, (n, v) in enumerate(zip(sizes, values)):
            check_filter(b, f, keys[s:s + n], ref, oracle, ocfg, value=v, tag=(seed, f))
            s += n


def _bench(args, env_extra, timeout=420):
    env = dict(os.environ, RF_BENCH_BACKEND="gloo", **env_extra)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, cwd=ROOT,
                       capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    return json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])


@pytest.mark.timeout(900)
@pytest.mark.parametrize("workload,filters", [("c4", 12), ("c2", 2)])
def test_bench_two_ranks_equal_one_process(tmp_path, workload, filters):
    """bench.py --gpus 2 (no torchrun in the environment: bench.py starts both ranks itself,
    here both on the one GPU with gloo for the timing collectives) builds the same filter
    images as one process building every filter: C4 strong (12 filters split 6 + 6), C2
    weak (2 filters per rank = 4 in all)."""
    n = 1 << 16
    common = ["--workload", workload, "--keys-per-filter", str(n), "--steps", "2", "--warmup", "1",
              "--no-cpu-baseline", "--no-e2e"]
    d2 = str(tmp_path / "two")
    d1 = str(tmp_path / "one")
    line2 = _bench(common + ["--gpus", "2", "--filters", str(filters), "--digest-out", d2], {})
    total = filters if workload == "c4" else 2 * filters
    line1 = _bench(common + ["--gpus", "1", "--filters", str(total), "--digest-out", d1], {})
    assert line2["n_gpus"] == 2 and line1["n_gpus"] == 1
    assert line2["verified"] and line1["verified"]
    two = {}
    for r in range(2):
        with open(f"{d2}.rank{r}") as fh:
            part = json.load(fh)
        assert part and not (set(part) & set(two))  # disjoint, contiguous key-range shards
        two.update(part)
    with open(f"{d1}.rank0") as fh:
        one = json.load(fh)
    assert len(one) == total and two == one


@pytest.mark.timeout(900)
def test_c5_full_shape_sampled_against_reference(ref):
    """BASELINE C5 at bench.py's shape: 8 filters x 2^21 variable-length (8-100 B) keys built
    in one batch from device-resident bytes, then bench.py's probe stream (K.c5_inputs:
    Zipf(0.99) positives + 10 % negatives, shuffled over the filters). Filters 0 and 5 must be
    byte-identical to the reference's own routing_filter_add of the same keys (its
    data_key_hash over the bytes), and 100k probes of each equal to its routing_filter_lookup."""
    if ref is None:
        pytest.skip("oracle/_ref/libref_rf.so not built")
    F, n = 8, 1 << 21
    w = K.c5_inputs(F, n, seed=0x5EED)
    cfg = E.routing_config_init()
    b = E.FilterBatch(cfg, [n] * F)
    b.build_var_keys(dev(w["bytes"]), dev(w["offs"].view(np.int64)))
    P = int(w["probe_fid"].size)
    found = torch.empty(P, dtype=torch.int64, device="cuda:0")
    b.probe_var_keys(dev(w["probe_bytes"]), dev(w["probe_offs"].view(np.int64)), dev(w["probe_fid"].view(np.int32)),
                     P, found)
    torch.cuda.synchronize()
    got = found.cpu().numpy().view(np.uint64)
    assert ((got[w["positive"]] & np.uint64(1)) == 1).all()
    offs = w["offs"]
    for f in (0, 5):
        lo, hi = int(offs[f * n]), int(offs[(f + 1) * n])
        desc = ref.add(ref.hash_var_keys(w["bytes"][lo:hi], offs[f * n:(f + 1) * n + 1] - np.uint64(lo)))
        ir, img = ref.image(desc), b.image(f)
        assert (img.num_unique, img.num_pages) == (ir.num_unique, ir.num_pages), f
        assert (img.pages == ir.pages).all() and (img.slots == ir.slots).all(), f
        sel = np.nonzero(w["probe_fid"] == f)[0][:100_000]
        pb, po = K.gather_var(w["probe_bytes"], w["probe_offs"], sel)
        assert (got[sel] == ref.lookup_var_keys(desc, pb, po)).all(), f
        ref.dec_ref(desc)
