"""Compaction chains on the GPU: incremental routing_filter_add rounds with stream-ordered
release of the superseded batch (rf_amd_batch_destroy_on), stream-scoped infos and
read-back on a copy stream -- the pattern bench.py --workload compaction times.

Checkers: the reference's own chain (oracle/_ref/libref_rf.so: routing_filter_add with the
previous filter as old_filter, tests/functional/filter_test.c:53-82) round by round, and the
golden SHA-256s of full 8 x (2^20-1) chains the reference built (tests/golden/sha256.json
chain_*, oracle/gen_golden.py gen_chain_sha).
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT
from oracle import refimpl as R
from splinterdb_amd import engine as E
from splinterdb_amd import keys as K

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def chain_ids(g, v, n):
    return (np.uint64(g) << np.uint64(32)) + np.uint64(v + 1) * np.arange(n, dtype=np.uint64)


@pytest.mark.skipif(not R.available(), reason="reference library not built")
@pytest.mark.parametrize("entries", ["flag32", "flag32_decode", "wide64"])
def test_chain_rounds_match_reference(entries, monkeypatch):
    """both incremental pipelines: 32-bit flagged entries (fp_size + value_size <= 31, the
    default) and 64-bit entries (forced here). With 32-bit entries a round whose geometry is
    the previous round's (rounds 3 and 5: 40K -> 60K, 80K -> 100K fingerprints) reads the old
    entries in place from the previous batch; the others decode the old image
    (flag32_decode forces the decode for every round)"""
    if entries == "wide64":
        monkeypatch.setenv("RF_AMD_WIDE64", "1")
    if entries == "flag32_decode":
        monkeypatch.setenv("RF_AMD_OLD_DECODE", "1")
    F, V, n = 3, 5, 20000
    cfg = E.routing_config_init(fingerprint_size=26, log_index_size=8, seed=42)
    eng = E.Engine(0)
    stream, copy = torch.cuda.Stream(), torch.cuda.Stream()
    st = stream.cuda_stream
    keys = [np.concatenate([K.ids_keys(chain_ids(g, v, n)) for g in range(F)]) for v in range(V)]
    dkeys = [torch.from_numpy(k.reshape(-1)).to("cuda:0") for k in keys]
    torch.cuda.synchronize()
    hp = [torch.empty(4096 * 512, dtype=torch.uint8).pin_memory() for _ in range(F)]
    hs = [torch.empty(2048, dtype=torch.int64).pin_memory() for _ in range(F)]
    with R.Stack() as ref:
        rprev = [None] * F
        prev = None
        for v in range(V):
            b = E.FilterBatch(cfg, [n] * F, [v] * F, old=[(prev, f) for f in range(F)] if prev else None,
                              engine=eng)
            b.build_keys(dkeys[v], 24, stream=st)
            if prev is not None:
                stream.wait_stream(copy)
                prev.close(stream=st)  # stream-ordered: no device synchronisation
            inf = b.infos(stream=st)
            copy.wait_stream(stream)
            for f in range(F):
                b.read_image_async(f, hp[f][: inf[f].num_pages * 4096], hs[f][: inf[f].num_indices],
                                   copy.cuda_stream)
            copy.synchronize()
            for f in range(F):
                rf = ref.add(ref.hash_keys(keys[v][f * n:(f + 1) * n]), value=v, old=rprev[f])
                want = ref.image(rf)
                rprev[f] = rf
                assert inf[f].num_fingerprints == rf.num_fingerprints == (v + 1) * n
                assert inf[f].num_unique == rf.num_unique, (v, f)
                got = hp[f][: inf[f].num_pages * 4096].numpy()
                assert got.size == want.pages.size and (got == want.pages).all(), (v, f)
                assert (hs[f][: inf[f].num_indices].numpy().view(np.uint64) == want.slots).all(), (v, f)
            prev = b
        # lookups of every round's keys in the final filters (probe lines cut page by page
        # by K6 or by k_plines for the pages it flags) == the reference's routing_filter_lookup
        found = torch.empty(F * n, dtype=torch.int64, device="cuda:0")
        for v in range(V):
            prev.probe_keys_runs(dkeys[v], 24, [n] * F, found)
            got = found.cpu().numpy().view(np.uint64)
            for f in range(F):
                want = ref.lookup_keys(rprev[f], keys[v][f * n:(f + 1) * n])
                assert (got[f * n:(f + 1) * n] == want).all(), (v, f)
        prev.close()
        # the pool got the parked blocks back: a new batch of the same shape reuses them
        h0 = eng.pool_stats()["hits"]
        b = E.FilterBatch(cfg, [n] * F, engine=eng)
        b.close()
        assert eng.pool_stats()["hits"] > h0
    eng.close()


def _bench(args, timeout=600):
    env = dict(os.environ, RF_BENCH_BACKEND="gloo")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, cwd=ROOT,
                       capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    return json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])


@pytest.mark.timeout(900)
@pytest.mark.parametrize("gpus,filters", [(1, 2), (2, 1)])
def test_bench_compaction_full_chains_golden(gpus, filters):
    """full 8 x (2^20-1) chains through bench.py: every round's keys find their value in the
    final filters, and filters 0 and 1 equal the reference's chains byte for byte (filter 0
    is filter_test's basic chain: num_unique 4,254,486)"""
    line = _bench(["--workload", "compaction", "--gpus", str(gpus), "--filters", str(filters),
                   "--steps", "1", "--warmup", "0", "--no-cpu-baseline"])
    assert line["verified"], line
    assert line["n_gpus"] == gpus
    assert 0 in line["sha_checked_filters"]
    assert line["num_unique_filter0"] == 4254486
    assert len(line["round_wall_ms"]) == 8


@pytest.mark.skipif(not R.available(), reason="reference library not built")
def test_incremental_ties_and_duplicates():
    """an incremental add onto a filter of the same geometry (old entries read in place and
    merged with the sorted new ones in K4) whose new keys repeat old keys under the SAME
    value (equal old and new entries: the old one first, both kept, src/routing_filter.c
    :563-566) and repeat each other (new duplicates dropped, :473-482), over two rounds --
    byte-identical to the reference's chain, num_unique included"""
    cfg = E.routing_config_init(fingerprint_size=26, log_index_size=8, seed=42)
    eng = E.Engine(0)
    rng = np.random.default_rng(7)
    F = 2
    r0 = [rng.integers(0, 1 << 62, size=40000, dtype=np.uint64) for _ in range(F)]
    # round 1: 8,000 old keys again, 6,000 fresh keys each twice (20,000 keys, same value)
    r1 = []
    for f in range(F):
        fresh = rng.integers(0, 1 << 62, size=6000, dtype=np.uint64)
        r1.append(rng.permutation(np.concatenate([r0[f][:8000], fresh, fresh])))
    # round 2: 10,000 keys of rounds 0 and 1 again under another value
    r2 = [rng.permutation(np.concatenate([r0[f][8000:13000], r1[f][:5000]])) for f in range(F)]
    rounds = [(r0, 3), (r1, 3), (r2, 5)]
    with R.Stack() as ref:
        rprev = [None] * F
        prev = None
        for ids, val in rounds:
            n = ids[0].size
            keys = np.concatenate([K.ids_keys(ids[f]) for f in range(F)])
            dk = torch.from_numpy(keys.reshape(-1)).to("cuda:0")
            b = E.FilterBatch(cfg, [n] * F, [val] * F, old=[(prev, f) for f in range(F)] if prev else None,
                              engine=eng)
            b.build_keys(dk, 24)
            torch.cuda.synchronize()
            for f in range(F):
                rf = ref.add(ref.hash_keys(keys[f * n:(f + 1) * n]), value=val, old=rprev[f])
                want = ref.image(rf)
                img = b.image(f)
                assert (img.num_unique, img.num_pages) == (rf.num_unique, want.pages.size // 4096), (val, f)
                assert (img.pages == want.pages).all(), (val, f)
                assert (img.slots == want.slots).all(), (val, f)
                rprev[f] = rf
            if prev is not None:
                prev.close()
            prev = b
        for ids, _ in rounds:
            n = ids[0].size
            keys = np.concatenate([K.ids_keys(ids[f]) for f in range(F)])
            found = torch.empty(F * n, dtype=torch.int64, device="cuda:0")
            prev.probe_keys_runs(torch.from_numpy(keys.reshape(-1)).to("cuda:0"), 24, [n] * F, found)
            got = found.cpu().numpy().view(np.uint64)
            for f in range(F):
                assert (got[f * n:(f + 1) * n] == ref.lookup_keys(rprev[f], keys[f * n:(f + 1) * n])).all()
        prev.close()
    eng.close()
