"""The engine's lookup server (rf_amd_lookup_submit / _wait / _reap, k_lookup_server): single
lookups answered by a persistent wave that polls a ring of requests in device memory written
by the host through the BAR (or in pinned host memory, RF_AMD_SRV_RING=host). Every answer
must equal the batch probe's (k_probe) for the same filter and hash, through the waiting and
the reaping forms, from several threads at once, across the wave's idle exit and relaunch,
and after the batch's device memory was reused by another build while the wave kept running
(the wave must not answer from stale cached lines). The server runs with its default idle exit
(400 us) and lifetime (800 us) except where a test raises them through the host-controlled
keep-alive (rf_amd_lookup_server_set_times); a device-wide synchronisation taken while lookups
keep the server busy returns within about one lifetime."""
import ctypes
import os
import threading
import time

import numpy as np
import pytest
import torch

from splinterdb_amd import engine as E
from splinterdb_amd import keys as K

pytestmark = pytest.mark.gpu

# The server's CU-masked stream synchronises with the legacy null stream, so this module
# works on a non-blocking torch stream and synchronises that stream, never the device: a
# null-stream copy or torch.cuda.synchronize() would wait for the running wave to exit.
STREAM = None


def stream():
    global STREAM
    if STREAM is None:
        STREAM = torch.cuda.Stream()
    return STREAM


def sync():
    stream().synchronize()

L = None


def lib():
    global L
    if L is None:
        L = E.load_library()
    return L


def build(cfg, sizes, values, seed):
    """a batch of len(sizes) filters from random hashes; returns (batch, hashes, per-probe
    filter ids)"""
    rng = np.random.default_rng(seed)
    h = rng.integers(0, 1 << 32, size=sum(sizes), dtype=np.uint64).astype(np.uint32)
    with torch.cuda.stream(stream()):
        b = E.FilterBatch(cfg, sizes, values)
        b.build_hashes(torch.from_numpy(h.view(np.int32)).to("cuda:0"))
    sync()
    return b, h


def batch_probe(b, h, fid):
    """the reference answer: the batch probe kernel over the same (filter, hash) pairs"""
    with torch.cuda.stream(stream()):
        found = torch.zeros(h.size, dtype=torch.int64, device="cuda:0")
        b.probe_hashes(torch.from_numpy(h.view(np.int32)).to("cuda:0"),
                       torch.from_numpy(fid.astype(np.int32)).to("cuda:0"), h.size, found)
        sync()
        return found.cpu().numpy().view(np.uint64)


def submit(b, f, hash_, tag):
    t = ctypes.c_uint64()
    E._check(lib().rf_amd_lookup_submit(b.engine.h, b.h, int(f), int(hash_), tag, ctypes.byref(t)))
    return t.value


def wait(b, ticket):
    out = ctypes.c_uint64()
    E._check(lib().rf_amd_lookup_wait(b.engine.h, ticket, ctypes.byref(out)))
    return out.value


def reap_all(e, n, timeout_s=30.0):
    """reap n tagged answers: {tag: found}"""
    tags = (ctypes.c_void_p * 256)()
    found = (ctypes.c_uint64 * 256)()
    got = {}
    t0 = time.time()
    while len(got) < n:
        k = lib().rf_amd_lookup_reap(e.h, ctypes.addressof(tags), ctypes.addressof(found), 256)
        for i in range(k):
            got[tags[i]] = found[i]
        assert time.time() - t0 < timeout_s, f"reaped {len(got)} of {n}"
    return got


def probes(h, sizes, n, seed):
    """n (filter, hash) pairs: half inserted hashes, half random"""
    rng = np.random.default_rng(seed)
    starts = np.concatenate([[0], np.cumsum(sizes)])
    fid = rng.integers(0, len(sizes), size=n).astype(np.uint32)
    ph = rng.integers(0, 1 << 32, size=n, dtype=np.uint64).astype(np.uint32)
    hit = rng.random(n) < 0.5
    for i in np.nonzero(hit)[0]:
        ph[i] = h[starts[fid[i]] + rng.integers(0, sizes[fid[i]])]
    return fid, ph


def test_wait_and_reap_equal_batch_probe():
    cfg = E.routing_config_init(log_index_size=8)
    sizes, values = [200_000, 70_000, 3], [0, 9, 31]
    b, h = build(cfg, sizes, values, seed=1)
    fid, ph = probes(h, sizes, 6000, seed=2)
    want = batch_probe(b, ph, fid)
    # waiting form, one at a time
    got = np.array([wait(b, submit(b, fid[i], ph[i], None)) for i in range(1500)], dtype=np.uint64)
    assert (got == want[:1500]).all()
    # reaping form: 4,500 in flight at once (the 4,096-slot ring wraps while answers are reaped)
    e = b.engine
    res = {}
    done = threading.Event()

    def reaper():
        res.update(reap_all(e, 4500))
        done.set()

    th = threading.Thread(target=reaper)
    th.start()
    for i in range(1500, 6000):
        submit(b, fid[i], ph[i], i + 1)  # tag = index + 1 (never NULL)
    th.join(60)
    assert done.is_set()
    got = np.array([res[i + 1] for i in range(1500, 6000)], dtype=np.uint64)
    assert (got == want[1500:]).all()
    b.close(stream().cuda_stream)


def test_threads_idle_relaunch_and_reused_memory():
    cfg = E.routing_config_init(log_index_size=8)
    sizes = [100_000] * 4
    b, h = build(cfg, sizes, [1, 2, 3, 4], seed=3)
    fid, ph = probes(h, sizes, 8000, seed=4)
    want = batch_probe(b, ph, fid)
    # 8 threads waiting on their own lookups at once
    out = np.zeros(8000, dtype=np.uint64)

    def worker(t):
        for i in range(t, 8000, 8):
            out[i] = wait(b, submit(b, fid[i], ph[i], None))

    ths = [threading.Thread(target=worker, args=(t,)) for t in range(8)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(60)
    assert (out == want).all()
    # the wave exits after its idle time without requests (default 400 us); the next lookup
    # relaunches it and is answered
    st = (ctypes.c_uint64 * 3)()
    E._check(lib().rf_amd_lookup_server_stats(b.engine.h, st))
    launches0 = st[1]
    time.sleep(0.05)
    assert wait(b, submit(b, fid[0], ph[0], None)) == want[0]
    E._check(lib().rf_amd_lookup_server_stats(b.engine.h, st))
    assert st[1] > launches0
    # a keeper thread's lookups keep the wave busy (no idle exit) while the batch is replaced
    # by other builds in the same (pooled) device memory: the new batches' answers must not
    # come from lines the running wave cached before. The host-controlled keep-alive makes the
    # waves launched from here live long enough (5 s, 300 ms idle) to span a rebuild; the
    # next relaunch takes it (the current wave lives at most its default 800 us more).
    E._check(lib().rf_amd_lookup_server_set_times(b.engine.h, 300_000, 5_000_000))
    time.sleep(0.01)
    bk, hk = build(cfg, [5000], [0], seed=99)
    stop = threading.Event()
    kept = []

    def keeper():
        while not stop.is_set():
            kept.append(wait(bk, submit(bk, 0, hk[len(kept) % 5000], None)))

    kt = threading.Thread(target=keeper)
    kt.start()
    spanned = 0
    try:
        b.close(stream().cuda_stream)
        sync()
        for rnd in range(3):
            E._check(lib().rf_amd_lookup_server_stats(b.engine.h, st))
            l0 = st[1]
            b2, h2 = build(cfg, sizes, [5, 6, 7, 8], seed=10 + rnd)
            fid2, ph2 = probes(h2, sizes, 3000, seed=20 + rnd)
            want2 = batch_probe(b2, ph2, fid2)
            got2 = np.array([wait(b2, submit(b2, fid2[i], ph2[i], None)) for i in range(3000)], dtype=np.uint64)
            assert (got2 == want2).all(), rnd
            E._check(lib().rf_amd_lookup_server_stats(b.engine.h, st))
            spanned += st[1] == l0  # one wave served before and after this rebuild
            b2.close(stream().cuda_stream)
            sync()
    finally:
        stop.set()
        kt.join(30)
    assert spanned >= 1
    assert len(kept) > 100 and all(v & 1 for v in kept)  # every kept hash was inserted, value 0
    E._check(lib().rf_amd_lookup_server_set_times(b.engine.h, 400, 800))  # the defaults again
    stop_wave(b)
    bk.close(stream().cuda_stream)


def stop_wave(b):
    """lets a long-lived wave run out: one lookup after its idle time has passed relaunches a
    wave with the current (default) times"""
    time.sleep(0.35)
    bk, hk = build(E.routing_config_init(log_index_size=8), [100], [0], seed=5)
    wait(bk, submit(bk, 0, hk[0], None))
    bk.close(stream().cuda_stream)


def test_device_sync_while_server_busy_is_short():
    """hipDeviceSynchronize waits for every stream, the server's too: with the default 800-us
    lifetime it returns within about that long even while a thread keeps the server busy
    (up to 20 ms before)"""
    cfg = E.routing_config_init(log_index_size=8)
    b, h = build(cfg, [50_000], [0], seed=7)
    stop = threading.Event()
    n = [0]

    def keeper():
        while not stop.is_set():
            wait(b, submit(b, 0, h[n[0] % 50_000], None))
            n[0] += 1

    kt = threading.Thread(target=keeper)
    kt.start()
    try:
        time.sleep(0.05)
        ts = []
        for _ in range(30):
            t0 = time.perf_counter()
            torch.cuda.synchronize()  # device-wide
            ts.append(time.perf_counter() - t0)
            time.sleep(0.003)
    finally:
        stop.set()
        kt.join(30)
    ts.sort()
    assert n[0] > 100, n[0]
    # the median is the property (about one 800-us lifetime); the tail only bounds it loosely
    # (a scheduling hiccup on a shared box is not the server's lifetime)
    assert ts[len(ts) // 2] < 1.0e-3 and ts[-1] < 10 * 0.8e-3 + 5e-3, ts
    b.close(stream().cuda_stream)


def test_dead_server_returns_every_tag():
    """a server that dies while threads submit tagged lookups (the diagnostics hook
    stops its wave, then 2 ms later marks it dead, as a failed launch or a faulted stream marks
    it): every tag whose submit succeeded comes back exactly once, answered (rf_amd_lookup_reap)
    or with the error (rf_amd_lookup_server_failed) -- the tickets published in the gap, those
    published after `dead` was set and those of submitters that gave up waiting for a slot --
    and every later submit fails."""
    eng = E.Engine(0)  # a server killed for good: an engine of its own
    cfg = E.routing_config_init(log_index_size=8)
    rng = np.random.default_rng(11)
    h = rng.integers(0, 1 << 32, size=50_000, dtype=np.uint64).astype(np.uint32)
    with torch.cuda.stream(stream()):
        b = E.FilterBatch(cfg, [50_000], [0], engine=eng)
        b.build_hashes(torch.from_numpy(h.view(np.int32)).to("cuda:0"))
    sync()
    nth, per = 4, 3000
    ok = [[] for _ in range(nth)]
    refused = [0] * nth
    submitted = [0]
    done_submitting = threading.Event()
    lock = threading.Lock()

    def submitter(k):
        for i in range(per):
            tag = k * 100_000 + i + 1
            t = ctypes.c_uint64()
            rc = lib().rf_amd_lookup_submit(eng.h, b.h, 0, int(h[(k * per + i) % h.size]), tag, ctypes.byref(t))
            if rc == 0:
                ok[k].append(tag)
            else:
                refused[k] += 1
            with lock:
                submitted[0] += 1

    def killer():
        while submitted[0] < 2000:
            time.sleep(0.0002)
        E._check(lib().rf_amd_diag_lookup_server_kill(eng.h, 5, 2000))

    got = {}
    dup = []
    tags = (ctypes.c_void_p * 256)()
    found = (ctypes.c_uint64 * 256)()
    ths = [threading.Thread(target=submitter, args=(k,)) for k in range(nth)] + [threading.Thread(target=killer)]
    for t in ths:
        t.start()
    t0 = time.time()
    while True:
        k = lib().rf_amd_lookup_reap(eng.h, ctypes.addressof(tags), ctypes.addressof(found), 256)
        for i in range(k):
            if tags[i] in got:
                dup.append(tags[i])
            got[tags[i]] = "answered"
        if lib().rf_amd_lookup_server_error(eng.h):
            k = lib().rf_amd_lookup_server_failed(eng.h, ctypes.addressof(tags), 256)
            for i in range(k):
                if tags[i] in got:
                    dup.append(tags[i])
                got[tags[i]] = "failed"
        if not any(t.is_alive() for t in ths) and len(got) >= sum(len(o) for o in ok):
            break
        assert time.time() - t0 < 60, (len(got), sum(len(o) for o in ok))
    for t in ths:
        t.join(10)
    want = {t for o in ok for t in o}
    assert not dup
    assert set(got) == want
    assert sum(refused) > 0 and "failed" in got.values()
    assert lib().rf_amd_lookup_server_error(eng.h) == 5
    t = ctypes.c_uint64()
    assert lib().rf_amd_lookup_submit(eng.h, b.h, 0, 1, 1, ctypes.byref(t)) != 0
    b.close(stream().cuda_stream)
    sync()
    eng.close()


@pytest.mark.parametrize("placement", ["device", "host"])
def test_ring_placements_equal_batch_probe(placement, monkeypatch):
    """both request-ring placements (device memory written through the BAR: the default; pinned
    host memory: RF_AMD_SRV_RING=host) answer every lookup as the batch probe does, through the
    waiting and the reaping forms, on an engine of their own"""
    if placement == "host":
        monkeypatch.setenv("RF_AMD_SRV_RING", "host")
    else:
        monkeypatch.delenv("RF_AMD_SRV_RING", raising=False)
    eng = E.Engine(0)
    cfg = E.routing_config_init(log_index_size=8)
    sizes, values = [50_000, 20_000], [2, 7]
    rng = np.random.default_rng(11)
    h = rng.integers(0, 1 << 32, size=sum(sizes), dtype=np.uint64).astype(np.uint32)
    with torch.cuda.stream(stream()):
        b = E.FilterBatch(cfg, sizes, values, engine=eng)
        b.build_hashes(torch.from_numpy(h.view(np.int32)).to("cuda:0"))
    sync()
    fid, ph = probes(h, sizes, 3000, seed=12)
    want = batch_probe(b, ph, fid)
    got = np.array([wait(b, submit(b, fid[i], ph[i], None)) for i in range(500)], dtype=np.uint64)
    assert (got == want[:500]).all()
    lib().rf_amd_diag_lookup_ring.argtypes = [ctypes.c_void_p]
    assert lib().rf_amd_diag_lookup_ring(eng.h) == (1 if placement == "device" else 0)
    res = {}
    done = threading.Event()

    def reaper():
        res.update(reap_all(eng, 2500))
        done.set()

    th = threading.Thread(target=reaper)
    th.start()
    for i in range(500, 3000):
        submit(b, fid[i], ph[i], i + 1)
    th.join(60)
    assert done.is_set()
    got = np.array([res[i + 1] for i in range(500, 3000)], dtype=np.uint64)
    assert (got == want[500:]).all()
    b.close(stream().cuda_stream)
    eng.close()
