"""The multi-rank code path on one GPU: torch.distributed over RCCL ("nccl") with ONE rank,
every collective run (not the one-rank shortcuts). ProbeRouter's all-to-alls (counts, probe
pairs, found_values back) and replicate_images' all-gathers (filter infos, pages, slots, then
an imported probe-only batch) through RCCL must give the single-process probe's results, and
bench.py's multi-rank path (process group, barriers, max/sum over ranks, routed probes) must
run and verify. Each check runs in a subprocess of its own (its process group, its port)."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


ROUTER = r"""
import os, sys
sys.path.insert(0, os.environ["RF_ROOT"])
import numpy as np, torch, torch.distributed as dist
from splinterdb_amd import engine as E, keys as K, route as R, shard as S
dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=dev)
assert dist.get_backend() == "nccl" and dist.get_world_size() == 1
cfg = E.routing_config_init(log_index_size=8)
F, n = 4, 60_000
keys = torch.from_numpy(K.random_keys(F * n, seed=3)).to(dev)
b = E.FilterBatch(cfg, [n] * F, [0, 1, 2, 3])
b.build_keys(keys, 24)
P = 100_000
rng = np.random.default_rng(1)
gfid = rng.integers(0, F, size=P).astype(np.int32)
pk = K.random_keys(P, seed=9)
own = rng.random(P) < 0.5
idx = rng.integers(0, n, size=P)
kk = K.random_keys(F * n, seed=3)
pk[own] = kk[gfid[own] * n + idx[own]]
d_pk = torch.from_numpy(pk).to(dev)
d_h = torch.empty(P, dtype=torch.int32, device=dev)
E.hash_keys(cfg, d_pk, 24, P, d_h)
d_f = torch.from_numpy(gfid).to(dev)
want = torch.zeros(P, dtype=torch.int64, device=dev)
b.probe_hashes(d_h, d_f, P, want)
router = R.ProbeRouter(S.plan_shards(F, n, 1), 0, b, dev, dist=dist, coll_device=dev, ops=R.GpuRouteOps(),
                       collective_at_one=True)
assert not router.local
got = torch.zeros(P, dtype=torch.int64, device=dev)
send, recv = router.lookup_hashes(d_h, d_f, P, got)
torch.cuda.synchronize()
assert send == recv == [P], (send, recv)
assert torch.equal(got, want), int((got != want).sum())
assert bool(((want >> torch.from_numpy(gfid.astype(np.int64)).to(dev)) & 1)[torch.from_numpy(own).to(dev)].all())
x = torch.ones(1, device=dev)
dist.all_reduce(x)
dist.barrier()
dist.destroy_process_group()
print("ROUTER_OK", P)
"""


REPLICA = r"""
import os, sys
sys.path.insert(0, os.environ["RF_ROOT"])
import numpy as np, torch, torch.distributed as dist
from splinterdb_amd import engine as E, keys as K, route as R
dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=dev)
assert dist.get_backend() == "nccl" and dist.get_world_size() == 1
cfg = E.routing_config_init(log_index_size=8)
F, n = 5, 40_000
kk = K.random_keys(F * n, seed=5)
b = E.FilterBatch(cfg, [n] * F, [f % 8 for f in range(F)])
b.build_keys(torch.from_numpy(kk).to(dev), 24)
rep = R.replicate_images(b, 1, dev, dist=dist, coll_device=dev, collective_at_one=True)
assert rep.F == F
P = 80_000
rng = np.random.default_rng(2)
gfid = rng.integers(0, F, size=P).astype(np.int32)
pk = K.random_keys(P, seed=17)
own = rng.random(P) < 0.5
idx = rng.integers(0, n, size=P)
pk[own] = kk[gfid[own] * n + idx[own]]
d_pk = torch.from_numpy(pk).to(dev)
d_f = torch.from_numpy(gfid).to(dev)
want = torch.zeros(P, dtype=torch.int64, device=dev)
got = torch.zeros(P, dtype=torch.int64, device=dev)
b.probe_keys(d_pk, 24, d_f, P, want)
rep.probe_keys(d_pk, 24, d_f, P, got)
torch.cuda.synchronize()
assert torch.equal(got, want), int((got != want).sum())
vals = torch.from_numpy((gfid % 8).astype(np.int64)).to(dev)
assert bool(((want >> vals) & 1)[torch.from_numpy(own).to(dev)].all())
for f in range(F):  # the imported images are the built ones, byte for byte
    a, r = b.image(f), rep.image(f)
    assert (a.pages == r.pages).all() and (a.slots == r.slots).all(), f
dist.barrier()
dist.destroy_process_group()
print("REPLICA_OK", P)
"""


def test_replicated_images_all_gather_over_rccl_one_rank():
    env = dict(os.environ, RF_ROOT=ROOT, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()), RANK="0",
               WORLD_SIZE="1", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, "-c", REPLICA], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and "REPLICA_OK" in r.stdout, (r.stdout[-2000:], r.stderr[-4000:])


def test_router_all_to_all_over_rccl_one_rank():
    env = dict(os.environ, RF_ROOT=ROOT, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()), RANK="0",
               WORLD_SIZE="1", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, "-c", ROUTER], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and "ROUTER_OK" in r.stdout, (r.stdout[-2000:], r.stderr[-4000:])


def test_bench_multi_rank_path_over_rccl_one_rank():
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--dist-always", "--filters", "2", "--keys-per-filter",
           "300000", "--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--no-e2e", "--routed-probe",
           "--pmc", "none"]
    env = dict(os.environ)
    for k in ("MASTER_PORT", "RANK", "WORLD_SIZE", "LOCAL_RANK"):
        env.pop(k, None)
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    line = [x for x in r.stdout.splitlines() if x.startswith("{")][-1]
    out = json.loads(line)
    assert out["verified"] is True and out["n_gpus"] == 1
    assert out["routed_probe"]["verified"] is True
    assert "RCCL" in out["routed_probe"]["exchange"], out["routed_probe"]
