"""N > 1 path on CPU: two gloo ranks each process their own shard (the
bench's rank-local seeds), reduce counters and elapsed time; the sums equal
a single process over both shards. The per-rank compute here is the oracle
(no GPU in this test); the GPU pipeline per rank is covered by the gpu
tests, which are rank-independent."""
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

WORKER = r"""
import os, sys, json
import numpy as np
sys.path.insert(0, os.path.join(ROOT, "ghost-dataplane_amd")); sys.path.insert(0, os.path.join(ROOT, "oracle"))
import copgpu as cg, copdist, oracle as orc
rank, world, local = copdist.env()
g = copdist.Group(rank, world, "gloo")
fw = cg.gen_rules(0x5EED1004, 1000, cg.GEN_FW, 20)
lpm = orc.OracleLpm(1024, 24); lpm.setup(fw["ip"], fw["depth"], fw["next_hop"])
pk = cg.gen_trace(copdist.shard_seed(0x5EED0004, rank), 20000, fw)
hits = np.zeros(lpm.n_rules, np.uint64)
res, fwd, cnt = orc.process(pk, 20000, stages=3, fw=lpm, rule_hits=hits)
names = sorted(cnt)
tot = g.sum_u64(np.array([cnt[k] for k in names], dtype=np.uint64))
htot = g.sum_u64(hits)   # per-rule counters: same layout on every rank
uid = g.broadcast_bytes(bytes(range(128)) if rank == 0 else None)   # RCCL id distribution
assert uid == bytes(range(128)), uid
g.barrier()
mx = g.max(float(rank + 1))
mn = g.min(float(rank + 1))   # bench.py: per-GPU spread of the kernel rate
sm = g.sum(float(rank + 1.5))  # bench.py: node-wide achieved GB/s
if rank == 0:
    print(json.dumps({"names": names, "sum": [int(x) for x in tot], "max": mx, "min": mn, "fsum": sm,
                      "hits": [int(x) for x in htot]}))
g.close()
"""


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_rank_gloo_shards_and_reductions():
    port = free_port()
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, "-c", f"ROOT={ROOT!r}\n" + WORKER], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    outs = [p.communicate(timeout=240) for p in procs]
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 0, e
    import json

    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "ghost-dataplane_amd"))
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import copdist
    import copgpu as cg
    import oracle as orc
    got = json.loads(outs[0][0].strip().splitlines()[-1])
    assert got["max"] == 2.0 and got["min"] == 1.0 and got["fsum"] == 4.0
    fw = cg.gen_rules(0x5EED1004, 1000, cg.GEN_FW, 20)
    lpm = orc.OracleLpm(1024, 24)
    lpm.setup(fw["ip"], fw["depth"], fw["next_hop"])
    want = np.zeros(len(got["names"]), dtype=np.int64)
    whits = np.zeros(lpm.n_rules, np.uint64)
    for r in range(2):
        pk = cg.gen_trace(copdist.shard_seed(0x5EED0004, r), 20000, fw)
        _, _, cnt = orc.process(pk, 20000, stages=3, fw=lpm, rule_hits=whits)
        want += np.array([cnt[k] for k in got["names"]])
    assert list(want) == got["sum"]
    assert [int(x) for x in whits] == got["hits"] and whits.sum() > 0
    assert want[got["names"].index("rx")] == 40000
