"""Multi-process path on CPU (gloo, world_size 2): bench.py's sharding by
global system id plus its single collective (MAX time, SUM histograms) give
the same totals as one process over all systems. The per-rank engine here is
the CPU oracle (no GPU in this container); on the GPU box the same code runs
libdash over RCCL."""
import os
import socket

import numpy as np
import torch.multiprocessing as mp

import oracle_ctypes as oc

PER_RANK, LEN, SEED = 24, 48, 0xBEEF


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    import torch
    import torch.distributed as dist
    import bench
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    base, count = bench.shard(rank, world, PER_RANK)
    r = oc.run_batch(SEED, base, count, num_procs=8, cache_size=4, length=LEN, threads=1)
    counters = r["hist"].tolist() + [r["instructions"], int(r["rounds"].sum()),
                                     int((r["errors"] != 0).sum()), 0] + bench.digest_sum(r["digests"])
    elapsed, totals = bench.reduce_totals(float(rank + 1), counters, torch.device("cpu"), world)
    out[rank] = (elapsed, totals, r["digests"].tolist())
    dist.destroy_process_group()


def test_two_rank_shards_reduce_to_single_run():
    world = 2
    port = _free_port()
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_worker, args=(world, port, out), nprocs=world, join=True)
        res = dict(out)
    single = oc.run_batch(SEED, 0, PER_RANK * world, num_procs=8, cache_size=4, length=LEN, threads=2)
    import bench
    expect = single["hist"].tolist() + [single["instructions"], int(single["rounds"].sum()),
                                        int((single["errors"] != 0).sum()), 0] + bench.digest_sum(single["digests"])
    for rank in range(world):
        elapsed, totals, _ = res[rank]
        assert elapsed == float(world)  # MAX over ranks
        assert totals == expect
    digests = res[0][2] + res[1][2]
    assert digests == single["digests"].tolist()  # results independent of the GPU count


def _bench(*argv, env=None, timeout=180):
    import json
    import pathlib
    import subprocess
    import sys
    root = pathlib.Path(__file__).resolve().parent.parent
    e = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    e.update(env or {})
    r = subprocess.run([sys.executable, str(root / "bench.py"), *argv], capture_output=True, text=True,
                       timeout=timeout, env=e, cwd=root)
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    return r, (json.loads(lines[-1]) if lines else None)


def test_bench_launches_its_own_ranks():
    """`bench.py --gpus N` without torchrun starts N ranks itself (the driver's 1/2/4/8-GPU
    lines come from this same command form); each global system lands on exactly one rank."""
    r, d = _bench("--gpus", "2", "--dist-selftest", "--systems", "1000")
    assert r.returncode == 0, r.stderr[-2000:]
    # the group the ranks actually formed, and the per-rank spread (MIN / MAX all-reduce of rank + 1)
    assert d == {"world": 2, "systems_owned": 2000, "each_once": True, "local_rank": 0,
                 "rccl_world": 2, "backend": "gloo", "kernel_ms_rank": [1.0, 2.0]}
    r, d = _bench("--gpus", "4", "--dist-selftest", "--systems", "5")
    assert r.returncode == 0, r.stderr[-2000:]
    assert d["world"] == 4 and d["systems_owned"] == 20 and d["each_once"]
    assert d["rccl_world"] == 4 and d["kernel_ms_rank"] == [1.0, 4.0]
    assert len(r.stdout.encode()) <= 4096 and len(r.stderr.encode()) <= 1024, (len(r.stdout), r.stderr)


def test_bench_rejects_world_size_mismatch():
    r, d = _bench("--gpus", "1", "--dist-selftest", env={"WORLD_SIZE": "2", "RANK": "0"})
    assert r.returncode != 0 and d is None
    assert "must equal --gpus" in r.stderr
