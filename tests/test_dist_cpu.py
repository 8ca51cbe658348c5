"""The N>1 plumbing of bench.py on the CPU (gloo, world 2 and 4, one process per rank as torchrun
starts them): bench.Dist's barrier / max-over-ranks / gather, the contiguous name-rank shard split
(ksim.ingest.Cluster.shard, ShardedScheduler's [r*n/world, (r+1)*n/world)) and merge_sharded, and the
C5 scenario split (rank r takes a contiguous share, no collective on the data path) — each rank
schedules its share on the C oracle and the gathered result equals one process doing everything."""
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _worker(rank, world, port, out_dir):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "kubernetes-schedule-simulator_amd"), os.path.join(ROOT, "oracle")]
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    import torch.distributed as dist
    import cpu_ref
    from ksim import scheduler, synth
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench

    class A:  # the Dist wrapper's view of the parsed arguments
        one_device = True
    D = bench.Dist.__new__(bench.Dist)
    D.torch = __import__("torch")
    D.world, D.rank, D.local, D.one, D.dist = world, rank, rank, True, dist
    # C5-style scenario split: contiguous shares, each scheduled independently
    cl, preds, scen = synth.config_c5(600, 300, seed=7)
    scen = scen[:24]
    lo, hi = rank * len(scen) // world, (rank + 1) * len(scen) // world
    mine = [cpu_ref.run(cl, scheduler.make_config(preds, s), 0, 300, threads=1)[0] for s in scen[lo:hi]]
    allv = D.gather(np.stack(mine) if mine else np.zeros((0, 300), np.int32))
    # node-shard split of one cluster: every rank's slice of the C oracle's node state
    cl3, p, q = synth.config_c3(1000, 400, seed=3)
    n = cl3.n_nodes
    a, b = rank * n // world, (rank + 1) * n // world
    sub = cl3.shard(a, b)
    ref, _, st, _ = cpu_ref.run(cl3, scheduler.make_config(p, q), 0, 400, threads=1)
    out = np.where((ref >= a) & (ref < b), ref, np.where(ref < 0, -1, -2)).astype(np.int32)  # ksim_schedule's -2
    outs = D.gather(out)
    mx = D.allmax(float(rank + 1))
    # sharded FitError histograms: each rank's shard histogram, summed across the ranks by an
    # all_reduce(SUM) between processes equals merge_sharded_reasons of the gathered ones
    import torch
    hist = np.random.default_rng(100 + rank).integers(0, 50, size=(7, 16)).astype(np.int32)
    t = torch.from_numpy(hist.astype(np.int64))
    dist.all_reduce(t)
    hists = D.gather(hist)
    D.barrier()
    if rank == 0:
        np.savez(os.path.join(out_dir, "res.npz"), scen=np.concatenate(allv), merged=scheduler.merge_sharded(outs),
                 ref=ref, mx=mx, sub_n=sub.n_nodes, hsum=t.numpy(),
                 hmerge=scheduler.merge_sharded_reasons(hists))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_dist_split_and_merge_gloo(world, tmp_path):
    import torch.multiprocessing as mp
    import cpu_ref
    from ksim import scheduler, synth
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    mp.start_processes(_worker, args=(world, port, str(tmp_path)), nprocs=world, join=True, start_method="spawn")
    r = np.load(tmp_path / "res.npz")
    cl, preds, scen = synth.config_c5(600, 300, seed=7)
    want = np.stack([cpu_ref.run(cl, scheduler.make_config(preds, s), 0, 300, threads=1)[0] for s in scen[:24]])
    assert np.array_equal(r["scen"], want)
    assert np.array_equal(r["merged"], r["ref"])
    assert float(r["mx"]) == world
    assert np.array_equal(r["hsum"], r["hmerge"])  # sharded FitError histograms: all_reduce == merge
