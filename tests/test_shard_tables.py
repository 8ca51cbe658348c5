"""Node-sharded tables on the host (CPU only): a rank's affinity and volume tables over its
name-rank range [lo, hi) (ingest._shard_affinity, Cluster.shard) — the node pseudo key renumbered to
the shard with its counted pairs' / carried terms' segments sliced, every other key's domains and
counts unchanged, volume slots sliced — and the refusal of terms over shared domains.  The GPU
side (exchange and decisions) is tests/test_gpu_parity.py::test_node_sharded_c2x_multi_process."""
import numpy as np
import pytest

from ksim import abi, ingest, synth


@pytest.mark.parametrize("world", [2, 3])
def test_c2x_shard_tables_restrict_the_full_tables(world):
    cl, _, _, _ = synth.config_c2x(1200, 300, seed=4)
    d = cl.affinity
    n = cl.n_nodes
    for r in range(world):
        lo, hi = r * n // world, (r + 1) * n // world
        sub = cl.shard(lo, hi)
        a = sub.affinity
        assert a["n_nodes"] == hi - lo and a["dom"].shape == (d["dom"].shape[0], hi - lo)
        assert (a["dom"][1] == np.arange(hi - lo)).all()
        for k in range(2, d["dom"].shape[0]):
            assert (a["dom"][k] == d["dom"][k][lo:hi]).all()
        for c in range(int(d["n_pair"])):
            k = int(d["pair_key"][c])
            full = d["cnt"][d["pair_off"][c]:d["pair_off"][c] + int(d["n_dom"][k])]
            got = a["cnt"][a["pair_off"][c]:a["pair_off"][c] + int(a["n_dom"][k])]
            assert (got == (full[lo:hi] if k == 1 else full)).all(), c
        v = sub.volumes
        assert v["n_nodes"] == hi - lo
        assert (v["slot_count"] == cl.volumes["slot_count"][lo:hi]).all()
        assert (v["slots"] == cl.volumes["slots"][:, lo:hi]).all()


def test_shared_domain_terms_refused():
    """A preferred / required term on a zone-like key (a domain several ranks' nodes share) cannot
    be kept rank-local: refused rather than sharded."""
    from workloads import rnd_affinity_workload
    nodes, running, pods = rnd_affinity_workload(2, n_nodes=16, n_pods=40)
    cl = ingest.Cluster.from_objects(nodes, running, pods)
    with pytest.raises(abi.KsimUnsupported):
        cl.shard(0, 8)
