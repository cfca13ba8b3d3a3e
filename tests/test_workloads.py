"""The vectorised 1000align lowering (reflow_amd.workloads.Dag1000) against the
oracle: CPU simulation of the job arrays (hole fill + SHA-256) must equal the
oracle digests of the same graph built as oracle flows.  The GPU run of the
same arrays is in test_gpu_dag.py."""
import hashlib

import numpy as np
import pytest

from reflow_amd.workloads import Dag1000, c2_sizes, arena_layout

PHYS = {"pR1": "R1", "pE1": "E1", "pE2": "E2", "pE3": "E3", "pES": "ES", "pXS": "XS"}


def simulate(a, inputs):
    """Evaluate the job arrays on the CPU: fill holes, hash (test checker)."""
    D = dict(inputs)
    n = len(a["out_slot"])
    pending = list(range(n))
    blob = a["blob"]
    while pending:
        nxt = []
        for j in pending:
            h0, h1 = int(a["hole_ptr"][j]), int(a["hole_ptr"][j + 1])
            slots = a["hole_slot"][h0:h1]
            if all(int(s) in D for s in slots):
                o, L = int(a["tmpl_off"][j]), int(a["tmpl_len"][j])
                m = bytearray(blob[o:o + L].tobytes())
                for h in range(h0, h1):
                    p = int(a["hole_pos"][h])
                    m[p:p + 32] = D[int(a["hole_slot"][h])]
                D[int(a["out_slot"][j])] = hashlib.sha256(bytes(m)).digest()
            else:
                nxt.append(j)
        assert len(nxt) < len(pending), "cycle"
        pending = nxt
    return D


@pytest.mark.parametrize("S,P", [(1, 1), (2, 3), (3, 4)])
def test_dag1000_lowering_matches_oracle(S, P):
    dag = Dag1000(S, P)
    a = dag.arrays()
    assert len(a["out_slot"]) == dag.n_jobs
    inputs = {int(s): dag.leaf_ids[i].tobytes() for i, s in enumerate(dag.file_slots)}
    D = simulate(a, inputs)
    T = dag.oflow()
    n_nodes = 0
    for name, nodes in T.items():
        if name in PHYS:
            continue
        for i, f in enumerate(nodes):
            assert D[int(dag.kinds[name].out_slot[i])] == f.digest(), (name, i)
            n_nodes += 1
    assert n_nodes == dag.n_nodes
    for pname, name in PHYS.items():
        for i, f in enumerate(T[name]):
            assert D[int(dag.kinds[pname].out_slot[i])] == f.physical_digest(), (pname, i)


def test_dag1000_change_set_and_counts():
    dag = Dag1000(20, 8)
    slots, old, new = dag.change_set(0.01)
    assert len(slots) == max(1, round(0.01 * 2 * 20 * 8))
    assert (old != new).any(axis=1).all()
    assert dag.n_nodes == 3 + 20 * (14 * 8 + 5)


def test_c2_sizes_distribution():
    GiB = 1 << 30
    lens = c2_sizes(total_bytes=64 * GiB)
    assert int(lens.sum()) == 64 * GiB
    assert lens.max() <= 2 * GiB and lens.min() >= 1
    big = lens >= (64 << 20)
    assert 0.01 < big.mean() < 0.03  # ~2% of files by count
    assert lens[big].sum() / lens.sum() > 0.9  # most bytes in the big files
    offs, total = arena_layout(lens)
    assert (offs % 256 == 0).all() and total >= int(lens.sum())


def _critical_path_dp(desc, changed):
    """Generic longest path, in blocks, over the jobs a change of `changed`
    slots dirties (creation order is a dependency order): each job counts its
    blocks after the constant leading ones (before its first hole)."""
    osl, tl, hp, hs, hpos = (desc[k] for k in ("out_slot", "tmpl_len", "hole_ptr", "hole_slot", "hole_pos"))
    path = {int(s): 0 for s in changed}
    best = 0
    for j in range(len(osl)):
        deps = [path[x] for x in hs[int(hp[j]):int(hp[j + 1])].tolist() if x in path]
        if deps:
            lead = int(hpos[int(hp[j])]) // 64
            path[int(osl[j])] = max(deps) + (int(tl[j]) + 9 + 63) // 64 - lead
            best = max(best, path[int(osl[j])])
    return best


def test_critical_path_matches_generic_dp():
    """bench.py's latency floor for the DAG legs (critical_path) == a generic
    longest-path DP over the dirtied jobs, for configs[2]'s shape and a piece
    of the strong-scaling layout (its Merge tree and global root)."""
    from reflow_amd.workloads import Dag1000, PartitionedDag1000
    d = Dag1000(40, 8)
    for frac in (0.01, 0.2):
        s, _, _ = d.change_set(frac)
        assert d.critical_path(s) == _critical_path_dp(d.arrays(), s)
    for nranks, rank in ((1, 0), (2, 0), (2, 1)):
        p = PartitionedDag1000(300, 8, nranks, rank, nparts=2)
        s, _, _ = p.dag.change_set(0.02, n_global=2 * 8 * 300 * 2)
        assert p.critical_path(s) == _critical_path_dp(p.desc, s) > d.critical_path(s)
