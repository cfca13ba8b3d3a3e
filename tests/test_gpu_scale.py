"""Full-size GPU checks of BASELINE.json's configs, through size-independent
properties plus oracle samples (configs[1] in full is in test_gpu_hybrid.py,
against its committed fixture):

  configs[2]  10M-node 1000align DAG (S = 22075, P = 32), 1% of leaf File IDs
              changed: the incremental recompute equals a full recompute slot
              for slot, hashes exactly the oracle's dirty-job count
              (oracle/oracle.c orc_graph_update on the same arrays), and the
              changed slots' digests equal the oracle's.
  configs[4]  1e8-key bloomlive filter, 1e9 probes (half inserted keys): no
              false negative, false-positive rate at the filter's design
              point, and a 1e6-probe sample bit-exact against the oracle's
              Contains over the device's own words.
"""
import numpy as np
import pytest

import reflow_oracle as O
from reflow_amd import capi
from reflow_amd.workloads import Dag1000

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = capi.Context(0, host_threads=0)
    yield c
    c.close()


def test_configs2_incremental_full_size(ctx):
    dag = Dag1000(22075, 32)
    assert dag.n_nodes > 9_900_000
    a = dag.arrays()
    g = capi.Graph(ctx, a["n_slots"], a["out_slot"], a["tmpl_off"], a["tmpl_len"], a["hole_ptr"],
                   a["hole_pos"], a["hole_slot"], a["blob"])
    g.set_slots(dag.file_slots, dag.leaf_ids)
    g.recompute(full=True)
    slots, old, new = dag.change_set(0.01)
    g.set_slots(slots, new)
    n_inc = g.recompute(full=False)
    all_slots = np.arange(a["n_slots"], dtype=np.uint32)
    inc = g.get_slots(all_slots)
    g.recompute(full=True)
    full = g.get_slots(all_slots)
    assert (inc == full).all(), "incremental != full recompute"
    # the oracle's dirty closure on the same arrays and change set
    og = O.OGraph(a)
    og.set_inputs(dag.file_slots, dag.leaf_ids)
    og.full()
    n_ref = og.update(slots, new)
    assert n_inc == n_ref, (n_inc, n_ref)
    # digests of the jobs the change reached (the pair chains' outputs and
    # the per-sample roots) equal the oracle's
    roots = dag.kinds["XS"].out_slot
    assert (og.slots[roots] == inc[roots]).all()
    assert (og.slots[:a["n_slots"]] == inc).all()
    # and back: restoring the old IDs restores the original digests
    g.set_slots(slots, old)
    g.recompute(full=False)
    og.update(slots, old)
    assert (g.get_slots(roots) == og.slots[roots]).all()
    og.close()
    g.close()


def test_configs4_probe_full_size(ctx):
    n_ins, n_probe = 100_000_000, 1_000_000_000
    m, k = O.estimate_parameters(n_ins, 0.001)
    half = n_probe // 2
    keys = ctx.alloc(32 * n_probe)
    lens = np.array([32 * n_ins, 32 * (n_probe - half)], dtype=np.uint64)
    offs = np.array([0, 32 * half], dtype=np.uint64)
    d_offs, d_lens = ctx.upload(offs), ctx.upload(lens)
    ctx.gen_fill(keys.ptr, d_offs.ptr, d_lens.ptr, 2, 0x5EED0005, 32 * n_probe)
    ctx.sync()
    for r in range(1, half // n_ins):
        capi._check(capi.lib().rf_memcpy_d2d(ctx.handle, keys.ptr + 32 * n_ins * r, keys.ptr, 32 * n_ins))
    b = capi.Bloom.new(ctx, m, k)
    b.add_device(keys.ptr, n_ins, ctx.stream)
    out = ctx.alloc(n_probe)
    b.probe_device(keys.ptr, n_probe, out.ptr, ctx.stream)
    res = out.to_numpy()
    present = (half // n_ins) * n_ins
    assert res[:present].all(), "false negative"
    fp = int(res[present:].astype(np.int64).sum()) / (n_probe - present)
    assert 0.0007 < fp < 0.0013, fp  # p = 0.001 by construction (bloom.go:120-124)
    # 1e6 probes bit-exact against the oracle over the device's own words
    words = b.words()
    _, _, length, _ = b.params()
    idx = np.concatenate([np.arange(0, 500_000), np.arange(present, present + 500_000)])
    sample = np.zeros(32 * len(idx), dtype=np.uint8)
    for j, row in enumerate((0, present)):  # the two sample windows only (not 32 GB)
        capi._check(capi.lib().rf_memcpy_d2h(ctx.handle, sample.ctypes.data + 16_000_000 * j,
                                             keys.ptr + 32 * row, 16_000_000))
    want = np.zeros(len(idx), dtype=np.uint8)
    O.lib().orc_bloomlive_contains_batch(words.ctypes.data, length, m, k, sample.ctypes.data, len(idx),
                                         want.ctypes.data, 16)
    assert (res[idx] == want).all()
    for x in (keys, d_offs, d_lens, out):
        x.free()
    b.close()
