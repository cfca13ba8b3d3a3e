"""GPU parity of K2's memoized chaining values (GraphDev::memo_*, round 6).

A job's holes are written in a fixed order -- deps in Deps order
(/root/reference/flow.go:692-698), sorted paths (executor.go:214-233) -- so
after an input change the blocks before the job's first changed hole hash as
before.  A memo job (>= 8 blocks after its constant leading blocks, >= 2
holes) keeps the chaining value before each block, and the throughput form
resumes it at the first block a changed hole reaches.  These graphs hold
1000align-like wide jobs (32 holes at 34 i + 2: the per-sample OpK), one with
a constant prefix (midstate-trimmed) and holes straddling block boundaries,
one longer than 30 blocks (the queued word's block bits saturate at 30), and
a wide root over the wide jobs.  Each step is checked slot for slot against a
CPU evaluation (oracle SHA-256), the jobs hashed against the dirty closure,
and the blocks NOT hashed (rf_graph_memo_stats) against the exact expectation:
per memo job hashed in the throughput form with current stored values, the
first block its changed holes start in.  Changes in the first, a middle and
the last hole, two in one job (resume from the earlier), a latency-form step
(stored values then stale: hashed from block 0 next time), a full recompute
and a checkpoint restore (both: every stored value stale)."""
import random

import numpy as np
import pytest

import reflow_oracle as O

pytestmark = pytest.mark.gpu

MEMO_MIN = 8
NEVER = 2**64 - 1


@pytest.fixture(scope="module")
def ctx():
    from reflow_amd import capi
    c = capi.Context(0, host_threads=0)
    yield c
    c.close()


class Net:
    """Jobs in topological order: (out_slot, template, [(pos, slot)])."""

    def __init__(self, seed, n_wide=6):
        rng = random.Random(seed)
        self.jobs = []
        wide_specs = []
        for k in range(n_wide):
            if k == 4:  # constant prefix (3 trimmed blocks), holes every 40 B: some straddle blocks
                first, gap, nh = 200, 40, 24
            elif k == 5:  # longer than 30 blocks after trimming
                first, gap, nh = 2, 60, 40
            else:  # the per-sample OpK: U = "" then WD(dep_i) at 34 i + 2
                first, gap, nh = 2, 34, 32
            wide_specs.append((first, gap, nh))
        n_in = sum(nh for _, _, nh in wide_specs) * 2 + 8
        self.n_in = n_in
        inputs = list(range(n_in))
        cur = [0]

        def take():
            cur[0] += 1
            return inputs[cur[0] - 1]

        q_jobs = []  # level 0: two-hole jobs over two inputs
        self.wide_holes = []  # per wide job: [(pos, src slot, (input a, input b) or (input,))]
        for k, (first, gap, nh) in enumerate(wide_specs):
            holes = []
            for i in range(nh):
                pos = first + gap * i
                if i % 3 == 2:  # read an input directly (marked by the mark kernel)
                    a = take()
                    holes.append((pos, ("in", a), (a,)))
                else:
                    a, b = take(), take()
                    q_jobs.append((a, b))
                    holes.append((pos, ("q", len(q_jobs) - 1), (a, b)))
            self.wide_holes.append(holes)
        # slots: inputs, then q jobs, wide jobs, their single-hole consumers, root, root's consumer
        q_slot = [n_in + i for i in range(len(q_jobs))]
        base = n_in + len(q_jobs)
        wide_slot = [base + k for k in range(n_wide)]
        tail_slot = [base + n_wide + k for k in range(n_wide)]
        root_slot = base + 2 * n_wide
        root_tail = root_slot + 1
        self.n_slots = root_tail + 1
        rb = lambda n: bytes(rng.getrandbits(8) for _ in range(n))  # noqa: E731
        for i, (a, b) in enumerate(q_jobs):
            self.jobs.append((q_slot[i], rb(3) + bytes(32) + rb(5) + bytes(32) + rb(9), [(3, a), (40, b)]))
        self.wide_pos = []
        for k, holes in enumerate(self.wide_holes):
            first, gap, nh = wide_specs[k]
            end = holes[-1][0] + 32
            tlen = end + 37  # "OpK" + WD(FlowDigest)-sized suffix
            t = bytearray(rb(tlen))
            hl = []
            for pos, (kind, x), _ in holes:
                t[pos:pos + 32] = bytes(32)
                hl.append((pos, x if kind == "in" else q_slot[x]))
            self.jobs.append((wide_slot[k], bytes(t), hl))
            self.wide_pos.append([p for p, _, _ in holes])
        for k in range(n_wide):
            self.jobs.append((tail_slot[k], b"\x00\x05" + bytes(32) + rb(30), [(2, wide_slot[k])]))
        rt = bytearray(rb(34 * n_wide + 2 + 400))
        rh = []
        for k in range(n_wide):
            rt[34 * k + 2:34 * k + 34] = bytes(32)
            rh.append((34 * k + 2, wide_slot[k]))
        self.jobs.append((root_slot, bytes(rt), rh))
        self.jobs.append((root_tail, b"\x00\x05" + bytes(32), [(2, root_slot)]))
        self.wide_slot, self.root_slot, self.q_jobs = wide_slot, root_slot, q_jobs

    def evaluate(self, inputs):
        val = dict(enumerate(inputs))
        for out, tmpl, holes in self.jobs:
            m = bytearray(tmpl)
            for p, s in holes:
                m[p:p + 32] = val[s]
            val[out] = O.sha256(bytes(m))
        return val

    def load(self, ctx):
        from reflow_amd import capi
        blob, off, ln, hp, hpos, hslot = bytearray(), [], [], [0], [], []
        for out, tmpl, holes in self.jobs:
            off.append(len(blob))
            ln.append(len(tmpl))
            blob += tmpl
            for p, s in holes:
                hpos.append(p)
                hslot.append(s)
            hp.append(len(hpos))
        return capi.Graph(ctx, self.n_slots, np.array([o for o, _, _ in self.jobs], np.uint32),
                          np.array(off, np.uint64), np.array(ln, np.uint32), np.array(hp, np.uint64),
                          np.array(hpos, np.uint32), np.array(hslot, np.uint32), bytes(blob))


def memo_geometry(tmpl, holes):
    """(memo?, blocks after the constant lead, trimmed start block of each hole)."""
    nb = (len(tmpl) + 9 + 63) // 64
    lead = min(holes[0][0] // 64, nb - 1) if holes else 0
    nbt = nb - lead
    starts = [(p - 64 * lead) // 64 for p, _ in holes]
    return nbt >= MEMO_MIN and len(holes) >= 2, nbt, starts


def test_memo_resume_matches_cpu(ctx, tmp_path):
    from reflow_amd import capi
    net = Net(31)
    g = net.load(ctx)
    rng = random.Random(7)
    inputs = [bytes(rng.getrandbits(8) for _ in range(32)) for _ in range(net.n_in)]
    every = list(range(net.n_slots))
    g.set_slots(list(range(net.n_in)), np.frombuffer(b"".join(inputs), np.uint8))
    g.recompute(full=True)
    want = net.evaluate(inputs)
    got = g.get_slots(every)
    assert all(got[s].tobytes() == want[s] for s in every)
    geo = {out: memo_geometry(tmpl, holes) for out, tmpl, holes in net.jobs}
    n_memo = sum(1 for v in geo.values() if v[0])
    jobs0, entries0, skip0 = g.memo_stats()
    assert jobs0 == n_memo and entries0 == sum(v[1] - 1 for v in geo.values() if v[0])
    assert skip0 == 0
    valid = {out: False for out in geo}  # stored chaining values current (after a full recompute: none)
    state = {"g": g}

    def step(changes, form):
        """changes: {input slot: new value}; form 'lf' (memo) or 'pl'."""
        nonlocal inputs, want
        gg = state["g"]
        if form == "lf":
            gg.set_forms(0, 0, 0)
        else:
            gg.set_forms(NEVER, NEVER, NEVER)
        new = list(inputs)
        for s, v in changes.items():
            new[s] = v
        ch = sorted(changes)
        _, _, before = gg.memo_stats()
        gg.set_slots(ch, np.frombuffer(b"".join(new[s] for s in ch), np.uint8))
        n = gg.recompute(full=False)
        nxt = net.evaluate(new)
        got = gg.get_slots(every)
        bad = [s for s in every if got[s].tobytes() != nxt[s]]
        assert not bad, (form, bad[:10])
        # jobs hashed: every job with an input whose value changed; the
        # memo skip: per memo job hashed in the throughput form with current
        # stored values, the first block its changed holes start in
        changed = {s for s in range(net.n_in) if new[s] != inputs[s]}
        expect_jobs, expect_skip = 0, 0
        for out, tmpl, holes in net.jobs:
            hit = [i for i, (_, s) in enumerate(holes) if s in changed]
            if not hit:
                continue
            expect_jobs += 1
            memo, nbt, starts = geo[out]
            if memo:
                if form == "lf" and valid[out]:
                    expect_skip += min(min(min(starts[i], 30) for i in hit), nbt - 1)
                valid[out] = form == "lf"
            if nxt[out] != want[out]:
                changed.add(out)
        _, _, after = gg.memo_stats()
        assert n == expect_jobs, (form, n, expect_jobs)
        assert after - before == expect_skip, (form, after - before, expect_skip)
        inputs, want = new, nxt
        return expect_skip

    def bump(s):
        return O.sha256(inputs[s] + b"v%d" % rng.getrandbits(16))

    def src_inputs(k, i):
        return net.wide_holes[k][i][2]

    # every wide job hashed once in the throughput form: stored values current
    step({src_inputs(k, 1)[0]: bump(src_inputs(k, 1)[0]) for k in range(6)}, "lf")
    # first hole, a middle hole, the last hole, two holes (the earlier one
    # wins), the trimmed / straddling job, a hole past block 30
    ch = {}
    for k, i in ((0, 0), (1, 15), (2, 31), (3, 5), (3, 20), (4, 13), (5, 37)):
        a = src_inputs(k, i)[-1]
        ch[a] = bump(a)
    assert step(ch, "lf") > 0
    # an input change that re-sets the same value: nothing hashed for it
    a = src_inputs(0, 7)[0]
    step({a: inputs[a]}, "lf")
    # a latency-form step: the jobs it hashes keep no values
    ch = {src_inputs(k, 9)[0]: bump(src_inputs(k, 9)[0]) for k in (0, 2)}
    step(ch, "pl")
    ch = {src_inputs(k, 20)[-1]: bump(src_inputs(k, 20)[-1]) for k in (0, 1, 2)}
    step(ch, "lf")  # job 0 and 2 from block 0 (stale), job 1 resumes
    step({src_inputs(1, 25)[0]: bump(src_inputs(1, 25)[0]),
          src_inputs(0, 30)[0]: bump(src_inputs(0, 30)[0])}, "lf")
    # a full recompute: every stored value stale
    g.recompute(full=True)
    for k in valid:
        valid[k] = False
    step({src_inputs(0, 3)[0]: bump(src_inputs(0, 3)[0])}, "lf")
    step({src_inputs(0, 28)[0]: bump(src_inputs(0, 28)[0])}, "lf")
    # a checkpoint restore: the memo structures are rebuilt, values stale
    path = str(tmp_path / "memo.ckpt")
    g.save(path)
    g.close()
    r = capi.Graph.restore(ctx, path)
    state["g"] = r
    assert r.memo_stats()[:2] == (jobs0, entries0)
    for k in valid:
        valid[k] = False
    step({src_inputs(0, 28)[0]: bump(src_inputs(0, 28)[0])}, "lf")
    assert step({src_inputs(0, 31)[0]: bump(src_inputs(0, 31)[0])}, "lf") > 0
    r.close()
