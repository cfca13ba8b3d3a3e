"""GPU parity of K2's fused chains and material cursor on raw job graphs.

The 1000align graphs place every single-input job's hole at byte 2; these
random graphs put holes anywhere (block 0, straddling a block boundary, deep
in a long template), mix single-hole jobs (fusion targets, k2_level_pc) with
multi-hole ones, give one producer several single-hole consumers (only one
can be fused, the others are queued), and re-set some inputs to their old
value (early cut-off must stop the chain).  Checked against a CPU evaluation
of the same jobs (oracle SHA-256), slot for slot, and the number of jobs hashed
against the exact dirty closure."""
import random

import numpy as np
import pytest

import reflow_oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    from reflow_amd import capi
    c = capi.Context(0, host_threads=0)
    yield c
    c.close()


def random_jobs(seed, n_in=64, n_jobs=1500):
    """Jobs in topological order: (out_slot, template bytes, [(pos, slot)])."""
    rng = random.Random(seed)
    produced = list(range(n_in))  # slots readable so far
    jobs = []
    for j in range(n_jobs):
        out = n_in + j
        r = rng.random()
        if r < 0.55:  # single hole: a fusion candidate
            nh = 1
        elif r < 0.85:
            nh = rng.randint(2, 4)
        else:
            nh = rng.randint(5, 12)
        # holes >= 32 B apart, anywhere: pick gaps
        pos, holes = rng.choice([0, 1, 2, 3, 30, 31, 32, 33, 58, 62, 63, 64, 65, 90, 127]), []
        for _ in range(nh):
            # prefer recent producers so chains form
            src = produced[-1 - min(int(rng.expovariate(0.3)), len(produced) - 1)] if rng.random() < 0.8 \
                else rng.choice(produced)
            holes.append((pos, src))
            pos += 32 + rng.choice([0, 0, 1, 2, 5, 17, 40])
        tlen = pos + rng.choice([0, 1, 9, 23, 55, 56, 64, 100, 200])
        tmpl = bytes(rng.getrandbits(8) for _ in range(tlen))
        jobs.append((out, tmpl, holes))
        produced.append(out)
    return jobs


def evaluate(n_in, jobs, inputs):
    val = dict(enumerate(inputs))
    for out, tmpl, holes in jobs:
        m = bytearray(tmpl)
        for p, s in holes:
            m[p:p + 32] = val[s]
        val[out] = O.sha256(bytes(m))
    return val


def load(ctx, n_in, jobs):
    from reflow_amd import capi
    blob, off, ln, hp, hpos, hslot = bytearray(), [], [], [0], [], []
    for out, tmpl, holes in jobs:
        off.append(len(blob))
        ln.append(len(tmpl))
        blob += tmpl
        for p, s in holes:
            hpos.append(p)
            hslot.append(s)
        hp.append(len(hpos))
    return capi.Graph(ctx, n_in + len(jobs), np.array([o for o, _, _ in jobs], np.uint32),
                      np.array(off, np.uint64), np.array(ln, np.uint32), np.array(hp, np.uint64),
                      np.array(hpos, np.uint32), np.array(hslot, np.uint32), bytes(blob))


@pytest.mark.parametrize("seed", [21, 22, 23])
def test_fused_chains_match_cpu(ctx, seed):
    n_in = 64
    jobs = random_jobs(seed, n_in)
    rng = random.Random(seed * 7)
    inputs = [bytes(rng.getrandbits(8) for _ in range(32)) for _ in range(n_in)]
    g = load(ctx, n_in, jobs)
    slots = list(range(n_in + len(jobs)))
    g.set_slots(list(range(n_in)), np.frombuffer(b"".join(inputs), np.uint8))
    g.recompute(full=True)
    want = evaluate(n_in, jobs, inputs)
    got = g.get_slots(slots)
    assert all(got[s].tobytes() == want[s] for s in slots)
    for rnd in range(4):
        ch = rng.sample(range(n_in), 6)
        new = list(inputs)
        for k, s in enumerate(ch):
            # every other change re-sets the same value: nothing may be rehashed for it
            if k % 2 == 0:
                new[s] = O.sha256(inputs[s] + b"v2")
        g.set_slots(ch, np.frombuffer(b"".join(new[s] for s in ch), np.uint8))
        n = g.recompute(full=False)
        nxt = evaluate(n_in, jobs, new)
        got = g.get_slots(slots)
        bad = [s for s in slots if got[s].tobytes() != nxt[s]]
        assert not bad, (rnd, bad[:10])
        # jobs hashed == jobs with an input whose value changed (cut-off included)
        changed = {s for s in range(n_in) if new[s] != inputs[s]}
        expect = 0
        for out, _, holes in jobs:
            if any(s in changed for _, s in holes):
                expect += 1
                if nxt[out] != want[out]:
                    changed.add(out)
        assert n == expect, (rnd, n, expect)
        inputs, want = new, nxt
