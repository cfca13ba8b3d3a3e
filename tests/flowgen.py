"""Seeded random Flow DAGs over every op the digest grammar distinguishes
(test/flow/constructor.go:17-74 shapes plus K/Coerce/Requirements/Data)."""
from __future__ import annotations

import random

from reflow_oracle import OFlow, OFileset, from_string


def rand_fileset(rng: random.Random, nfiles=None, prefix="f"):
    n = rng.randint(0, 4) if nfiles is None else nfiles
    m = {}
    for i in range(n):
        path = "%s%d/%s" % (prefix, rng.randint(0, 3), "x" * rng.randint(0, 9)) if i else "."
        m[path] = (bytes(rng.getrandbits(8) for _ in range(32)), rng.randint(0, 1 << 20))
    return OFileset(map=m)


def rand_value(rng):
    if rng.random() < 0.2:
        return OFileset(list=[rand_fileset(rng) for _ in range(rng.randint(0, 3))])
    return rand_fileset(rng)


def random_dag(seed: int, n: int = 60, universe_safe=True):
    """Returns (root, nodes).  Every node is reachable from root."""
    rng = random.Random(seed)
    nodes = []

    def pick(k):
        return [rng.choice(nodes) for _ in range(k)]

    for i in range(n):
        kind = rng.random() if nodes else 0.0
        if kind < 0.25 or len(nodes) < 3:
            leaf = rng.randint(0, 3)
            if leaf == 0:
                f = OFlow("OpIntern", url="s3://bucket/%d/%s" % (i, "p" * rng.randint(0, 40)))
            elif leaf == 1:
                f = OFlow("OpVal", value=rand_value(rng), done=True)
            elif leaf == 2:
                f = OFlow("OpData", data=bytes(rng.getrandbits(8) for _ in range(rng.randint(0, 90))))
            else:
                f = OFlow("OpVal", flow_digest=from_string("v%d" % i))
        else:
            op = rng.choice(["exec", "exec", "exec", "merge", "pullup", "k", "coerce", "groupby",
                             "collect", "map", "req", "extern"])
            if op == "exec":
                deps = pick(rng.randint(0, 5))
                am = None
                if rng.random() < 0.7:
                    am = [(rng.random() < 0.3, rng.randint(0, max(len(deps) - 1, 0)))
                          for _ in range(rng.randint(0, len(deps) + 1))]
                f = OFlow("OpExec", deps, image="img%d" % rng.randint(0, 5),
                          cmd="cmd %s" % ("z" * rng.randint(0, 120)), argmap=am,
                          done=rng.random() < 0.8, value=rand_value(rng))
            elif op == "merge":
                f = OFlow("OpMerge", pick(rng.randint(1, 6)))
            elif op == "pullup":
                f = OFlow("OpPullup", pick(rng.randint(1, 4)))
            elif op == "k":
                f = OFlow("OpK", pick(rng.randint(1, 40 if rng.random() < 0.1 else 4)),
                          flow_digest=from_string("k%d" % i))
            elif op == "coerce":
                f = OFlow("OpCoerce", pick(1), flow_digest=from_string("c%d" % i))
            elif op == "groupby":
                f = OFlow("OpGroupby", pick(1), re="foo-(.*)%d" % i)
            elif op == "collect":
                f = OFlow("OpCollect", pick(1), re=".*", repl="$%d" % i)
            elif op == "map":
                val = OFlow("OpVal", value=OFileset(map=None))
                mf = OFlow("OpExec", [val], image="image", cmd="command %d" % i)
                f = OFlow("OpMap", pick(1), mapflow=mf)
            elif op == "req":
                f = OFlow("OpRequirements", pick(1))
            else:
                f = OFlow("OpExtern", pick(1), url="s3://out/%d" % i, done=False)
            if f.value is None and rng.random() < 0.5:
                f.done = True
                f.value = rand_value(rng)
        nodes.append(f)
    # join everything under a root so all nodes are reachable
    root = OFlow("OpMerge", list(nodes))
    return root, nodes + [root]
