"""JSON (de)serialisation of oracle objects for the committed golden fixtures.

A flow fixture is a node list in topological order; each node names its
deps / mapflow / parent by index, so a test rebuilds the exact OFlow graph
(sharing included) and can lower it to the GPU graph engine.
"""
from __future__ import annotations

import json
import os

from reflow_oracle import OFileset, OFlow, OPS

HERE = os.path.dirname(os.path.abspath(__file__))


def path(name: str) -> str:
    return os.path.join(HERE, name)


def load(name: str):
    with open(path(name)) as f:
        return json.load(f)


def fileset_to_json(v: OFileset):
    if v is None:
        return None
    if v.list is not None:
        return {"list": [fileset_to_json(x) for x in v.list]}
    if v.map is None:
        return {"map": None}
    return {"map": {p: [fid.hex(), size] for p, (fid, size) in v.map.items()}}


def json_to_fileset(d):
    if d is None:
        return None
    if "list" in d:
        return OFileset(list=[json_to_fileset(x) for x in d["list"]])
    if d["map"] is None:
        return OFileset(map=None)
    return OFileset(map={p: (bytes.fromhex(h), s) for p, (h, s) in d["map"].items()})


def topo(root: OFlow):
    """Every flow reachable from root (deps, mapflow, parent), children first."""
    order, seen = [], set()
    stack = [(root, False)]
    while stack:
        f, done = stack.pop()
        if done:
            order.append(f)
            continue
        if id(f) in seen:
            continue
        seen.add(id(f))
        stack.append((f, True))
        kids = list(f.deps) + [x for x in (f.mapflow, f.parent) if x is not None]
        for c in reversed(kids):
            if id(c) not in seen:
                stack.append((c, False))
    return order


def flow_to_json(root: OFlow):
    nodes = topo(root)
    idx = {id(f): i for i, f in enumerate(nodes)}
    out = []
    for f in nodes:
        n = {"op": OPS[f.op - 1], "deps": [idx[id(d)] for d in f.deps]}
        for k in ("image", "cmd", "url", "re", "repl"):
            if getattr(f, k):
                n[k] = getattr(f, k)
        if f.mapflow is not None:
            n["mapflow"] = idx[id(f.mapflow)]
        if f.parent is not None:
            n["parent"] = idx[id(f.parent)]
        if f.argmap is not None:
            n["argmap"] = [[bool(o), int(i)] for o, i in f.argmap]
        if f.flow_digest is not None:
            n["flow_digest"] = f.flow_digest.hex()
        if f.value is not None:
            n["value"] = fileset_to_json(f.value)
        if f.done:
            n["done"] = True
        if f.data:
            n["data"] = f.data.hex()
        if f.hashv1:
            n["hashv1"] = True
        out.append(n)
    return {"nodes": out, "root": len(nodes) - 1}


def json_to_flow(d):
    """Returns (root, nodes) with nodes in fixture order."""
    nodes = []
    for n in d["nodes"]:
        kw = {k: n[k] for k in ("image", "cmd", "url", "re", "repl") if k in n}
        if "mapflow" in n:
            kw["mapflow"] = nodes[n["mapflow"]]
        if "parent" in n:
            kw["parent"] = nodes[n["parent"]]
        if "argmap" in n:
            kw["argmap"] = [(bool(o), int(i)) for o, i in n["argmap"]]
        if "flow_digest" in n:
            kw["flow_digest"] = bytes.fromhex(n["flow_digest"])
        if "value" in n:
            kw["value"] = json_to_fileset(n["value"])
        kw["done"] = n.get("done", False)
        if "data" in n:
            kw["data"] = bytes.fromhex(n["data"])
        kw["hashv1"] = n.get("hashv1", False)
        nodes.append(OFlow(n["op"], [nodes[i] for i in n["deps"]], **kw))
    return nodes[d["root"]], nodes


def json_to_fs_tree(d):
    """Inverse of make_golden.fs_tree_to_json (byte paths)."""
    return OFileset(list=None if d["list"] is None else [json_to_fs_tree(x) for x in d["list"]],
                    map=None if d["map"] is None else
                    {bytes.fromhex(p): (bytes.fromhex(f), s) for p, f, s in d["map"]})
