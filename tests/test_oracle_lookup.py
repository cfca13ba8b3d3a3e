"""Oracle restatement of Eval.lookup's assoc step (eval.go:1172-1258): first
usable hit in CacheKeys order wins (a fsid that does not unmarshal moves the
loop on, :1210-1218); read repair -- blind (the reference) or precise (its
TODO, eval.go:1199-1201) -- only after the value passed missing() and the
RecomputeEmpty check (:1227-1258).  CPU only."""
import reflow_oracle as O

ZERO = bytes(32)


def test_oracle_lookup_semantics():
    """Hand cases: first hit wins, blind repair overwrites a later synonym,
    precise repair only fills misses."""
    A, B, C, V1, V2 = (bytes([i]) * 32 for i in (1, 2, 3, 4, 5))
    for repair, want_c in [(0, V2), (1, V1), (2, V2)]:
        ref = O.InmemoryAssoc()
        ref.put(0, None, B, V1)
        ref.put(0, None, C, V2)
        assert O.eval_lookup(ref, 0, [[A, B, C], [], [A]], repair) == [(1, V1), (-1, ZERO), (-1, ZERO)]
        assert ref.get(0, A) == (None if repair == 0 else V1)
        assert ref.get(0, C) == want_c


def test_oracle_lookup_unmarshal_fail_and_unverified():
    """A fsid that does not unmarshal is skipped for the next key; a node whose
    files are missing (verified fails) is a miss and repairs nothing."""
    A, B, C, V1, V2 = (bytes([i]) * 32 for i in (1, 2, 3, 4, 5))
    ref = O.InmemoryAssoc()
    ref.put(0, None, A, V1)  # V1: unmarshal fails
    ref.put(0, None, B, V2)
    got = O.eval_lookup(ref, 0, [[A, B, C]], repair=1, usable=lambda i, v: v != V1)
    assert got == [(1, V2)]
    assert ref.get(0, A) == V2 and ref.get(0, C) == V2  # blind: every other key
    ref = O.InmemoryAssoc()
    ref.put(0, None, B, V2)
    got = O.eval_lookup(ref, 0, [[A, B]], repair=2, verified=lambda i, v: False)
    assert got == [(1, V2)] and ref.get(0, A) is None  # unverified: no write
