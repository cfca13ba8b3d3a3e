"""Oracle restatement of Eval.lookup's assoc step (eval.go:1172-1258):
first hit in CacheKeys order wins; read repair blind (the reference) or
precise (its TODO, eval.go:1199-1201).  CPU only."""
import reflow_oracle as O

ZERO = bytes(32)


def test_oracle_lookup_semantics():
    """Hand cases of eval.go:1202-1258 on the oracle: first hit wins, blind
    repair overwrites a later synonym, precise repair only fills misses."""
    A, B, C, V1, V2 = (bytes([i]) * 32 for i in (1, 2, 3, 4, 5))
    for repair, want_c in [(0, V2), (1, V1), (2, V2)]:
        ref = O.InmemoryAssoc()
        ref.put(0, None, B, V1)
        ref.put(0, None, C, V2)
        assert O.assoc_lookup(ref, 0, [[A, B, C], [], [A]], repair) == [(1, V1), (-1, ZERO), (-1, ZERO)]
        assert ref.get(0, A) == (None if repair == 0 else V1)
        assert ref.get(0, C) == want_c
