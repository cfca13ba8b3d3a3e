"""Streaming SHA-256 (rf_sha_streams: Digester.NewWriter carried across Write
calls, as Repository.Put hashes an io.Reader, repository/file/repository.go:
237-264 / repository/s3/s3.go:120-147) and the integrity checks
(rf_sha_streams_verify / rf_sha256_verify: ReadFrom / WriteTo's re-digest,
repository/file/repository.go:126-166), against the oracle's one-shot SHA-256
of each stream's concatenated bytes.  Every chunking boundary a stream can
carry -- 0, 55, 56, 63, 64 bytes and their neighbours -- on each leg: the GPU
resume kernel alone (NO_HOST), the host leg alone (ALL_HOST), and the split."""
import random

import pytest

from reflow_amd import capi

pytestmark = pytest.mark.gpu

EDGE = [0, 1, 2, 54, 55, 56, 57, 62, 63, 64, 65, 119, 120, 127, 128, 129, 1000, 4096, 70001]
MODES = [("gpu", capi.RF_SHA_NO_HOST), ("host", capi.RF_SHA_ALL_HOST), ("split", 0)]


@pytest.fixture(scope="module")
def ctx():
    c = capi.Context(0)
    yield c
    c.close()


def _skip_host(ctx, flags):
    if flags == capi.RF_SHA_ALL_HOST and ctx.host_info()[0] == 0:
        pytest.skip("host leg unavailable")


@pytest.mark.parametrize("name,flags", MODES)
def test_streams_chunk_edges(ctx, oracle, name, flags):
    """40 streams written in 6 batches of chunks with lengths at every
    partial-block edge, several chunks per stream per batch, streams
    interleaved; each digest equals SHA-256 of the stream's bytes."""
    _skip_host(ctx, flags)
    rng = random.Random(7)
    n = 40
    s = ctx.sha_streams(n, flags)
    data = [bytearray() for _ in range(n)]
    for b in range(6):
        ids, chunks = [], []
        for _ in range(120):
            i = rng.randrange(n)
            c = oracle.fill_stream(rng.getrandbits(32), rng.choice(EDGE))
            ids.append(i)
            chunks.append(c)
            data[i] += c
        s.write(ids, chunks)
    assert [s.length(i) for i in range(n)] == [len(d) for d in data]
    got = s.digest(list(range(n)))
    assert got == [oracle.sha256(bytes(d)) for d in data]
    # restarted empty: a second round of writes digests from scratch
    s.write([3, 3], [b"abc", b"def"])
    assert s.digest([3, 0]) == [oracle.sha256(b"abcdef"), oracle.sha256(b"")]
    s.close()


@pytest.mark.parametrize("name,flags", MODES)
def test_streams_single_chunk_lengths(ctx, oracle, name, flags):
    """One chunk per stream of each edge length, then the digest: the padding
    of the carried block alone (0..63 bytes carried, 0 and 1+ blocks hashed)."""
    _skip_host(ctx, flags)
    s = ctx.sha_streams(len(EDGE), flags)
    msgs = [oracle.fill_stream(0xABC ^ i, n) for i, n in enumerate(EDGE)]
    s.write(list(range(len(EDGE))), msgs)
    assert s.digest(list(range(len(EDGE)))) == [oracle.sha256(m) for m in msgs]
    s.close()


def test_streams_upload_like_put(ctx, oracle):
    """Repository.Put of a 40 MiB object through 1 MiB + 17-byte reads (the
    io.Copy buffer does not align with SHA-256 blocks), beside 300 small
    concurrent uploads: the split puts the long stream on the host leg."""
    s = ctx.sha_streams(301)
    big = oracle.fill_stream(99, 40 * (1 << 20) + 5)
    small = [oracle.fill_stream(1000 + i, 3000 + i) for i in range(300)]
    off, step = 0, (1 << 20) + 17
    while off < len(big):
        ids = [0] + list(range(1, 301))
        chunks = [big[off:off + step]] + [m[off // step * 100:(off // step + 1) * 100] for m in small]
        s.write(ids, chunks)
        off += step
    want_small = [m[:((len(big) + step - 1) // step) * 100] for m in small]
    assert s.digest(list(range(301))) == [oracle.sha256(big)] + [oracle.sha256(m) for m in want_small]
    s.close()


def test_streams_verify_integrity(ctx, oracle):
    s = ctx.sha_streams(3)
    msgs = [b"x" * 100, b"", b"reflow" * 1000]
    s.write([0, 2], [msgs[0], msgs[2]])
    want = [oracle.sha256(m) for m in msgs]
    rc, st = s.verify([0, 1, 2], want)
    assert rc == capi.RF_OK and list(st) == [0, 0, 0]
    s.write([0, 1, 2], msgs)
    rc, st = s.verify([0, 1, 2], [want[0], want[2], want[2]])
    assert rc == capi.RF_EINTEGRITY and list(st) == [capi.RF_OK, capi.RF_EINTEGRITY, capi.RF_OK]
    s.close()


def test_sha256_verify(ctx, oracle):
    msgs = [oracle.fill_stream(i, n) for i, n in enumerate([0, 64, 1000, 1 << 20])]
    want = [oracle.sha256(m) for m in msgs]
    rc, st = ctx.sha256_verify(msgs, want)
    assert rc == capi.RF_OK and not st.any()
    bad = list(want)
    bad[2] = bytes(32)
    rc, st = ctx.sha256_verify(msgs, bad)
    assert rc == capi.RF_EINTEGRITY and list(st) == [0, 0, capi.RF_EINTEGRITY, 0]


def test_streams_bad_ids(ctx):
    s = ctx.sha_streams(2)
    with pytest.raises(capi.RfError):
        s.write([2], [b"x"])
    with pytest.raises(capi.RfError):
        s.digest([1, 1])
    s.close()
