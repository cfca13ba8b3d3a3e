"""The bench's CPU baseline legs (oracle/baseline_openssl.c: OpenSSL SHA-256
on native threads, one shared queue) agree with hashlib: in-memory batches at
the padding-edge lengths in any queue order, and files read from disk
(missing files reported)."""
import ctypes
import hashlib
import os

import numpy as np

import reflow_oracle as O


def test_batch_matches_hashlib():
    L = O.lib()
    rng = np.random.default_rng(5)
    lens = np.array([0, 1, 55, 56, 63, 64, 65, 119, 4096, 262144, 1 << 20], dtype=np.uint64)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
    arena = rng.integers(0, 256, size=int(lens.sum()) + 1, dtype=np.uint8)
    out = np.zeros((len(lens), 32), dtype=np.uint8)
    order = np.argsort(-lens.astype(np.int64)).astype(np.uint64)
    for o in (None, order):
        out[:] = 0
        rc = L.orc_openssl_sha256_batch(arena.ctypes.data, offs.ctypes.data, lens.ctypes.data,
                                        None if o is None else o.ctypes.data, len(lens), out.ctypes.data, 4)
        assert rc == 0
        for i in range(len(lens)):
            a, n = int(offs[i]), int(lens[i])
            assert out[i].tobytes() == hashlib.sha256(arena[a:a + n].tobytes()).digest()


def test_files_match_hashlib(tmp_path):
    L = O.lib()
    paths = []
    for i, n in enumerate([0, 1, 64, (1 << 20) - 1, 1 << 20, (1 << 20) + 1, 3 << 20]):
        p = tmp_path / ("f%d" % i)
        p.write_bytes(os.urandom(n))
        paths.append(str(p).encode())
    arr = (ctypes.c_char_p * len(paths))(*paths)
    out = np.zeros((len(paths), 32), dtype=np.uint8)
    assert L.orc_openssl_sha256_files(ctypes.cast(arr, ctypes.c_void_p), len(paths), out.ctypes.data, 3) == 0
    for i, p in enumerate(paths):
        assert out[i].tobytes() == hashlib.sha256(open(p, "rb").read()).digest()
    bad = (ctypes.c_char_p * 1)(str(tmp_path / "missing").encode())
    assert L.orc_openssl_sha256_files(ctypes.cast(bad, ctypes.c_void_p), 1, out.ctypes.data, 1) == -1
