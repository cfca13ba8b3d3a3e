"""Generates tests/golden/c2_ids.bin + c2_ids.json: the File IDs of the whole
configs[1] set (64 GiB, sizes from reflow_amd.workloads.c2_sizes, content =
the splitmix64 stream (seed ^ i) that rf_gen_fill writes on the device),
computed by the oracle's scalar SHA-256 (oracle/oracle.c orc_stream_sha256,
streamed: no 2 GiB file is materialised).  Run in the container; the GPU test
(tests/test_gpu_hybrid.py) compares the device's digests with these."""
import hashlib
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]

import reflow_oracle as O  # noqa: E402
from reflow_amd.workloads import GiB, c2_sizes  # noqa: E402

SEED = 0x5EED0002


def main():
    lens = c2_sizes(total_bytes=64 * GiB, seed=SEED)
    out = np.zeros(32 * len(lens), dtype=np.uint8)
    t0 = time.time()
    O.lib().orc_stream_sha256_batch(SEED, lens.ctypes.data, len(lens), out.ctypes.data, os.cpu_count() or 1)
    dt = time.time() - t0
    out.tofile(os.path.join(HERE, "c2_ids.bin"))
    meta = {"what": "configs[1] File IDs: SHA256(splitmix64 stream seed^i, lens[i]) for the c2_sizes set",
            "seed": SEED, "total_bytes": int(lens.sum()), "n_files": int(len(lens)),
            "max_len": int(lens.max()), "lens_sha256": hashlib.sha256(lens.tobytes()).hexdigest(),
            "ids_sha256": hashlib.sha256(out.tobytes()).hexdigest(),
            "generator": "tests/golden/make_c2_fixture.py (oracle/oracle.c orc_stream_sha256_batch)"}
    json.dump(meta, open(os.path.join(HERE, "c2_ids.json"), "w"), indent=1)
    print("%d files, %.1f GiB in %.1f s" % (len(lens), lens.sum() / GiB, dt))


if __name__ == "__main__":
    main()
