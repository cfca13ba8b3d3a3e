"""Probe of the GPU box's host CPU share: affinity, cgroup quota, and hashlib
(OpenSSL, SHA-NI) SHA-256 throughput at several thread counts."""
import hashlib, os, time
from concurrent.futures import ThreadPoolExecutor
print("cpu_count", os.cpu_count(), "affinity", len(os.sched_getaffinity(0)))
for p in ("/sys/fs/cgroup/cpu.max", "/sys/fs/cgroup/cpuset.cpus.effective", "/sys/fs/cgroup/memory.max"):
    try:
        print(p, open(p).read().strip())
    except OSError as e:
        print(p, "n/a", e)
for k in ("OMP_NUM_THREADS", "MAX_JOBS", "LOCAL_WORLD_SIZE"):
    print(k, os.environ.get(k))
buf = os.urandom(64 << 20)
t0 = time.perf_counter(); hashlib.sha256(buf).digest(); dt = time.perf_counter() - t0
print("1 thread 64 MiB: %.2f GB/s" % (len(buf) / dt / 1e9))
for nt in (8, 16, 32, 60):
    with ThreadPoolExecutor(nt) as ex:
        t0 = time.perf_counter()
        list(ex.map(lambda i: hashlib.sha256(buf).digest(), range(2 * nt)))
        dt = time.perf_counter() - t0
    print("%d threads: %.2f GB/s" % (nt, 2 * nt * len(buf) / dt / 1e9), flush=True)
