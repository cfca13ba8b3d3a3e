"""Runs the K1 diagnostic microbenchmarks (tools/micro.hip) on the GPU."""
import ctypes
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "_micro.so")


def build():
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
                           "-fPIC", "-Wno-unused-value", "-shared", os.path.join(HERE, "micro.hip"), "-o", SO])


def main():
    if not os.path.exists(SO) or (len(sys.argv) > 1 and sys.argv[1] == "build"):
        build()
        if len(sys.argv) > 1 and sys.argv[1] == "build":
            return
    L = ctypes.CDLL(SO)
    if len(sys.argv) > 1 and sys.argv[1] == "atomic":
        # same-address atomics from waves that arrive together (the level
        # lists' append cursors): launch time vs the number of counters
        L.micro_atomic.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32]
        L.micro_atomic.restype = ctypes.c_float
        for waves in (256, 2200, 8800):
            for work in (0, 20000):
                base = L.micro_atomic(waves, work, 0)
                row = ["waves %5d work %5d: none %.1f us" % (waves, work, base * 1e3)]
                for n_addr in (1, 8, 64, 512):
                    ms = L.micro_atomic(waves, work, n_addr)
                    row.append("%d addr %+.1f us" % (n_addr, (ms - base) * 1e3))
                print(", ".join(row))
        return
    if len(sys.argv) > 1 and sys.argv[1] == "barrier":
        L.micro_barrier.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int]
        L.micro_barrier.restype = ctypes.c_float
        it = 100000
        for grid, block in ((1, 64), (1, 128), (1, 256), (64, 128), (256, 128)):
            for raw in (0, 1):
                ms = L.micro_barrier(grid, block, it, raw)
                print("barrier grid %4d block %3d %-14s %.3f ms  %.1f ns/iter" %
                      (grid, block, "s_barrier" if raw else "__syncthreads", ms, ms * 1e6 / it))
        return
    if len(sys.argv) > 1 and sys.argv[1] == "hwid":
        import numpy as np
        for grid, block in ((64, 128), (64, 256), (512, 128), (1024, 128)):
            out = np.zeros(grid * block // 64, dtype=np.uint32)
            L.micro_hwid.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p]
            L.micro_hwid(grid, block, out.ctypes.data)
            simd = (out >> 4) & 3
            per_wg = simd.reshape(grid, block // 64)
            same = int((per_wg == per_wg[:, :1]).all(axis=1).sum())
            print("grid %d block %d: workgroups with all waves on one SIMD: %d/%d; first WGs %s"
                  % (grid, block, same, grid, per_wg[:4].tolist()))
        return
    L.micro_compute.argtypes = [ctypes.c_uint32, ctypes.c_uint32]
    L.micro_compute.restype = ctypes.c_float
    L.micro_loads.argtypes = [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int, ctypes.c_int]
    L.micro_loads.restype = ctypes.c_float
    L.micro_op.argtypes = [ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32]
    L.micro_op.restype = ctypes.c_float
    L.micro_lat.argtypes = [ctypes.c_int, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint64)]
    L.micro_lat.restype = ctypes.c_float
    lat_names = ["dep v_add_u32", "dep v_alignbit", "dep v_bitop3", "dep v_add3", "dep add_dpp ror8",
                 "dep add_dpp ror8 bank", "indep v_add_u32", "dep add+s_nop0", "duo round (dpp)",
                 "duo round (plain)", "lag2 step",
                 "indep8 alignbit", "indep8 v_add", "indep8 bitop3 3src", "indep8 add_dpp", "indep8 bitop3 2src",
                 "indep8 bitop3 no-bank-conflict", "indep8 bitop3 bank-conflict",
                 "lag2 order V1", "lag2 order V5", "lag2 order V6", "lag2 order V7", "lag2 order V8",
                 "cost alignbit vshift", "cost alignbit imm", "cost bitop3 3v", "cost add3 3v", "cost xad 3v",
                 "cost v_add vop2", "cost add_dpp", "cost v_xor vop2", "cost v_add e64", "cost lshl_add", "cost v_add same-reg", "cost bitop3 2reg", "cost v_mov",
                 "cost s_add x64", "64 v_add + 64 s_add interleaved", "64 bitop3 + 64 s_add interleaved",
                 "cost v_add exec16", "cost v_add exec1", "cost alignbit exec16", "cost alignbit exec1"]
    for op, name in enumerate(lat_names):
        iters = 1 << 17
        cyc = ctypes.c_uint64(0)
        ms = L.micro_lat(op, iters, ctypes.byref(cyc))
        n = iters * 8 * (9 if op == 10 or 18 <= op <= 22 else 10 if op in (8, 9) else 8 if op >= 39 else 16 if op >= 37 else 8 if op >= 23 else 1)
        print("lat %-22s 1 wave  %.3f ms  %.2f ns/instr  memtime %.2f ticks/instr  %s"
              % (name, ms, ms * 1e6 / n, cyc.value / n, "(%.1f ns/round)" % (ms * 1e6 / (iters * 8)) if op >= 8 else ""),
              flush=True)
    if len(sys.argv) > 1 and sys.argv[1] == "lat":
        return
    L.micro_gather.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int, ctypes.c_int]
    L.micro_gather.restype = ctypes.c_float
    for tb in [171 * 2**20, 2 * 2**30]:
        for r, km in [(10, 0), (10, 1), (10, 2), (6, 1), (2, 1)]:
            n = 1 << 28
            ms = L.micro_gather(tb, n, r, km)
            print("gather table=%6.0f MiB reads/thread=%2d keys=%s  %.2f ms  %.2f G reads/s  %.2f G threads/s"
                  % (tb / 2**20, r, ["none", "default", "nt"][km], ms, n * r / ms / 1e6, n / ms / 1e6),
                  flush=True)
    if len(sys.argv) > 1 and sys.argv[1] == "gather":
        return
    names = ["v_add_u32", "v_alignbit_b32", "v_bitop3_b32", "v_add3_u32", "v_xor_b32", "v_perm_b32",
             "v_lshrrev_b32", "v_fma_f32"]
    for op, name in enumerate(names):
        for grid in [256, 2048]:
            iters = 4096
            ms = L.micro_op(op, grid, iters)
            n = grid * 256 * iters * 8
            print("op %-16s grid=%5d (%d waves/SIMD)  %.3f ms  %.2f T lane-ops/s  (%.0f%% of 78.6)"
                  % (name, grid, grid // 256, ms, n / ms / 1e9, 100 * n / ms / 1e9 / 78.64), flush=True)
    peak = 256 * 128 * 2.4e9
    for grid in [256, 512, 1024, 1280, 2048]:
        nblk = 256
        ms = L.micro_compute(grid, nblk)
        ops = grid * 256 * nblk * 1464
        print("compute grid=%5d waves/SIMD=%.1f  %.3f ms  %.2f Tops/s  (%.0f%% of 78.6)  %.0f GB/s-equiv"
              % (grid, grid / 256.0, ms, ops / ms / 1e9, 100 * ops / ms / 1e9 / (peak / 1e12) / 1e3 * 1e3 / 1e3,
                 grid * 256 * nblk * 64 / ms / 1e6), flush=True)
    KB = 1024
    for layout, stride, nlanes, nblk, pf in [
        (1, 0, 65536, 1024, 0), (1, 0, 65536, 1024, 1), (1, 0, 262144, 256, 0), (1, 0, 262144, 256, 1),
        (0, 64 * KB, 65536, 1024, 0), (0, 64 * KB, 65536, 1024, 1), (0, 64 * KB + 256, 65536, 1024, 1),
        (0, 16 * KB, 262144, 256, 0), (0, 16 * KB, 262144, 256, 1), (0, 16 * KB + 256, 262144, 256, 1),
        (0, 16 * KB + 64, 262144, 256, 1), (0, 4 * KB, 262144, 64, 1), (0, 4 * KB + 64, 262144, 64, 1)]:
        ms = L.micro_loads(stride, nblk, nlanes, layout, pf)
        b = nlanes * nblk * 64
        print("loads layout=%d stride=%7d lanes=%7d nblk=%5d prefetch=%d  %.3f ms  %.1f GB/s  %.2f Tops/s"
              % (layout, stride, nlanes, nblk, pf, ms, b / ms / 1e6, b / 64 * 1464 / ms / 1e9), flush=True)


if __name__ == "__main__":
    main()
