"""ctypes binding of include/reflow_hip.h (libreflow_hip.so).

This is plumbing for the Python test-suite and bench.py: every call goes
through the C-ABI into the gfx950 kernels.  There is no CPU fallback: if the
library or a gfx950 device is missing, the calls raise.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libreflow_hip.so")

RF_OK, RF_EINVAL, RF_EIO, RF_EINTEGRITY, RF_EDEVICE, RF_ENOMEM, RF_ENOTFOUND, RF_EPRECONDITION = range(8)
RF_SHA_NO_SOLO = 1
RF_SHA_ALL_SOLO = 2
RF_SHA_ONE_LANE_CHAIN = 4
RF_SHA_NO_PAIR = 8
RF_SHA_NO_OCTO = 16
RF_SHA_ALL_HOST = 32
RF_SHA_NO_HOST = 64

# Every symbol include/reflow_hip.h declares (checked by tests/test_capi_symbols.py).
EXPORTS = [
    "rf_init", "rf_destroy", "rf_last_error", "rf_device_count", "rf_sync", "rf_version",
    "rf_sha256_batch", "rf_sha256_arena", "rf_sha_plan_create", "rf_sha_plan_run",
    "rf_sha_plan_stats", "rf_sha_plan_destroy", "rf_gen_fill", "rf_fileset_digest_batch",
    "rf_fileset_digest_device", "rf_install_dir", "rf_install_info", "rf_install_entries",
    "rf_install_destroy",
    "rf_graph_load", "rf_graph_destroy", "rf_graph_set_slots", "rf_graph_set_slots_device",
    "rf_graph_save", "rf_graph_restore", "rf_graph_set_forms",
    "rf_graph_adopt_slots",
    "rf_graph_recompute", "rf_graph_recompute_async", "rf_graph_get_slots", "rf_graph_stats_get",
    "rf_bloom_load", "rf_bloom_load_json", "rf_bloom_load_binary", "rf_bloom_new",
    "rf_bloom_destroy", "rf_bloom_probe", "rf_bloom_probe_device", "rf_bloom_add",
    "rf_bloom_add_device", "rf_bloom_params", "rf_bloom_words",
    "rf_malloc", "rf_free", "rf_memcpy_h2d", "rf_memcpy_d2h", "rf_memset_d", "rf_stream",
    "rf_timer_start", "rf_timer_stop", "rf_comm_unique_id", "rf_comm_init", "rf_comm_destroy",
    "rf_comm_allgather", "rf_comm_allreduce_or", "rf_memcpy_d2d", "rf_graph_gather_device",
    "rf_fileset_marshal_json", "rf_fileset_value_digest_batch",
    "rf_bloom_marshal_json", "rf_bloom_marshal_binary", "rf_bloom_parse_binary", "rf_bloom_parse_json",
    "rf_bloom_format_binary", "rf_bloom_format_json", "rf_bloom_collect", "rf_bloom_collect_device",
    "rf_dedup_digests", "rf_dedup_digests_device", "rf_assoc_lookup",
    "rf_assoc_new", "rf_assoc_destroy", "rf_assoc_put", "rf_assoc_get", "rf_assoc_get_device",
    "rf_assoc_get_abbrev", "rf_assoc_stats", "rf_assoc_put_device",
    "rf_set_host_threads", "rf_host_info", "rf_host_rate", "rf_host_link", "rf_assoc_repair",
    "rf_sha_streams_open", "rf_sha_streams_close", "rf_sha_streams_write", "rf_sha_streams_digest",
    "rf_sha_streams_len", "rf_sha_streams_verify", "rf_sha256_verify", "rf_flow_dirty",
    "rf_coalescer_open", "rf_coalescer_close", "rf_coalesce_sha256", "rf_coalesce_probe", "rf_coalesce_assoc_get",
    "rf_coalesce_sha256_async", "rf_coalesce_poll", "rf_coalesce_wait", "rf_coalesce_ticket_free",
    "rf_coalescer_stats", "rf_graph_update_recompute_async", "rf_walk_dir", "rf_walk_info", "rf_walk_entries", "rf_walk_free",
    "rf_graph_set_part", "rf_graph_recompute_part", "rf_graph_part_gathered", "rf_graph_split",
    "rf_graph_piece_free", "rf_graph_piece_desc", "rf_graph_piece_part", "rf_graph_piece_slots",
]


class RfError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("rf error %d: %s" % (code, msg))
        self.code = code


class ShaStats(ctypes.Structure):
    _fields_ = [("n_msgs", ctypes.c_uint64), ("n_solo", ctypes.c_uint64),
                ("total_blocks", ctypes.c_uint64), ("max_blocks", ctypes.c_uint64),
                ("total_bytes", ctypes.c_uint64), ("last_ms_lanes", ctypes.c_float),
                ("last_ms_solo", ctypes.c_float), ("last_ms_total", ctypes.c_float),
                ("last_ms_host", ctypes.c_float), ("host_threads", ctypes.c_uint32),
                ("n_host", ctypes.c_uint64), ("host_bytes", ctypes.c_uint64)]


class GraphDesc(ctypes.Structure):
    _fields_ = [("n_jobs", ctypes.c_uint32), ("n_slots", ctypes.c_uint32),
                ("out_slot", ctypes.c_void_p), ("tmpl_off", ctypes.c_void_p),
                ("tmpl_len", ctypes.c_void_p), ("hole_ptr", ctypes.c_void_p),
                ("hole_pos", ctypes.c_void_p), ("hole_slot", ctypes.c_void_p),
                ("blob", ctypes.c_void_p), ("blob_len", ctypes.c_uint64)]


class FilesetTree(ctypes.Structure):
    _fields_ = [("n_nodes", ctypes.c_uint64), ("list_ptr", ctypes.c_void_p),
                ("list_child", ctypes.c_void_p), ("entry_ptr", ctypes.c_void_p),
                ("paths", ctypes.c_void_p), ("path_lens", ctypes.c_void_p),
                ("ids32", ctypes.c_void_p), ("sizes", ctypes.c_void_p)]


class FilesetTreeBuilder:
    """Flattens nested filesets into the rf_fileset_tree CSR form.  A fileset
    is any object with .list (None or a list of filesets) and .map (None or a
    dict path -> (id32, size)); add() returns its root node index."""

    def __init__(self):
        self.list_ptr, self.list_child, self.entry_ptr = [0], [], [0]
        self.paths, self.ids, self.sizes = [], [], []
        self._pending = []

    def add(self, fs) -> int:
        # nodes are numbered in pre-order; children lists refer forward
        node = len(self.list_ptr) - 1
        self.list_ptr.append(None)
        self.entry_ptr.append(None)
        for path, (id32, size) in (fs.map or {}).items():
            self.paths.append(path.encode("utf-8", "surrogateescape") if isinstance(path, str) else path)
            self.ids.append(bytes(id32))
            self.sizes.append(int(size))
        self.entry_ptr[node + 1] = len(self.paths)
        kids = [self.add(c) for c in (fs.list or [])]
        self._pending.append((node, kids))
        return node

    def struct(self):
        n = len(self.list_ptr) - 1
        children = dict(self._pending)
        lp, lc = [0], []
        for i in range(n):
            lc.extend(children[i])
            lp.append(len(lc))
        # a node's entries are recorded before its children's (pre-order), so
        # entry_ptr is already the CSR; list_ptr is rebuilt from the children
        self._keep = dict(
            lp=np.array(lp, dtype=np.uint64), lc=np.array(lc or [0], dtype=np.uint32),
            ep=np.array(self.entry_ptr, dtype=np.uint64),
            pb=[ctypes.create_string_buffer(p, max(len(p), 1)) for p in self.paths],
            pl=np.array([len(p) for p in self.paths] or [0], dtype=np.uint32),
            ids=np.frombuffer(b"".join(self.ids) or b"\0" * 32, dtype=np.uint8).copy(),
            sz=np.array(self.sizes or [0], dtype=np.int64))
        k = self._keep
        k["pp"] = (ctypes.c_void_p * max(len(self.paths), 1))(*[ctypes.addressof(b) for b in k["pb"]])
        return FilesetTree(n, _ptr(k["lp"]), _ptr(k["lc"]), _ptr(k["ep"]),
                           ctypes.cast(k["pp"], ctypes.c_void_p), _ptr(k["pl"]), _ptr(k["ids"]),
                           _ptr(k["sz"]))


def fileset_marshal_json(fs) -> bytes:
    """json.Marshal(Fileset) through the C-ABI (host code, no device)."""
    b = FilesetTreeBuilder()
    root = b.add(fs)
    t = b.struct()
    need = ctypes.c_uint64(0)
    rc = lib().rf_fileset_marshal_json(ctypes.byref(t), root, None, 0, ctypes.byref(need))
    if rc != RF_OK and need.value == 0:
        _check(rc)
    out = ctypes.create_string_buffer(max(need.value, 1))
    _check(lib().rf_fileset_marshal_json(ctypes.byref(t), root, out, need.value, ctypes.byref(need)))
    return out.raw[:need.value]


class GraphPart(ctypes.Structure):
    _fields_ = [("nranks", ctypes.c_int), ("rank", ctypes.c_int), ("max_export", ctypes.c_uint32),
                ("n_export", ctypes.c_uint32), ("export_slot", ctypes.c_void_p),
                ("n_import", ctypes.c_uint32), ("import_slot", ctypes.c_void_p),
                ("import_bid", ctypes.c_void_p), ("any_import", ctypes.c_int), ("rounds", ctypes.c_uint32)]


# int (*)(void *user, const void *send, void *recv, uint64_t bytes)
HOST_ALLGATHER = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64)


def host_allgather_fn(allgather, nranks):
    """Wraps allgather(bytes) -> [bytes per rank] (e.g. torch.distributed
    gloo) as the library's host all-gather callback."""
    def fn(user, send, recv, nbytes):
        try:
            parts = allgather(ctypes.string_at(send, nbytes))
            assert len(parts) == nranks and all(len(p) == nbytes for p in parts)
            ctypes.memmove(recv, b"".join(parts), nranks * nbytes)
            return 0
        except Exception:  # noqa: BLE001 -- reported to the library as a failure
            import traceback
            traceback.print_exc()
            return 1
    return HOST_ALLGATHER(fn)


def _arr(ptr, n, dtype):
    if n == 0:
        return np.zeros(0, dtype=dtype)
    c = {np.uint32: ctypes.c_uint32, np.uint64: ctypes.c_uint64}[dtype]
    return np.ctypeslib.as_array(ctypes.cast(ptr, ctypes.POINTER(c)), shape=(n,)).copy()


class GraphPiece:
    """rf_graph_split (host only): rank `rank`'s piece of a global job graph
    given as rf_graph_desc arrays (a dict like Dag1000.arrays()); owner[j] =
    the rank hashing job j, -1 = every rank.  Attributes: desc (the piece's
    arrays, templates in the global blob), part (exports / imports / boundary
    ids), global_of_local."""

    def __init__(self, arrays, nranks, rank, owner):
        k = {n: np.ascontiguousarray(arrays[n], dtype=dt) for n, dt in
             (("out_slot", np.uint32), ("tmpl_off", np.uint64), ("tmpl_len", np.uint32),
              ("hole_ptr", np.uint64), ("hole_pos", np.uint32), ("hole_slot", np.uint32))}
        blob = arrays["blob"]
        self.blob = np.frombuffer(bytes(blob), np.uint8) if isinstance(blob, (bytes, bytearray)) \
            else np.ascontiguousarray(blob, dtype=np.uint8)
        own = np.ascontiguousarray(owner, dtype=np.int32)
        d = GraphDesc(len(k["out_slot"]), int(arrays["n_slots"]), _ptr(k["out_slot"]), _ptr(k["tmpl_off"]),
                      _ptr(k["tmpl_len"]), _ptr(k["hole_ptr"]), _ptr(k["hole_pos"]) if len(k["hole_pos"]) else None,
                      _ptr(k["hole_slot"]) if len(k["hole_slot"]) else None, _ptr(self.blob), len(self.blob))
        h = ctypes.c_void_p()
        _check(lib().rf_graph_split(ctypes.byref(d), nranks, rank, _ptr(own), ctypes.byref(h)))
        try:
            ld = GraphDesc()
            _check(lib().rf_graph_piece_desc(h, ctypes.byref(ld)))
            J = ld.n_jobs
            hp = _arr(ld.hole_ptr, J + 1, np.uint64)
            H = int(hp[-1]) if J else 0
            self.desc = dict(n_slots=ld.n_slots, out_slot=_arr(ld.out_slot, J, np.uint32),
                             tmpl_off=_arr(ld.tmpl_off, J, np.uint64), tmpl_len=_arr(ld.tmpl_len, J, np.uint32),
                             hole_ptr=hp, hole_pos=_arr(ld.hole_pos, H, np.uint32),
                             hole_slot=_arr(ld.hole_slot, H, np.uint32), blob=self.blob)
            pt = GraphPart()
            _check(lib().rf_graph_piece_part(h, ctypes.byref(pt)))
            self.part = dict(nranks=pt.nranks, rank=pt.rank, max_export=pt.max_export,
                             export_slot=_arr(pt.export_slot, pt.n_export, np.uint32),
                             import_slot=_arr(pt.import_slot, pt.n_import, np.uint32),
                             import_bid=_arr(pt.import_bid, pt.n_import, np.uint32), any_import=bool(pt.any_import),
                             rounds=int(pt.rounds))
            gp, gn = ctypes.c_void_p(), ctypes.c_uint32()
            _check(lib().rf_graph_piece_slots(h, ctypes.byref(gp), ctypes.byref(gn)))
            self.global_of_local = _arr(gp, gn.value, np.uint32)
        finally:
            lib().rf_graph_piece_free(h)


class GraphStats(ctypes.Structure):
    _fields_ = [("n_jobs", ctypes.c_uint32), ("n_slots", ctypes.c_uint32),
                ("n_levels", ctypes.c_uint32), ("max_level_jobs", ctypes.c_uint32),
                ("total_blocks", ctypes.c_uint64), ("hole_count", ctypes.c_uint64),
                ("template_bytes", ctypes.c_uint64), ("last_recomputed", ctypes.c_uint64),
                ("last_ms", ctypes.c_float), ("last_levels_lf", ctypes.c_uint32),
                ("last_mark_lf", ctypes.c_uint32), ("last_levels_oct", ctypes.c_uint32),
                ("split_block0", ctypes.c_uint32),
                ("last_sink_attach", ctypes.c_uint32), ("last_levels_half", ctypes.c_uint32)]


_lib = None


class FilesetPaths:
    """Argument arrays of rf_fileset_digest_device, built once: sets is a list
    of filesets, each a list of groups (a Map is one group), each a list of
    paths; File ID of entry e = d_ids32[e] (flattened order)."""

    def __init__(self, ctx, sets):
        self.ctx = ctx
        set_group, group_entry, paths = [0], [0], []
        for groups in sets:
            for g in groups:
                paths.extend(p.encode() if isinstance(p, str) else p for p in g)
                group_entry.append(len(paths))
            set_group.append(len(group_entry) - 1)
        self.n = len(sets)
        self.n_entries = len(paths)
        self.sg = np.array(set_group, dtype=np.uint64)
        self.ge = np.array(group_entry, dtype=np.uint64)
        self._pb = [ctypes.create_string_buffer(p, max(len(p), 1)) for p in paths]
        self.pp = (ctypes.c_void_p * max(len(paths), 1))(*[ctypes.addressof(b) for b in self._pb])
        self.pl = np.array([len(p) for p in paths] or [0], dtype=np.uint32)

    def digest_device(self, d_ids32) -> list:
        out = np.zeros(32 * self.n, dtype=np.uint8)
        _check(lib().rf_fileset_digest_device(self.ctx._h, self.n, _ptr(self.sg), _ptr(self.ge), self.pp,
                                              _ptr(self.pl), d_ids32, _ptr(out)))
        return [out[32 * i:32 * i + 32].tobytes() for i in range(self.n)]


def lib():
    """Load libreflow_hip.so.  Raises if it was not built (no fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError("libreflow_hip.so not built: run __graft_entry__.build() "
                               "(make -C reflow_amd/csrc)")
        L = ctypes.CDLL(LIB_PATH)
        vp, u64, u32, i32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int
        sigs = {
            "rf_init": ([i32, vp], i32), "rf_destroy": ([vp], None),
            "rf_last_error": ([], ctypes.c_char_p), "rf_device_count": ([vp], i32),
            "rf_sync": ([vp], i32), "rf_version": ([], ctypes.c_char_p),
            "rf_sha256_batch": ([vp, vp, vp, u64, vp], i32),
            "rf_sha256_arena": ([vp, vp, vp, vp, u64, vp], i32),
            "rf_sha_plan_create": ([vp, vp, vp, u64, u32, vp], i32),
            "rf_sha_plan_run": ([vp, vp, vp, vp], i32),
            "rf_sha_plan_stats": ([vp, vp], i32), "rf_sha_plan_destroy": ([vp], None),
            "rf_gen_fill": ([vp, vp, vp, vp, u64, u64, u64, vp], i32),
            "rf_fileset_digest_batch": ([vp, u64, vp, vp, vp, vp, vp, vp], i32),
            "rf_fileset_digest_device": ([vp, u64, vp, vp, vp, vp, vp, vp], i32),
            "rf_install_dir": ([vp, ctypes.c_char_p, vp], i32),
            "rf_install_info": ([vp, vp, vp, vp], i32),
            "rf_install_entries": ([vp, vp, vp, vp, vp], i32),
            "rf_install_destroy": ([vp], None),
            "rf_graph_load": ([vp, vp, vp], i32), "rf_graph_destroy": ([vp], None),
            "rf_graph_save": ([vp, ctypes.c_char_p], i32), "rf_graph_restore": ([vp, ctypes.c_char_p, vp], i32),
            "rf_graph_set_forms": ([vp, u64, u64, u64], i32),
            "rf_graph_set_slots": ([vp, vp, vp, u32], i32),
            "rf_graph_set_slots_device": ([vp, vp, vp, u32, vp], i32),
            "rf_graph_recompute": ([vp, i32, vp], i32),
            "rf_graph_recompute_async": ([vp, i32, vp], i32),
            "rf_graph_get_slots": ([vp, vp, u32, vp], i32),
            "rf_graph_stats_get": ([vp, vp], i32),
            "rf_graph_adopt_slots": ([vp, vp], i32),
            "rf_bloom_load": ([vp, u64, u64, vp, u64, u64, vp], i32),
            "rf_bloom_load_json": ([vp, ctypes.c_char_p, ctypes.c_size_t, vp], i32),
            "rf_bloom_load_binary": ([vp, vp, ctypes.c_size_t, vp], i32),
            "rf_bloom_new": ([vp, u64, u64, vp], i32), "rf_bloom_destroy": ([vp], None),
            "rf_bloom_probe": ([vp, vp, u64, vp], i32),
            "rf_bloom_probe_device": ([vp, vp, u64, vp, vp], i32),
            "rf_bloom_add": ([vp, vp, u64], i32),
            "rf_bloom_add_device": ([vp, vp, u64, vp], i32),
            "rf_bloom_params": ([vp, vp, vp, vp, vp], i32),
            "rf_bloom_words": ([vp, vp, u64], i32),
            "rf_malloc": ([vp, u64, vp], i32), "rf_free": ([vp, vp], i32),
            "rf_memcpy_h2d": ([vp, vp, vp, u64], i32), "rf_memcpy_d2h": ([vp, vp, vp, u64], i32),
            "rf_memset_d": ([vp, vp, i32, u64], i32), "rf_stream": ([vp], vp),
            "rf_timer_start": ([vp], i32), "rf_timer_stop": ([vp, vp], i32),
            "rf_comm_unique_id": ([vp], i32), "rf_comm_init": ([vp, i32, i32, vp, vp], i32),
            "rf_comm_destroy": ([vp], None), "rf_comm_allgather": ([vp, vp, vp, u64, vp], i32),
            "rf_comm_allreduce_or": ([vp, vp, u64, vp], i32),
            "rf_memcpy_d2d": ([vp, vp, vp, u64], i32),
            "rf_graph_gather_device": ([vp, vp, u32, vp, vp], i32),
            "rf_fileset_marshal_json": ([vp, u32, vp, u64, vp], i32),
            "rf_fileset_value_digest_batch": ([vp, vp, vp, u64, vp], i32),
            "rf_bloom_marshal_json": ([vp, vp, u64, vp], i32),
            "rf_bloom_marshal_binary": ([vp, vp, u64, vp], i32),
            "rf_bloom_collect": ([vp, vp, vp, u64, vp, vp, vp], i32),
            "rf_bloom_collect_device": ([vp, vp, vp, u64, vp, vp, vp], i32),
            "rf_dedup_digests": ([vp, vp, u32, vp, vp], i32),
            "rf_dedup_digests_device": ([vp, vp, u32, vp, vp, vp], i32),
            "rf_assoc_new": ([vp, u64, vp], i32), "rf_assoc_destroy": ([vp], None),
            "rf_assoc_put": ([vp, i32, vp, vp, vp, u64, vp], i32),
            "rf_assoc_get": ([vp, i32, vp, u64, vp, vp], i32),
            "rf_assoc_lookup": ([vp, i32, vp, vp, u64, vp, vp, vp, vp], i32),
            "rf_assoc_repair": ([vp, i32, vp, vp, u64, vp, vp, vp], i32),
            "rf_assoc_get_device": ([vp, i32, vp, u64, vp, vp, vp], i32),
            "rf_assoc_get_abbrev": ([vp, i32, vp, vp, u64, vp, vp, vp], i32),
            "rf_assoc_stats": ([vp, vp, vp], i32),
            "rf_assoc_put_device": ([vp, i32, vp, vp, vp, u64, vp], i32),
            "rf_set_host_threads": ([vp, i32], i32),
            "rf_sha_streams_open": ([vp, u64, u32, vp], i32), "rf_sha_streams_close": ([vp], None),
            "rf_sha_streams_write": ([vp, vp, vp, vp, u64], i32),
            "rf_sha_streams_digest": ([vp, vp, u64, vp], i32),
            "rf_sha_streams_len": ([vp, u64, vp], i32),
            "rf_sha_streams_verify": ([vp, vp, vp, u64, vp], i32),
            "rf_sha256_verify": ([vp, vp, vp, u64, vp, vp], i32),
            "rf_flow_dirty": ([vp, u64, vp, vp, vp, i32, vp], i32),
            "rf_graph_set_part": ([vp, vp], i32),
            "rf_graph_recompute_part": ([vp, vp, vp, vp, i32, vp], i32),
            "rf_graph_part_gathered": ([vp, vp, vp, vp], i32),
            "rf_graph_split": ([vp, i32, i32, vp, vp], i32), "rf_graph_piece_free": ([vp], None),
            "rf_graph_piece_desc": ([vp, vp], i32), "rf_graph_piece_part": ([vp, vp], i32),
            "rf_graph_piece_slots": ([vp, vp, vp], i32),
            "rf_host_info": ([vp, vp, vp, vp], i32), "rf_host_rate": ([vp, vp, vp], i32),
            "rf_host_link": ([vp, vp, vp], i32),
            "rf_bloom_parse_binary": ([vp, u64, vp, vp, vp, vp, u64, vp], i32),
            "rf_bloom_parse_json": ([vp, u64, vp, vp, vp, vp, u64, vp], i32),
            "rf_bloom_format_binary": ([u64, u64, u64, vp, u64, vp, u64, vp], i32),
            "rf_bloom_format_json": ([u64, u64, u64, vp, u64, vp, u64, vp], i32),
            "rf_coalescer_open": ([vp, i32, vp, i32, u64, u64, vp], i32), "rf_coalescer_close": ([vp], None),
            "rf_coalesce_sha256": ([vp, vp, u64, vp], i32), "rf_coalesce_probe": ([vp, vp, vp], i32),
            "rf_coalesce_assoc_get": ([vp, vp, vp, vp], i32),
            "rf_coalesce_sha256_async": ([vp, vp, u64, vp, vp], i32),
            "rf_coalesce_poll": ([vp, vp, vp], i32), "rf_coalesce_wait": ([vp, vp], i32),
            "rf_coalesce_ticket_free": ([vp, vp], None), "rf_coalescer_stats": ([vp, vp, vp, vp], i32),
            "rf_graph_update_recompute_async": ([vp, vp, vp, u32, vp], i32),
            "rf_walk_dir": ([ctypes.c_char_p, vp], i32), "rf_walk_info": ([vp, vp, vp], i32),
            "rf_walk_entries": ([vp, vp, vp, vp], i32), "rf_walk_free": ([vp], None),
        }
        for name, (args, res) in sigs.items():
            f = getattr(L, name)
            f.argtypes = args
            f.restype = res
        _lib = L
    return _lib


def _check(rc):
    if rc != RF_OK:
        raise RfError(rc, lib().rf_last_error().decode(errors="replace"))


def _ptr(a):
    return None if a is None else a.ctypes.data


def device_count():
    n = ctypes.c_int(0)
    rc = lib().rf_device_count(ctypes.byref(n))
    return n.value if rc == RF_OK else 0


class Context:
    """One rf_ctx bound to one HIP device (one process per GPU).

    host_threads: width of K1's host leg (rf_set_host_threads): None keeps the
    library default (min(60, CPU share)), 0 pins every message to the GPU
    kernels -- what the kernel parity tests use."""

    def __init__(self, device=0, host_threads=None):
        self._h = ctypes.c_void_p()
        _check(lib().rf_init(device, ctypes.byref(self._h)))
        self.device = device
        if host_threads is not None:
            self.set_host_threads(host_threads)

    def set_host_threads(self, n):
        _check(lib().rf_set_host_threads(self._h, -1 if n is None else int(n)))

    def host_info(self):
        """(threads, one core's SHA-NI bytes/s, has SHA extensions)."""
        t, r, e = ctypes.c_int(0), ctypes.c_double(0), ctypes.c_int(0)
        _check(lib().rf_host_info(self._h, ctypes.byref(t), ctypes.byref(r), ctypes.byref(e)))
        return t.value, r.value, bool(e.value)

    def host_link(self):
        """rf_host_link: (bytes/s the planner prices the host leg's HBM feed at,
        whether a run on this context measured it)."""
        r, m = ctypes.c_double(0), ctypes.c_int(0)
        _check(lib().rf_host_link(self._h, ctypes.byref(r), ctypes.byref(m)))
        return r.value, bool(m.value)

    def host_rate(self):
        """(chains per host-leg thread, one thread's measured bytes/s at that interleave)."""
        w, r = ctypes.c_int(0), ctypes.c_double(0)
        _check(lib().rf_host_rate(self._h, ctypes.byref(w), ctypes.byref(r)))
        return w.value, r.value

    def close(self):
        if self._h:
            lib().rf_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    # ---- device memory (HBM owned through the engine's HIP runtime) ------
    def alloc(self, nbytes) -> "DeviceBuffer":
        return DeviceBuffer(self, nbytes)

    def upload(self, arr: np.ndarray) -> "DeviceBuffer":
        arr = np.ascontiguousarray(arr)
        b = DeviceBuffer(self, arr.nbytes)
        b.copy_from(arr)
        return b

    def timer_start(self):
        _check(lib().rf_timer_start(self._h))

    def timer_stop(self) -> float:
        ms = ctypes.c_float(0)
        _check(lib().rf_timer_stop(self._h, ctypes.byref(ms)))
        return ms.value

    @property
    def stream(self):
        return lib().rf_stream(self._h)

    def sync(self):
        _check(lib().rf_sync(self._h))

    # ---- K1 -----------------------------------------------------------
    def sha256_batch(self, msgs):
        """SHA-256 of each bytes object (Digester.FromBytes, batched)."""
        n = len(msgs)
        if n == 0:
            return []
        bufs = [ctypes.create_string_buffer(bytes(m), max(len(m), 1)) for m in msgs]
        ptrs = (ctypes.c_void_p * n)(*[ctypes.addressof(b) for b in bufs])
        lens = np.array([len(m) for m in msgs], dtype=np.uint64)
        out = np.zeros(32 * n, dtype=np.uint8)
        _check(lib().rf_sha256_batch(self._h, ptrs, _ptr(lens), n, _ptr(out)))
        return [out[32 * i:32 * i + 32].tobytes() for i in range(n)]

    def sha256_arena(self, arena: np.ndarray, offs: np.ndarray, lens: np.ndarray) -> np.ndarray:
        n = len(lens)
        out = np.zeros((n, 32), dtype=np.uint8)
        arena = np.ascontiguousarray(arena, dtype=np.uint8)
        offs = np.ascontiguousarray(offs, dtype=np.uint64)
        lens = np.ascontiguousarray(lens, dtype=np.uint64)
        _check(lib().rf_sha256_arena(self._h, _ptr(arena), _ptr(offs), _ptr(lens), n, _ptr(out)))
        return out

    def sha256_verify(self, msgs, want):
        """(rc, status per message) of rf_sha256_verify."""
        n = len(msgs)
        bufs = [ctypes.create_string_buffer(bytes(m), max(len(m), 1)) for m in msgs]
        ptrs = (ctypes.c_void_p * max(n, 1))(*[ctypes.addressof(b) for b in bufs])
        lens = np.array([len(m) for m in msgs] or [0], dtype=np.uint64)
        w = np.frombuffer(b"".join(want) or bytes(32), dtype=np.uint8).copy()
        st = np.zeros(max(n, 1), dtype=np.int32)
        rc = lib().rf_sha256_verify(self._h, ptrs, _ptr(lens), n, _ptr(w), _ptr(st))
        if rc not in (RF_OK, RF_EINTEGRITY):
            _check(rc)
        return rc, st[:n]

    def flow_dirty(self, dep_ptr, deps, is_extern, no_cache_extern=True):
        """rf_flow_dirty: Eval.dirty of every node (bool array)."""
        dp = np.ascontiguousarray(dep_ptr, dtype=np.uint64)
        dv = np.ascontiguousarray(deps, dtype=np.uint32)
        ex = np.ascontiguousarray(is_extern, dtype=np.uint8)
        n = len(dp) - 1
        out = np.zeros(max(n, 1), dtype=np.uint8)
        _check(lib().rf_flow_dirty(self._h, n, _ptr(dp), _ptr(dv) if len(dv) else None, _ptr(ex),
                                   1 if no_cache_extern else 0, _ptr(out)))
        return out[:n].astype(bool)

    def sha_streams(self, n, flags=0):
        return ShaStreams(self, n, flags)

    def sha_plan(self, offs, lens, flags=0):
        return ShaPlan(self, offs, lens, flags)

    def gen_fill(self, d_arena, d_offs, d_lens, n, seed, arena_bytes, stream=None):
        _check(lib().rf_gen_fill(self._h, d_arena, d_offs, d_lens, n, seed & (2**64 - 1),
                                 arena_bytes, stream))

    # ---- Executor.install -------------------------------------------------
    def install_dir(self, root):
        """rf_install_dir: walk `root` (walker.go semantics), digest every file
        on the GPU.  Returns (entries, fileset_digest32) with entries a list of
        (relpath bytes, id32, size) in walk order (local/executor.go:514-557)."""
        h = ctypes.c_void_p()
        r = root.encode() if isinstance(root, str) else root
        _check(lib().rf_install_dir(self._h, r, ctypes.byref(h)))
        try:
            n, pb = ctypes.c_uint64(0), ctypes.c_uint64(0)
            fs = np.zeros(32, dtype=np.uint8)
            _check(lib().rf_install_info(h, ctypes.byref(n), ctypes.byref(pb), _ptr(fs)))
            n, pb = n.value, pb.value
            paths = np.zeros(max(pb, 1), dtype=np.uint8)
            offs = np.zeros(n + 1, dtype=np.uint64)
            ids = np.zeros(max(32 * n, 1), dtype=np.uint8)
            sizes = np.zeros(max(n, 1), dtype=np.int64)
            _check(lib().rf_install_entries(h, _ptr(paths), _ptr(offs), _ptr(ids), _ptr(sizes)))
        finally:
            lib().rf_install_destroy(h)
        pbytes = paths.tobytes()
        ents = [(pbytes[int(offs[i]):int(offs[i + 1])], ids[32 * i:32 * i + 32].tobytes(), int(sizes[i]))
                for i in range(n)]
        return ents, fs.tobytes()

    # ---- Fileset --------------------------------------------------------
    def fileset_digest_batch(self, sets):
        """sets: list of filesets, each a list of groups (a Map is one group,
        a List its flattened Map leaves); a group is a list of (path, id32)."""
        set_group = [0]
        group_entry = [0]
        paths, ids = [], []
        for groups in sets:
            for g in groups:
                for path, id32 in g:
                    paths.append(path.encode() if isinstance(path, str) else path)
                    ids.append(id32)
                group_entry.append(len(paths))
            set_group.append(len(group_entry) - 1)
        n = len(sets)
        sg = np.array(set_group, dtype=np.uint64)
        ge = np.array(group_entry, dtype=np.uint64)
        pb = [ctypes.create_string_buffer(p, max(len(p), 1)) for p in paths]
        pp = (ctypes.c_void_p * max(len(paths), 1))(*[ctypes.addressof(b) for b in pb])
        pl = np.array([len(p) for p in paths] or [0], dtype=np.uint32)
        idb = np.frombuffer(b"".join(ids) or b"\0" * 32, dtype=np.uint8).copy()
        out = np.zeros(32 * n, dtype=np.uint8)
        _check(lib().rf_fileset_digest_batch(self._h, n, _ptr(sg), _ptr(ge), pp, _ptr(pl),
                                             _ptr(idb), _ptr(out)))
        return [out[32 * i:32 * i + 32].tobytes() for i in range(n)]

    def fileset_paths(self, sets):
        """Marshals the paths of `sets` once (groups of paths; entry e = the
        e-th path in order) for repeated digests with device-resident IDs."""
        return FilesetPaths(self, sets)

    def dedup_digests(self, digests: np.ndarray):
        """Canonicalize's flowMap: (canon[i] = first index with digest i's value, n_unique)."""
        d = np.ascontiguousarray(digests, dtype=np.uint8).reshape(-1)
        n = len(d) // 32
        canon = np.zeros(max(n, 1), dtype=np.uint32)
        nu = ctypes.c_uint32(0)
        _check(lib().rf_dedup_digests(self._h, _ptr(d), n, _ptr(canon), ctypes.byref(nu)))
        return canon[:n], nu.value

    def dedup_digests_device(self, d_digests, n, d_canon, d_n_unique, stream=None):
        _check(lib().rf_dedup_digests_device(self._h, d_digests, n, d_canon, d_n_unique, stream))

    def fileset_value_digests(self, sets):
        """SHA256(json.Marshal(fs)) per fileset: CacheWrite's assoc values."""
        if not sets:
            return []
        b = FilesetTreeBuilder()
        roots = np.array([b.add(fs) for fs in sets], dtype=np.uint32)
        t = b.struct()
        out = np.zeros(32 * len(sets), dtype=np.uint8)
        _check(lib().rf_fileset_value_digest_batch(self._h, ctypes.byref(t), _ptr(roots), len(sets),
                                                   _ptr(out)))
        return [out[32 * i:32 * i + 32].tobytes() for i in range(len(sets))]


class ShaStreams:
    """rf_sha_streams: n streaming SHA-256 writers (Digester.NewWriter)."""

    def __init__(self, ctx, n, flags=0):
        self.ctx = ctx
        self._h = ctypes.c_void_p()
        _check(lib().rf_sha_streams_open(ctx.handle, n, flags, ctypes.byref(self._h)))

    def write(self, ids, chunks):
        """chunks[i] (bytes) to stream ids[i], in order."""
        n = len(ids)
        if n == 0:
            return
        bufs = [ctypes.create_string_buffer(bytes(c), max(len(c), 1)) for c in chunks]
        ptrs = (ctypes.c_void_p * n)(*[ctypes.addressof(b) for b in bufs])
        lens = np.array([len(c) for c in chunks], dtype=np.uint64)
        idv = np.ascontiguousarray(ids, dtype=np.uint64)
        _check(lib().rf_sha_streams_write(self._h, _ptr(idv), ptrs, _ptr(lens), n))

    def digest(self, ids):
        idv = np.ascontiguousarray(ids, dtype=np.uint64)
        out = np.zeros(32 * max(len(idv), 1), dtype=np.uint8)
        _check(lib().rf_sha_streams_digest(self._h, _ptr(idv), len(idv), _ptr(out)))
        return [out[32 * i:32 * i + 32].tobytes() for i in range(len(idv))]

    def length(self, i):
        n = ctypes.c_uint64(0)
        _check(lib().rf_sha_streams_len(self._h, i, ctypes.byref(n)))
        return n.value

    def verify(self, ids, want):
        """(rc, status per stream): rc RF_OK or RF_EINTEGRITY."""
        idv = np.ascontiguousarray(ids, dtype=np.uint64)
        w = np.frombuffer(b"".join(want), dtype=np.uint8).copy()
        st = np.zeros(max(len(idv), 1), dtype=np.int32)
        rc = lib().rf_sha_streams_verify(self._h, _ptr(idv), _ptr(w), len(idv), _ptr(st))
        if rc not in (RF_OK, RF_EINTEGRITY):
            _check(rc)
        return rc, st[:len(idv)]

    def close(self):
        if self._h:
            lib().rf_sha_streams_close(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class DeviceBuffer:
    """HBM allocated through rf_malloc; .ptr is the device address."""

    def __init__(self, ctx: Context, nbytes):
        self.ctx = ctx
        self.nbytes = int(nbytes)
        p = ctypes.c_void_p()
        _check(lib().rf_malloc(ctx.handle, self.nbytes, ctypes.byref(p)))
        self._p = p

    @property
    def ptr(self):
        return self._p.value

    def copy_from(self, arr: np.ndarray):
        arr = np.ascontiguousarray(arr)
        assert arr.nbytes <= self.nbytes
        _check(lib().rf_memcpy_h2d(self.ctx.handle, self._p, arr.ctypes.data, arr.nbytes))

    def to_numpy(self, dtype=np.uint8, count=None, offset=0) -> np.ndarray:
        """count elements of dtype from byte `offset` (default: the rest)."""
        dt = np.dtype(dtype)
        n = (self.nbytes - offset) // dt.itemsize if count is None else count
        assert 0 <= offset and offset + n * dt.itemsize <= self.nbytes
        out = np.empty(n, dtype=dt)
        _check(lib().rf_memcpy_d2h(self.ctx.handle, out.ctypes.data, ctypes.c_void_p(self.ptr + offset),
                                   out.nbytes))
        return out

    def zero(self):
        _check(lib().rf_memset_d(self.ctx.handle, self._p, 0, self.nbytes))

    def free(self):
        if self._p and self._p.value:
            lib().rf_free(self.ctx.handle, self._p)
            self._p = ctypes.c_void_p()

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class Comm:
    """RCCL communicator (one rank per GPU) inside the engine."""

    @staticmethod
    def unique_id() -> bytes:
        b = ctypes.create_string_buffer(128)
        _check(lib().rf_comm_unique_id(b))
        return b.raw

    def __init__(self, ctx: Context, nranks, rank, uid: bytes):
        self.ctx = ctx
        self._h = ctypes.c_void_p()
        _check(lib().rf_comm_init(ctx.handle, nranks, rank, ctypes.c_char_p(uid), ctypes.byref(self._h)))

    def allgather(self, d_send, d_recv, nbytes, stream=None):
        _check(lib().rf_comm_allgather(self._h, d_send, d_recv, nbytes, stream))

    def allreduce_or(self, d_words, nwords, stream=None):
        _check(lib().rf_comm_allreduce_or(self._h, d_words, nwords, stream))

    def close(self):
        if self._h:
            lib().rf_comm_destroy(self._h)
            self._h = ctypes.c_void_p()


class ShaPlan:
    def __init__(self, ctx: Context, offs, lens, flags=0):
        self.ctx = ctx
        self._offs = np.ascontiguousarray(offs, dtype=np.uint64)
        self._lens = np.ascontiguousarray(lens, dtype=np.uint64)
        self._h = ctypes.c_void_p()
        _check(lib().rf_sha_plan_create(ctx.handle, _ptr(self._offs), _ptr(self._lens),
                                        len(self._lens), flags, ctypes.byref(self._h)))

    def run(self, d_arena: int, d_out: int, stream=None):
        _check(lib().rf_sha_plan_run(self._h, d_arena, d_out, stream))

    def stats(self) -> ShaStats:
        s = ShaStats()
        _check(lib().rf_sha_plan_stats(self._h, ctypes.byref(s)))
        return s

    def close(self):
        if self._h:
            lib().rf_sha_plan_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Graph:
    """rf_graph: jobs over digest slots (see include/reflow_hip.h)."""

    def __init__(self, ctx: Context, n_slots, out_slot, tmpl_off, tmpl_len, hole_ptr, hole_pos,
                 hole_slot, blob: bytes | np.ndarray):
        self.ctx = ctx
        self._keep = dict(
            out_slot=np.ascontiguousarray(out_slot, dtype=np.uint32),
            tmpl_off=np.ascontiguousarray(tmpl_off, dtype=np.uint64),
            tmpl_len=np.ascontiguousarray(tmpl_len, dtype=np.uint32),
            hole_ptr=np.ascontiguousarray(hole_ptr, dtype=np.uint64),
            hole_pos=np.ascontiguousarray(hole_pos, dtype=np.uint32),
            hole_slot=np.ascontiguousarray(hole_slot, dtype=np.uint32),
            blob=np.frombuffer(bytes(blob), dtype=np.uint8) if isinstance(blob, (bytes, bytearray))
            else np.ascontiguousarray(blob, dtype=np.uint8),
        )
        k = self._keep
        d = GraphDesc(len(k["out_slot"]), n_slots, _ptr(k["out_slot"]), _ptr(k["tmpl_off"]),
                      _ptr(k["tmpl_len"]), _ptr(k["hole_ptr"]),
                      _ptr(k["hole_pos"]) if len(k["hole_pos"]) else None,
                      _ptr(k["hole_slot"]) if len(k["hole_slot"]) else None,
                      _ptr(k["blob"]) if len(k["blob"]) else None, len(k["blob"]))
        self._h = ctypes.c_void_p()
        _check(lib().rf_graph_load(ctx.handle, ctypes.byref(d), ctypes.byref(self._h)))
        self._keep = None  # not retained by the library

    def set_slots(self, slots, digests: np.ndarray):
        slots = np.ascontiguousarray(slots, dtype=np.uint32)
        dg = np.ascontiguousarray(digests, dtype=np.uint8).reshape(-1)
        _check(lib().rf_graph_set_slots(self._h, _ptr(slots), _ptr(dg), len(slots)))

    def set_slots_device(self, d_slots, d_digests, n, stream=None):
        _check(lib().rf_graph_set_slots_device(self._h, d_slots, d_digests, n, stream))

    def recompute(self, full=False) -> int:
        n = ctypes.c_uint64(0)
        _check(lib().rf_graph_recompute(self._h, 1 if full else 0, ctypes.byref(n)))
        return n.value

    def recompute_async(self, full=False, stream=None):
        _check(lib().rf_graph_recompute_async(self._h, 1 if full else 0, stream))

    def update_recompute_async(self, d_slots, d_digests32, n, stream=None):
        """set_slots_device + recompute_async(full=False) as one graph launch."""
        _check(lib().rf_graph_update_recompute_async(self._h, d_slots, d_digests32, n, stream))

    def gather_device(self, d_slots, n, d_out, stream=None):
        _check(lib().rf_graph_gather_device(self._h, d_slots, n, d_out, stream))

    def get_slots(self, slots) -> np.ndarray:
        slots = np.ascontiguousarray(slots, dtype=np.uint32)
        out = np.zeros((len(slots), 32), dtype=np.uint8)
        _check(lib().rf_graph_get_slots(self._h, _ptr(slots), len(slots), _ptr(out)))
        return out

    def stats(self) -> GraphStats:
        s = GraphStats()
        _check(lib().rf_graph_stats_get(self._h, ctypes.byref(s)))
        return s

    def adopt_slots(self, src):
        """rf_graph_adopt_slots: take src's whole slot table (same numbering),
        ready for incremental steps without a full recompute."""
        _check(lib().rf_graph_adopt_slots(self._h, src._h))

    # kernel-form thresholds (include/reflow_hip.h RF_K2_THRU*_DEFAULT)
    THRU_DEFAULT, THRU_WIDE_DEFAULT, THRU_MARK_DEFAULT = 24576, 65536, 98304
    NEVER = (1 << 64) - 1

    def set_forms(self, thru, thru_wide=None, thru_mark=None):
        """rf_graph_set_forms: 0 = always the throughput form, Graph.NEVER =
        never; thru_wide / thru_mark default to thru."""
        _check(lib().rf_graph_set_forms(self._h, int(thru), int(thru if thru_wide is None else thru_wide),
                                        int(thru if thru_mark is None else thru_mark)))

    def save(self, path):
        """rf_graph_save: the lowered graph and its slot digests to `path`."""
        _check(lib().rf_graph_save(self._h, os.fsencode(path)))

    @classmethod
    def restore(cls, ctx, path):
        """rf_graph_restore: a graph saved by save(), ready for incremental steps."""
        g = cls.__new__(cls)
        g.ctx, g._keep = ctx, None
        g._h = ctypes.c_void_p()
        _check(lib().rf_graph_restore(ctx.handle, os.fsencode(path), ctypes.byref(g._h)))
        return g

    @classmethod
    def from_arrays(cls, ctx, a):
        return cls(ctx, a["n_slots"], a["out_slot"], a["tmpl_off"], a["tmpl_len"], a["hole_ptr"], a["hole_pos"],
                   a["hole_slot"], a["blob"])

    def set_part(self, part):
        """part: dict(nranks, rank, max_export, export_slot, import_slot,
        import_bid, any_import[, rounds]) (GraphPiece.part); rounds > 0 selects
        the fixed-round exchange (0: supersteps until nothing changes)."""
        ex = np.ascontiguousarray(part["export_slot"], dtype=np.uint32)
        im = np.ascontiguousarray(part["import_slot"], dtype=np.uint32)
        ib = np.ascontiguousarray(part["import_bid"], dtype=np.uint32)
        p = GraphPart(part["nranks"], part["rank"], part["max_export"], len(ex), _ptr(ex) if len(ex) else None,
                      len(im), _ptr(im) if len(im) else None, _ptr(ib) if len(ib) else None,
                      1 if part.get("any_import", True) else 0, int(part.get("rounds", 0)))
        _check(lib().rf_graph_set_part(self._h, ctypes.byref(p)))

    def recompute_part(self, comm=None, allgather=None, nranks=1, full=False, count=True) -> int:
        """Recompute across ranks: comm (Comm, RCCL) or allgather (bytes ->
        [bytes per rank], a host transport).  count=False: no readback of the
        jobs hashed (with comm and fixed rounds the call is then asynchronous)."""
        fn = host_allgather_fn(allgather, nranks) if allgather is not None else None
        self._fn = fn  # alive during the call
        n = ctypes.c_uint64(0)
        _check(lib().rf_graph_recompute_part(self._h, comm._h if comm is not None else None,
                                             ctypes.cast(fn, ctypes.c_void_p) if fn is not None else None, None,
                                             1 if full else 0, ctypes.byref(n) if count else None))
        return n.value

    def part_gathered(self):
        """(device pointer of the gathered export digests, count, supersteps)."""
        p, n, st = ctypes.c_void_p(), ctypes.c_uint64(), ctypes.c_uint64()
        _check(lib().rf_graph_part_gathered(self._h, ctypes.byref(p), ctypes.byref(n), ctypes.byref(st)))
        return p.value, n.value, st.value

    def close(self):
        if self._h:
            lib().rf_graph_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Bloom:
    """rf_bloom: device-resident willf/bloom filter with bloomlive semantics."""

    def __init__(self, ctx: Context, handle):
        self.ctx = ctx
        self._h = handle

    @classmethod
    def load(cls, ctx, m, k, words: np.ndarray, length):
        h = ctypes.c_void_p()
        w = np.ascontiguousarray(words, dtype=np.uint64)
        _check(lib().rf_bloom_load(ctx.handle, m, k, _ptr(w) if len(w) else None, len(w), length,
                                   ctypes.byref(h)))
        return cls(ctx, h)

    @classmethod
    def new(cls, ctx, m, k):
        h = ctypes.c_void_p()
        _check(lib().rf_bloom_new(ctx.handle, m, k, ctypes.byref(h)))
        return cls(ctx, h)

    @classmethod
    def from_json(cls, ctx, js: bytes):
        h = ctypes.c_void_p()
        _check(lib().rf_bloom_load_json(ctx.handle, js, len(js), ctypes.byref(h)))
        return cls(ctx, h)

    @classmethod
    def from_binary(cls, ctx, buf: bytes):
        h = ctypes.c_void_p()
        b = np.frombuffer(buf, dtype=np.uint8).copy()
        _check(lib().rf_bloom_load_binary(ctx.handle, _ptr(b), len(b), ctypes.byref(h)))
        return cls(ctx, h)

    def probe(self, digests: np.ndarray) -> np.ndarray:
        d = np.ascontiguousarray(digests, dtype=np.uint8).reshape(-1)
        n = len(d) // 32
        out = np.zeros(n, dtype=np.uint8)
        _check(lib().rf_bloom_probe(self._h, _ptr(d), n, _ptr(out)))
        return out

    def probe_device(self, d_digests, n, d_out, stream=None):
        _check(lib().rf_bloom_probe_device(self._h, d_digests, n, d_out, stream))

    def add(self, digests: np.ndarray):
        d = np.ascontiguousarray(digests, dtype=np.uint8).reshape(-1)
        _check(lib().rf_bloom_add(self._h, _ptr(d), len(d) // 32))

    def add_device(self, d_digests, n, stream=None):
        _check(lib().rf_bloom_add_device(self._h, d_digests, n, stream))

    def params(self):
        m, k, ln, nw = (ctypes.c_uint64() for _ in range(4))
        _check(lib().rf_bloom_params(self._h, ctypes.byref(m), ctypes.byref(k), ctypes.byref(ln),
                                     ctypes.byref(nw)))
        return m.value, k.value, ln.value, nw.value

    def words(self) -> np.ndarray:
        _, _, _, nw = self.params()
        out = np.zeros(nw, dtype=np.uint64)
        _check(lib().rf_bloom_words(self._h, _ptr(out) if nw else None, nw))
        return out

    def _marshal(self, fn) -> bytes:
        need = ctypes.c_uint64(0)
        rc = fn(self._h, None, 0, ctypes.byref(need))
        if rc != RF_OK and need.value == 0:
            _check(rc)
        out = ctypes.create_string_buffer(max(need.value, 1))
        _check(fn(self._h, out, need.value, ctypes.byref(need)))
        return out.raw[:need.value]

    def marshal_json(self) -> bytes:
        return self._marshal(lib().rf_bloom_marshal_json)

    def marshal_binary(self) -> bytes:
        return self._marshal(lib().rf_bloom_marshal_binary)

    def collect(self, digests: np.ndarray, sizes=None):
        """Repository.Collect over a batch: (ascending dead indices, dead bytes)."""
        d = np.ascontiguousarray(digests, dtype=np.uint8).reshape(-1)
        n = len(d) // 32
        sz = None if sizes is None else np.ascontiguousarray(sizes, dtype=np.int64)
        out = np.zeros(max(n, 1), dtype=np.uint64)
        nd, nb = ctypes.c_uint64(0), ctypes.c_int64(0)
        _check(lib().rf_bloom_collect(self._h, _ptr(d), _ptr(sz), n, _ptr(out), ctypes.byref(nd),
                                      ctypes.byref(nb)))
        return out[:nd.value], nb.value

    def collect_device(self, d_digests, d_sizes, n, d_dead_idx, d_counts2, stream=None):
        _check(lib().rf_bloom_collect_device(self._h, d_digests, d_sizes, n, d_dead_idx, d_counts2, stream))

    def close(self):
        if self._h:
            lib().rf_bloom_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def walk_dir(root):
    """rf_walk_dir (host-only, no device): internal/walker's Scan as install
    uses it -> [(relpath bytes, Stat size)] in walk order."""
    w = ctypes.c_void_p()
    _check(lib().rf_walk_dir(os.fsencode(root), ctypes.byref(w)))
    try:
        n, pb = ctypes.c_uint64(), ctypes.c_uint64()
        _check(lib().rf_walk_info(w, ctypes.byref(n), ctypes.byref(pb)))
        paths = ctypes.create_string_buffer(max(pb.value, 1))
        offs = np.zeros(n.value + 1, np.uint64)
        sizes = np.zeros(n.value + 1, np.int64)
        _check(lib().rf_walk_entries(w, paths, _ptr(offs), _ptr(sizes)))
        raw = paths.raw
        return [(raw[int(offs[i]):int(offs[i + 1])], int(sizes[i])) for i in range(n.value)]
    finally:
        lib().rf_walk_free(w)


RF_COALESCE_SHA256, RF_COALESCE_PROBE, RF_COALESCE_ASSOC_GET = 1, 2, 3


class Coalescer:
    """rf_coalescer: concurrent callers (threads) coalesced into device
    batches.  target: a Bloom (PROBE) or an Assoc (ASSOC_GET)."""

    def __init__(self, ctx, kind, target=None, assoc_kind=0, max_batch=4096, max_wait_us=200):
        self.ctx, self.kind, self.target = ctx, kind, target
        self._h = ctypes.c_void_p()
        _check(lib().rf_coalescer_open(ctx.handle, kind, target._h if target is not None else None, assoc_kind,
                                       max_batch, max_wait_us, ctypes.byref(self._h)))

    def sha256(self, msg: bytes) -> bytes:
        out = ctypes.create_string_buffer(32)
        _check(lib().rf_coalesce_sha256(self._h, msg, len(msg), out))
        return out.raw

    def probe(self, digest32: bytes) -> bool:
        out = ctypes.c_uint8(0)
        _check(lib().rf_coalesce_probe(self._h, digest32, ctypes.byref(out)))
        return bool(out.value)

    def assoc_get(self, key32: bytes):
        val, found = ctypes.create_string_buffer(32), ctypes.c_uint8(0)
        _check(lib().rf_coalesce_assoc_get(self._h, key32, val, ctypes.byref(found)))
        return bool(found.value), val.raw

    def sha256_async(self, msg: bytes):
        """-> ticket (msg and the result buffer are kept alive by it)."""
        buf = ctypes.create_string_buffer(msg, len(msg)) if msg else ctypes.create_string_buffer(1)
        out = ctypes.create_string_buffer(32)
        t = ctypes.c_void_p()
        _check(lib().rf_coalesce_sha256_async(self._h, buf, len(msg), out, ctypes.byref(t)))
        return {"t": t, "buf": buf, "out": out}

    def poll(self, ticket) -> bool:
        done = ctypes.c_int(0)
        _check(lib().rf_coalesce_poll(self._h, ticket["t"], ctypes.byref(done)))
        return bool(done.value)

    def wait(self, ticket) -> bytes:
        _check(lib().rf_coalesce_wait(self._h, ticket["t"]))
        return ticket["out"].raw

    def free(self, ticket):
        lib().rf_coalesce_ticket_free(self._h, ticket["t"])
        ticket["t"] = None

    def stats(self):
        b, r, m = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
        _check(lib().rf_coalescer_stats(self._h, ctypes.byref(b), ctypes.byref(r), ctypes.byref(m)))
        return b.value, r.value, m.value

    def close(self):
        if self._h:
            lib().rf_coalescer_close(self._h)
            self._h = ctypes.c_void_p()


class Assoc:
    """HBM assoc (assoc.Assoc with the in-memory assoc's semantics)."""

    def __init__(self, ctx: Context, capacity=1024):
        self.ctx = ctx
        self._h = ctypes.c_void_p()
        _check(lib().rf_assoc_new(ctx.handle, capacity, ctypes.byref(self._h)))

    def put(self, kind, keys, vals, expect=None) -> np.ndarray:
        k = np.ascontiguousarray(keys, dtype=np.uint8).reshape(-1)
        v = np.ascontiguousarray(vals, dtype=np.uint8).reshape(-1)
        e = None if expect is None else np.ascontiguousarray(expect, dtype=np.uint8).reshape(-1)
        n = len(k) // 32
        st = np.zeros(max(n, 1), dtype=np.int32)
        _check(lib().rf_assoc_put(self._h, kind, _ptr(e), _ptr(k), _ptr(v), n, _ptr(st)))
        return st[:n]

    def get(self, kind, keys):
        k = np.ascontiguousarray(keys, dtype=np.uint8).reshape(-1)
        n = len(k) // 32
        vals = np.zeros((max(n, 1), 32), dtype=np.uint8)
        found = np.zeros(max(n, 1), dtype=np.uint8)
        _check(lib().rf_assoc_get(self._h, kind, _ptr(k), n, _ptr(vals), _ptr(found)))
        return vals[:n], found[:n]

    def lookup(self, kind, keys, key_ptr):
        """rf_assoc_lookup (read only): keys (rows of 32 B) grouped per node by
        key_ptr (n_nodes + 1 offsets).  Returns (which int32 per node, values,
        found per key, value per key)."""
        k = np.ascontiguousarray(keys, dtype=np.uint8).reshape(-1)
        kp = np.ascontiguousarray(key_ptr, dtype=np.uint64)
        n, nk = len(kp) - 1, len(k) // 32
        which = np.zeros(max(n, 1), dtype=np.int32)
        vals = np.zeros((max(n, 1), 32), dtype=np.uint8)
        kf = np.zeros(max(nk, 1), dtype=np.uint8)
        kv = np.zeros((max(nk, 1), 32), dtype=np.uint8)
        _check(lib().rf_assoc_lookup(self._h, kind, _ptr(k) if len(k) else None, _ptr(kp), n, _ptr(which),
                                     _ptr(vals), _ptr(kf), _ptr(kv)))
        return which[:n], vals[:n], kf[:nk], kv[:nk]

    def repair(self, kind, keys, key_ptr, which, vals, key_found=None):
        """rf_assoc_repair: read repair of the nodes with which >= 0 (blind, or
        precise with key_found)."""
        k = np.ascontiguousarray(keys, dtype=np.uint8).reshape(-1)
        kp = np.ascontiguousarray(key_ptr, dtype=np.uint64)
        w = np.ascontiguousarray(which, dtype=np.int32)
        v = np.ascontiguousarray(vals, dtype=np.uint8).reshape(-1)
        kf = None if key_found is None else np.ascontiguousarray(key_found, dtype=np.uint8)
        _check(lib().rf_assoc_repair(self._h, kind, _ptr(k) if len(k) else None, _ptr(kp), len(kp) - 1, _ptr(w),
                                     _ptr(v), _ptr(kf) if kf is not None and len(kf) else None))

    def put_device(self, kind, d_keys, d_vals, n, d_status, d_expect=None):
        _check(lib().rf_assoc_put_device(self._h, kind, d_expect, d_keys, d_vals, n, d_status))

    def get_device(self, kind, d_keys, n, d_vals, d_found, stream=None):
        _check(lib().rf_assoc_get_device(self._h, kind, d_keys, n, d_vals, d_found, stream))

    def get_abbrev(self, kind, keys, nhex):
        k = np.ascontiguousarray(keys, dtype=np.uint8).reshape(-1)
        n = len(k) // 32
        nh = np.ascontiguousarray(nhex, dtype=np.uint8)
        ko = np.zeros((max(n, 1), 32), dtype=np.uint8)
        vo = np.zeros((max(n, 1), 32), dtype=np.uint8)
        st = np.zeros(max(n, 1), dtype=np.int32)
        _check(lib().rf_assoc_get_abbrev(self._h, kind, _ptr(k), _ptr(nh), n, _ptr(ko), _ptr(vo), _ptr(st)))
        return ko[:n], vo[:n], st[:n]

    def stats(self):
        o, c = ctypes.c_uint64(), ctypes.c_uint64()
        _check(lib().rf_assoc_stats(self._h, ctypes.byref(o), ctypes.byref(c)))
        return o.value, c.value

    def close(self):
        if self._h:
            lib().rf_assoc_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
