"""ctypes binding of libpfaai_hip.so (include/pfaai_hip.h).

This is the only way the Python mirror reaches the engine: every compute
call goes through the C ABI into the HIP kernels.  There is no CPU
fallback -- if the library is missing or no GPU is visible, calls raise.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

try:  # one HIP runtime per process: torch's bundled libamdhip64 must win
    import torch  # noqa: F401
except Exception:  # pragma: no cover - torch is optional for the binding
    torch = None

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PFAAI_HIP_LIB", os.path.join(_HERE, "lib", "libpfaai_hip.so"))
# the same engine built with -DPFAAI_DIAGNOSTICS: the A/B switches (PFAAI_ROWS_KERNEL,
# PFAAI_PL_WINDOWS, PFAAI_PL_V, ...) exist only here (tests of the variants, tools/gpu)
DIAG_LIB_PATH = os.path.join(_HERE, "lib", "libpfaai_hip_diag.so")

NTETRAMERS = 160000
ABI_VERSION = 6  # PFAAI_ABI_VERSION of include/pfaai_hip.h
PFAAI_OK = 0
ERR_NAMES = {1: "SQLITE_DB", 2: "SQLITE_MEM_ALLOC", 3: "CONSTRUCT", 4: "HIP", 5: "OOM", 6: "RCCL", 7: "INVALID"}
MODE_ALL, MODE_QSUB, MODE_QT = 0, 1, 2
FLAG_REF_COMPAT = 1
FLAG_EMIT_JAC = 2
FLAG_KEEP_RUNS = 4
FLAG_FULL_ROWS = 8

# every symbol include/pfaai_hip.h declares
EXPORTS = [
    "pfaai_version", "pfaai_create", "pfaai_destroy", "pfaai_last_error", "pfaai_load",
    "pfaai_shape", "pfaai_row_span", "pfaai_run", "pfaai_compute", "pfaai_last_stats",
    "pfaai_debug_row_counts", "pfaai_debug_div_check", "pfaai_debug_clocks", "pfaai_device_alloc", "pfaai_device_free", "pfaai_memcpy_d2h",
    "pfaai_synchronize", "pfaai_timing", "pfaai_stream", "pfaai_stream_events",
    "pfaai_build_f", "pfaai_compute_rows", "pfaai_run_info", "pfaai_run_walk", "pfaai_load_rows", "pfaai_load_timing", "pfaai_stream_matrix",
    "pfaai_load_info", "pfaai_set_row_order",
    "pfaai_group_create", "pfaai_group_create_flags", "pfaai_group_destroy", "pfaai_group_last_error",
    "pfaai_group_size", "pfaai_group_ctx", "pfaai_group_load", "pfaai_group_blocks", "pfaai_group_run",
]
GROUP_PEER_GATHER = 1  # pfaai_group_create_flags
LOAD_PATHS = {0: "as_given", 1: "g_checked", 2: "g_from_f", 3: "f_from_g", 4: "legacy"}
ROWS_KERNELS = {0: "pl", 1: "pl512", 2: "fused", 3: "worklist"}
WALKS = {-1: "none", 0: "splitters", 3: "gpos", 4: "spans"}  # pfaai_run_walk

# int sink(void* user, i64 row_begin, i64 row_end, i64 first, i64 count, const double* aji,
#          const double* S, const int32_t* N)   (pfaai_sink_fn)
SINK_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
                           ctypes.c_int64, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                           ctypes.POINTER(ctypes.c_int32))

# int sink(void* user, i64 row_begin, i64 row_end, i64 n_cols, const double* block)  (pfaai_matrix_sink_fn)
MATRIX_SINK_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
                                  ctypes.POINTER(ctypes.c_double))


class PfaaiError(RuntimeError):
    def __init__(self, code: int, msg: str = ""):
        super().__init__(f"pfaai error {code} ({ERR_NAMES.get(code, '?')}): {msg}")
        self.code = code


class Problem(ctypes.Structure):
    _fields_ = [
        ("mode", ctypes.c_int32), ("n_ids", ctypes.c_int32), ("n_prot", ctypes.c_int32),
        ("t_cols", ctypes.c_int32), ("n_qry", ctypes.c_int32), ("n_tgt", ctypes.c_int32),
        ("n_f", ctypes.c_int64),
        ("Lp", ctypes.c_void_p), ("F_prot", ctypes.c_void_p), ("F_genome", ctypes.c_void_p),
        ("T", ctypes.c_void_p), ("is_q", ctypes.c_void_p), ("q_index", ctypes.c_void_p),
        ("t_rank", ctypes.c_void_p), ("G_off", ctypes.c_void_p), ("G_tet", ctypes.c_void_p),
    ]


_libs = {}


def load_library(path=None):
    """Load libpfaai_hip.so, or the library at `path` (e.g. DIAG_LIB_PATH);
    raises if it was not built: no fallback."""
    path = path or LIB_PATH
    if path in _libs:
        return _libs[path]
    if not os.path.exists(path):
        raise RuntimeError(f"{os.path.basename(path)} not found at {path}; run __graft_entry__.build()")
    lib = ctypes.CDLL(path)
    vp, i32, i64, u32 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_uint32
    P64 = ctypes.POINTER(ctypes.c_int64)
    sig = {
        "pfaai_version": (ctypes.c_int, []),
        "pfaai_create": (ctypes.c_int, [ctypes.POINTER(vp), ctypes.c_int]),
        "pfaai_destroy": (ctypes.c_int, [vp]),
        "pfaai_last_error": (ctypes.c_char_p, [vp]),
        "pfaai_load": (ctypes.c_int, [vp, ctypes.POINTER(Problem)]),
        "pfaai_load_rows": (ctypes.c_int, [vp, ctypes.POINTER(Problem), i64, i64]),
        "pfaai_shape": (ctypes.c_int, [vp, P64, P64]),
        "pfaai_row_span": (ctypes.c_int, [vp, i64, i64, P64, P64]),
        "pfaai_run": (ctypes.c_int, [vp, i64, i64, u32, vp, vp, vp, vp]),
        "pfaai_compute": (ctypes.c_int, [vp, u32, vp, vp, vp]),
        "pfaai_last_stats": (ctypes.c_int, [vp, P64, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_float)]),
        "pfaai_debug_row_counts": (ctypes.c_int, [vp, i64, vp]),
        "pfaai_debug_div_check": (ctypes.c_int, [vp, ctypes.c_int32, ctypes.c_int32, vp]),
        "pfaai_debug_clocks": (ctypes.c_int, [vp, vp, ctypes.c_int64]),
        "pfaai_device_alloc": (ctypes.c_int, [vp, ctypes.POINTER(vp), i64]),
        "pfaai_device_free": (ctypes.c_int, [vp, vp]),
        "pfaai_memcpy_d2h": (ctypes.c_int, [vp, vp, vp, i64]),
        "pfaai_synchronize": (ctypes.c_int, [vp]),
        "pfaai_compute_rows": (ctypes.c_int, [vp, i64, i64, u32, vp, vp, vp]),
        "pfaai_build_f": (ctypes.c_int, [vp, vp, vp, vp, i64, i32, i32, vp, vp, vp, vp, vp]),
        "pfaai_stream": (ctypes.c_int, [vp, i64, i64, i64, u32, SINK_FN, vp]),
        "pfaai_stream_events": (ctypes.c_int, [vp, P64]),
        "pfaai_stream_matrix": (ctypes.c_int, [vp, i64, i64, i64, u32, MATRIX_SINK_FN, vp]),
        "pfaai_run_info": (ctypes.c_int, [vp, ctypes.POINTER(i32), ctypes.POINTER(i32)]),
        "pfaai_run_walk": (ctypes.c_int, [vp, ctypes.POINTER(i32), ctypes.POINTER(i32)]),
        "pfaai_set_row_order": (ctypes.c_int, [vp, vp, i64]),
        "pfaai_load_timing": (ctypes.c_int, [vp, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                                             ctypes.POINTER(ctypes.c_double)]),
        "pfaai_load_info": (ctypes.c_int, [vp, ctypes.POINTER(i32)]),
        "pfaai_timing": (ctypes.c_int, [vp, ctypes.c_int, ctypes.POINTER(i32), ctypes.POINTER(ctypes.c_double),
                                        ctypes.POINTER(ctypes.c_double)]),
        "pfaai_group_create": (ctypes.c_int, [ctypes.POINTER(vp), ctypes.POINTER(ctypes.c_int), ctypes.c_int]),
        "pfaai_group_create_flags": (ctypes.c_int, [ctypes.POINTER(vp), ctypes.POINTER(ctypes.c_int), ctypes.c_int, u32]),
        "pfaai_group_destroy": (ctypes.c_int, [vp]),
        "pfaai_group_last_error": (ctypes.c_char_p, [vp]),
        "pfaai_group_size": (ctypes.c_int, [vp, ctypes.POINTER(ctypes.c_int)]),
        "pfaai_group_ctx": (vp, [vp, ctypes.c_int]),
        "pfaai_group_load": (ctypes.c_int, [vp, ctypes.POINTER(Problem)]),
        "pfaai_group_blocks": (ctypes.c_int, [vp, P64]),
        "pfaai_group_run": (ctypes.c_int, [vp, u32, vp, vp, vp]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype, fn.argtypes = res, args
    _libs[path] = lib
    return lib


def _ptr(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def _problem(*, mode, n_ids, n_prot, T, Lp=None, F_prot=None, F_genome=None, n_qry=0, n_tgt=0, is_q=None,
             q_index=None, t_rank=None, G_off=None, G_tet=None):
    """-> (pfaai_problem, the contiguous arrays it points into: keep them alive)"""
    Lp = None if Lp is None else np.ascontiguousarray(Lp, dtype=np.int64)
    F_prot = None if F_prot is None else np.ascontiguousarray(F_prot, dtype=np.int32)
    F_genome = None if F_genome is None else np.ascontiguousarray(F_genome, dtype=np.int32)
    T = np.ascontiguousarray(T, dtype=np.int32)
    is_q = None if is_q is None else np.ascontiguousarray(is_q, dtype=np.uint8)
    q_index = None if q_index is None else np.ascontiguousarray(q_index, dtype=np.int32)
    t_rank = None if t_rank is None else np.ascontiguousarray(t_rank, dtype=np.int32)
    G_off = None if G_off is None else np.ascontiguousarray(G_off, dtype=np.int64)
    G_tet = None if G_tet is None else np.ascontiguousarray(G_tet, dtype=np.int32)
    assert Lp is None or Lp.shape == (NTETRAMERS + 1,)
    assert T.ndim == 2 and T.shape[0] == n_prot
    pb = Problem(mode=mode, n_ids=n_ids, n_prot=n_prot, t_cols=T.shape[1], n_qry=n_qry,
                 n_tgt=n_tgt, n_f=0 if F_prot is None else F_prot.shape[0], Lp=_ptr(Lp), F_prot=_ptr(F_prot),
                 F_genome=_ptr(F_genome), T=_ptr(T), is_q=_ptr(is_q), q_index=_ptr(q_index),
                 t_rank=_ptr(t_rank), G_off=_ptr(G_off), G_tet=_ptr(G_tet))
    return pb, (Lp, F_prot, F_genome, T, is_q, q_index, t_rank, G_off, G_tet)


class Engine:
    """One pfaai_ctx = one device.  Owns the device-resident problem."""

    def __init__(self, device: int = 0, lib_path=None):
        self.lib = load_library(lib_path)
        self.ctx = ctypes.c_void_p()
        rc = self.lib.pfaai_create(ctypes.byref(self.ctx), int(device))
        if rc != PFAAI_OK:
            raise PfaaiError(rc, f"pfaai_create(device={device}) failed (no visible GPU?)")
        self._keep = None

    def _check(self, rc, what):
        if rc != PFAAI_OK:
            msg = self.lib.pfaai_last_error(self.ctx)
            raise PfaaiError(rc, f"{what}: {msg.decode() if msg else ''}")

    def close(self):
        if self.ctx:
            self.lib.pfaai_destroy(self.ctx)
            self.ctx = ctypes.c_void_p()

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    # -- problem ----------------------------------------------------------------
    def load(self, *, mode, n_ids, n_prot, T, Lp=None, F_prot=None, F_genome=None, n_qry=0, n_tgt=0,
             is_q=None, q_index=None, t_rank=None, G_off=None, G_tet=None, rows=None):
        """F (Lp, F_prot, F_genome) and/or G (G_off, G_tet): whichever is
        missing is built on the device (pfaai_load).  rows=(begin, end): the
        output rows this context will run (pfaai_load_rows: a rank's block;
        the all-vs-all walk data is built for those rows only)."""
        pb, keep = _problem(mode=mode, n_ids=n_ids, n_prot=n_prot, T=T, Lp=Lp, F_prot=F_prot,
                            F_genome=F_genome, n_qry=n_qry, n_tgt=n_tgt, is_q=is_q, q_index=q_index,
                            t_rank=t_rank, G_off=G_off, G_tet=G_tet)  # (keep: borrowed for the call only)
        if rows is None:
            self._check(self.lib.pfaai_load(self.ctx, ctypes.byref(pb)), "pfaai_load")
        else:
            self._check(self.lib.pfaai_load_rows(self.ctx, ctypes.byref(pb), int(rows[0]), int(rows[1])),
                        "pfaai_load_rows")

    def shape(self):
        r, p = ctypes.c_int64(), ctypes.c_int64()
        self._check(self.lib.pfaai_shape(self.ctx, ctypes.byref(r), ctypes.byref(p)), "pfaai_shape")
        return r.value, p.value

    def row_span(self, row_begin, row_end):
        f, c = ctypes.c_int64(), ctypes.c_int64()
        self._check(self.lib.pfaai_row_span(self.ctx, row_begin, row_end, ctypes.byref(f), ctypes.byref(c)),
                    "pfaai_row_span")
        return f.value, c.value

    # -- compute ------------------------------------------------------------------
    def compute(self, flags: int = 0):
        """All rows; returns host (aji, S, N) in JAC-index order."""
        _, np_ = self.shape()
        aji = np.empty(np_, dtype=np.float64)
        S = np.empty(np_, dtype=np.float64)
        N = np.empty(np_, dtype=np.int32)
        self._check(self.lib.pfaai_compute(self.ctx, flags, _ptr(aji), _ptr(S), _ptr(N)), "pfaai_compute")
        return aji, S, N

    def run(self, row_begin, row_end, flags, d_aji, d_S=None, d_N=None, stream=None):
        """Device-resident run; d_* are device pointers (ints), stream a hipStream_t (int)."""
        self._check(self.lib.pfaai_run(self.ctx, row_begin, row_end, flags, d_aji, d_S, d_N, stream),
                    "pfaai_run")

    def set_row_order(self, genomes=None):
        """pfaai_set_row_order: rows [0, len(genomes)) of later runs are these
        genomes (strictly ascending ids, all-vs-all); None -> id order."""
        if genomes is None or len(genomes) == 0:
            self._check(self.lib.pfaai_set_row_order(self.ctx, None, 0), "pfaai_set_row_order")
            return
        g = np.ascontiguousarray(genomes, dtype=np.int32)
        self._check(self.lib.pfaai_set_row_order(self.ctx, g.ctypes.data, len(g)), "pfaai_set_row_order")

    def build_f(self, prot, genome, tetra, n_prot, n_genome, with_T=True):
        """F construction on the device (pfaai_build_f) from (protein, genome,
        tetramer) triples, each protein's in non-decreasing genome order ->
        dict(Lc int32[160000], Lp int64[160001], F_prot, F_genome int32[n],
        T int32[n_prot, n_genome] or None), F by (tetramer, protein, genome)."""
        prot = np.ascontiguousarray(prot, dtype=np.int32)
        genome = np.ascontiguousarray(genome, dtype=np.int32)
        tetra = np.ascontiguousarray(tetra, dtype=np.int32)
        n = prot.shape[0]
        assert genome.shape == (n,) and tetra.shape == (n,)
        Lc = np.zeros(NTETRAMERS, dtype=np.int32)
        Lp = np.zeros(NTETRAMERS + 1, dtype=np.int64)
        Fp = np.empty(max(n, 1), dtype=np.int32)
        Fg = np.empty(max(n, 1), dtype=np.int32)
        T = np.zeros((n_prot, n_genome), dtype=np.int32) if with_T else None
        self._check(self.lib.pfaai_build_f(self.ctx, _ptr(prot), _ptr(genome), _ptr(tetra), n, n_prot, n_genome,
                                           _ptr(Lc), _ptr(Lp), _ptr(Fp), _ptr(Fg), _ptr(T)), "pfaai_build_f")
        return dict(Lc=Lc, Lp=Lp, F_prot=Fp[:n], F_genome=Fg[:n], T=T)

    def stream(self, row_begin, row_end, tile_pairs, flags, sink):
        """Output-tile streaming (pfaai_stream): sink(row_begin, row_end, first,
        aji, S, N) gets numpy views of each tile in row order (valid during the
        call only; S, N are None without FLAG_EMIT_JAC); a truthy return stops
        the stream.  Returns |E| over all tiles."""
        jac = bool(flags & FLAG_EMIT_JAC)
        err = []

        def _cb(_user, rb, re, first, count, aji, S, N):
            try:
                a = np.ctypeslib.as_array(aji, shape=(count,)) if count else np.zeros(0)
                s_ = np.ctypeslib.as_array(S, shape=(count,)) if (jac and count) else None
                n_ = np.ctypeslib.as_array(N, shape=(count,)) if (jac and count) else None
                return 7 if sink(rb, re, first, a, s_, n_) else 0
            except Exception as e:  # surfaced after the call
                err.append(e)
                return 7

        cb = SINK_FN(_cb)
        rc = self.lib.pfaai_stream(self.ctx, row_begin, row_end, int(tile_pairs), flags, cb, None)
        if err:
            raise err[0]
        self._check(rc, "pfaai_stream")
        ne = ctypes.c_int64()
        self._check(self.lib.pfaai_stream_events(self.ctx, ctypes.byref(ne)), "pfaai_stream_events")
        return ne.value

    def stream_matrix(self, row_begin, row_end, tile_rows, flags, sink):
        """Dense output rows (pfaai_stream_matrix): sink(row_begin, row_end,
        block) gets a numpy view [rows, n_cols] of each tile in row order
        (valid during the call); a truthy return stops the stream.  Returns
        |E| over the tiles (both orientations of every pair)."""
        err = []

        def _cb(_user, rb, re, n_cols, block):
            try:
                a = np.ctypeslib.as_array(block, shape=(re - rb, n_cols))
                return 7 if sink(rb, re, a) else 0
            except Exception as e:  # surfaced after the call
                err.append(e)
                return 7

        cb = MATRIX_SINK_FN(_cb)
        rc = self.lib.pfaai_stream_matrix(self.ctx, row_begin, row_end, int(tile_rows), flags, cb, None)
        if err:
            raise err[0]
        self._check(rc, "pfaai_stream_matrix")
        ne = ctypes.c_int64()
        self._check(self.lib.pfaai_stream_events(self.ctx, ctypes.byref(ne)), "pfaai_stream_events")
        return ne.value

    def stats(self):
        ne, mb, mr = ctypes.c_int64(), ctypes.c_float(), ctypes.c_float()
        self._check(self.lib.pfaai_last_stats(self.ctx, ctypes.byref(ne), ctypes.byref(mb), ctypes.byref(mr)),
                    "pfaai_last_stats")
        rk, win = ctypes.c_int32(), ctypes.c_int32()
        self._check(self.lib.pfaai_run_info(self.ctx, ctypes.byref(rk), ctypes.byref(win)), "pfaai_run_info")
        wk, nar = ctypes.c_int32(), ctypes.c_int32()
        self._check(self.lib.pfaai_run_walk(self.ctx, ctypes.byref(wk), ctypes.byref(nar)), "pfaai_run_walk")
        return {"n_events": ne.value, "ms_build": mb.value, "ms_rows": mr.value,
                "rows_kernel": ROWS_KERNELS.get(rk.value, "?"), "column_windows": bool(win.value),
                "walk": WALKS.get(wk.value, "?"), "narrow_launch": bool(nar.value)}

    def load_timing(self):
        """(ms host checks, ms H2D, ms device F/G build) of the last load."""
        a, b, c = ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
        self._check(self.lib.pfaai_load_timing(self.ctx, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)),
                    "pfaai_load_timing")
        return a.value, b.value, c.value

    def load_info(self):
        """Which orientation the last load built on the device (LOAD_PATHS)."""
        k = ctypes.c_int32()
        self._check(self.lib.pfaai_load_info(self.ctx, ctypes.byref(k)), "pfaai_load_info")
        return LOAD_PATHS.get(k.value, "?")

    def timing(self, reset=True):
        """(n_runs, ms_build_total, ms_rows_total) of the runs since the last reset."""
        n, b, r = ctypes.c_int32(), ctypes.c_double(), ctypes.c_double()
        self._check(self.lib.pfaai_timing(self.ctx, int(reset), ctypes.byref(n), ctypes.byref(b), ctypes.byref(r)),
                    "pfaai_timing")
        return n.value, b.value, r.value

    def debug_div_check(self, c_max, d_max):
        """Mismatches of the kernels' exact small-integer division vs IEEE '/'."""
        n = ctypes.c_int64()
        self._check(self.lib.pfaai_debug_div_check(self.ctx, c_max, d_max, ctypes.byref(n)), "pfaai_debug_div_check")
        return n.value

    def debug_clocks(self, arm=False):
        """k_rows_pl stage clocks (PFAAI_PL_CLK=1): arm=True clears the buffer;
        otherwise returns u64 [256 workgroups, 16 waves, 8 stages]."""
        if arm:
            self._check(self.lib.pfaai_debug_clocks(self.ctx, None, 0), "pfaai_debug_clocks")
            return None
        out = np.zeros((256, 16, 8), dtype=np.uint64)
        self._check(self.lib.pfaai_debug_clocks(self.ctx, _ptr(out), out.size), "pfaai_debug_clocks")
        return out

    def debug_row_counts(self, row, n_prot, n_ids):
        out = np.zeros((n_prot, n_ids), dtype=np.int32)
        self._check(self.lib.pfaai_debug_row_counts(self.ctx, row, _ptr(out)), "pfaai_debug_row_counts")
        return out

    def synchronize(self):
        self._check(self.lib.pfaai_synchronize(self.ctx), "pfaai_synchronize")

    # -- raw device buffers (callers without a GPU framework) ---------------------
    def alloc(self, nbytes: int) -> int:
        p = ctypes.c_void_p()
        self._check(self.lib.pfaai_device_alloc(self.ctx, ctypes.byref(p), int(nbytes)), "pfaai_device_alloc")
        return p.value

    def free(self, ptr: int):
        self._check(self.lib.pfaai_device_free(self.ctx, ptr), "pfaai_device_free")

    def d2h(self, ptr: int, count: int, dtype) -> np.ndarray:
        out = np.empty(count, dtype=dtype)
        self._check(self.lib.pfaai_memcpy_d2h(self.ctx, _ptr(out), ptr, out.nbytes), "pfaai_memcpy_d2h")
        return out


class Group:
    """pfaai_group: several devices in one process, one RCCL communicator
    over them.  load() puts the problem on every device (each
    builds the walk data of its own row block); run() computes every block
    and gathers them into device-0 arrays (grouped ncclSend / ncclRecv).
    peer_gather=True: no communicator, the gather by peer copies, and a
    device may repeat (pfaai_group_create_flags, PFAAI_GROUP_PEER_GATHER)."""

    def __init__(self, devices, lib_path=None, peer_gather=False):
        self.lib = load_library(lib_path)
        self.g = ctypes.c_void_p()
        ids = (ctypes.c_int * len(devices))(*[int(d) for d in devices])
        if peer_gather:
            rc = self.lib.pfaai_group_create_flags(ctypes.byref(self.g), ids, len(devices), GROUP_PEER_GATHER)
        else:
            rc = self.lib.pfaai_group_create(ctypes.byref(self.g), ids, len(devices))
        if rc != PFAAI_OK:
            raise PfaaiError(rc, f"pfaai_group_create(devices={list(devices)})")
        self.n = len(devices)
        self._keep = None

    def _check(self, rc, what):
        if rc != PFAAI_OK:
            msg = self.lib.pfaai_group_last_error(self.g)
            raise PfaaiError(rc, f"{what}: {msg.decode() if msg else ''}")

    def close(self):
        if self.g:
            self.lib.pfaai_group_destroy(self.g)
            self.g = ctypes.c_void_p()

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def load(self, **kw):
        pb, keep = _problem(**kw)  # (keep: borrowed for the call only)
        self._check(self.lib.pfaai_group_load(self.g, ctypes.byref(pb)), "pfaai_group_load")
        del keep

    def blocks(self):
        cuts = (ctypes.c_int64 * (self.n + 1))()
        self._check(self.lib.pfaai_group_blocks(self.g, cuts), "pfaai_group_blocks")
        return [(cuts[i], cuts[i + 1]) for i in range(self.n)]

    def shape(self):
        r, p = ctypes.c_int64(), ctypes.c_int64()
        ctx = self.lib.pfaai_group_ctx(self.g, 0)
        rc = self.lib.pfaai_shape(ctx, ctypes.byref(r), ctypes.byref(p))
        if rc != PFAAI_OK:
            raise PfaaiError(rc, "pfaai_shape")
        return r.value, p.value

    def run(self, flags, d_aji, d_S=None, d_N=None):
        """Device pointers on the group's first device, length n_pairs; synchronous."""
        self._check(self.lib.pfaai_group_run(self.g, flags, d_aji, d_S, d_N), "pfaai_group_run")
