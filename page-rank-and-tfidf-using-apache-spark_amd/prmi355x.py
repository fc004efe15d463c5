"""Python host mirror of the reference job's entry point, over the prmi355x C ABI.

The reference's host code is Java (PageRank.java); no JVM exists in this image, so this
module mirrors ``PageRank.main`` (PageRank.java:21-206) in Python with the same argument
meaning, file contract and failure behaviour, and calls the MI355X engine through the
C ABI in ``include/prmi355x.h`` via ctypes.  The Java (Panama FFM / JNI) binding a
maintainer would add is in INTEGRATION.md.

The engine is the HIP library ``_build/libprmi355x.so``.  There is NO CPU fallback: if the
library is missing or no GPU is present, every compute call raises.
"""
from __future__ import annotations

import ctypes as C
import os
import re
import subprocess
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO_DIR = os.path.dirname(PKG_DIR)
LIB_PATH = os.path.join(PKG_DIR, "_build", "libprmi355x.so")
HEADER_PATH = os.path.join(REPO_DIR, "include", "prmi355x.h")

PR_OK = 0
PR_E_ARG = -1
PR_E_PARSE = -2
PR_E_EMPTY_DANGLING = -3
PR_E_HIP = -4
PR_E_RCCL = -5
PR_E_OOM = -6
PR_E_IO = -7
PR_E_NODEV = -8
PR_DEVICE_FROM_RANK = -1
PR_DEVICE_NONE = -2
PR_F_TRACK_RESIDUAL = 0x1
PR_F_VERBOSE = 0x2
PR_F_NORMALIZED = 0x4


# ---- the reference's failure modes ------------------------------------------------------
class PageRankError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(msg)
        self.code = code


class ArrayIndexOutOfBoundsException(PageRankError):
    """Malformed input line (PageRank.java:40 / :49)."""


class UnsupportedOperationException(PageRankError):
    """``reduce`` on an empty danglingMap (PageRank.java:125): "empty collection"."""


class IOException(PageRankError):
    """Reading inputs / writing ./topPage failed (PageRank.java:201-204)."""


_EXC = {PR_E_PARSE: ArrayIndexOutOfBoundsException,
        PR_E_EMPTY_DANGLING: UnsupportedOperationException,
        PR_E_IO: IOException}


# ---- ctypes structs mirroring include/prmi355x.h ------------------------------------------
class Opts(C.Structure):
    _fields_ = [("device", C.c_int32), ("n_ranks", C.c_int32), ("rank", C.c_int32),
                ("topk", C.c_uint32), ("flags", C.c_uint32), ("reserved", C.c_uint32 * 7)]


class Stats(C.Structure):
    _fields_ = [("iterations", C.c_int32), ("failed_iteration", C.c_int32),
                ("ms_total", C.c_double), ("ms_per_iter", C.c_double),
                ("ms_spmv_kernel", C.c_double), ("gteps", C.c_double),
                ("residual", C.c_double), ("rank_sum", C.c_double),
                ("nnz", C.c_uint64), ("n_vertices", C.c_uint64), ("defined", C.c_uint64),
                ("bytes_per_iter", C.c_uint64), ("reserved", C.c_uint64 * 6)]

    def as_dict(self) -> Dict[str, float]:
        return {k: getattr(self, k) for k, _t in self._fields_ if k != "reserved"}


class GraphInfo(C.Structure):
    _fields_ = [("n_vertices", C.c_uint64), ("raw_edges", C.c_uint64), ("nnz", C.c_uint64),
                ("n_tot", C.c_uint64), ("n_pairs", C.c_uint64),
                ("dangling_entries", C.c_uint64), ("n_sources", C.c_uint64),
                ("n_rows", C.c_uint64), ("local_rows", C.c_uint64), ("local_nnz", C.c_uint64),
                ("ms_ingest", C.c_double), ("ms_build", C.c_double),
                ("ingest_flags", C.c_uint64), ("place_tried", C.c_uint64),
                ("place_ms_first", C.c_double), ("place_ms_best", C.c_double),
                ("reserved", C.c_uint64 * 2)]

    def as_dict(self) -> Dict[str, float]:
        return {k: getattr(self, k) for k, _t in self._fields_ if k != "reserved"}


_lib = None


def build() -> str:
    """Compile the engine in-tree (hipcc --offload-arch=gfx950) -> _build/libprmi355x.so."""
    jobs = str(min(8, os.cpu_count() or 4))
    subprocess.run(["make", "-s", "-j", jobs, "-C", PKG_DIR], check=True)
    return LIB_PATH


def declared_symbols() -> List[str]:
    """Function names declared in include/prmi355x.h."""
    src = open(HEADER_PATH).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(pr_[a-z_0-9]+)\s*\(", src)))


def lib():
    """Load the engine; raises if it has not been built (no fallback path exists)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"prmi355x engine not built: {LIB_PATH} missing "
                           "(run __graft_entry__.build() or make -C the package)")
    L = C.CDLL(LIB_PATH)
    P, I32, U32, U64, D, SZ = C.c_void_p, C.c_int32, C.c_uint32, C.c_uint64, C.c_double, C.c_size_t
    sig = {
        "pr_version": (C.c_char_p, []),
        "pr_build_id": (C.c_char_p, []),
        "pr_opts_default": (None, [C.POINTER(Opts)]),
        "pr_create": (I32, [C.POINTER(P), C.POINTER(Opts)]),
        "pr_destroy": (None, [P]),
        "pr_last_error": (C.c_char_p, [P]),
        "pr_comm_unique_id": (I32, [C.c_char_p]),
        "pr_comm_init": (I32, [P, C.c_char_p]),
        "pr_comm_init_local": (I32, [C.POINTER(P), I32]),
        "pr_run_group": (I32, [C.POINTER(P), I32, I32, D, C.POINTER(Stats)]),
        "pr_comm_init_external": (I32, [P]),
        "pr_ext_begin": (I32, [P, I32, D, C.POINTER(U64)]),
        "pr_ext_round": (I32, [P, I32, P]),
        "pr_ext_complete": (I32, [P, I32, P, C.POINTER(I32)]),
        "pr_ext_end": (I32, [P, C.POINTER(Stats)]),
        "pr_progress": (I32, [P, C.POINTER(I32), C.POINTER(I32)]),
        "pr_comm_query": (I32, [P, C.POINTER(I32), C.POINTER(I32), C.POINTER(I32)]),
        "pr_layout_map": (I32, [I32, I32, U32, U32, U32, U64, P, P, P, P, P]),
        "pr_selftest_sum_order": (I32, [P, U32, U32, C.POINTER(U64), C.POINTER(U64), C.POINTER(U64)]),
        "pr_ingest_files": (I32, [P, C.c_char_p, C.c_char_p]),
        "pr_ingest_buffers": (I32, [P, C.c_char_p, SZ, C.c_char_p, SZ]),
        "pr_load_edges": (I32, [P, P, P, U64, U32, P, U64]),
        "pr_generate_rmat": (I32, [P, I32, I32, U64]),
        "pr_graph_get_info": (I32, [P, C.POINTER(GraphInfo)]),
        "pr_run": (I32, [P, I32, D, C.POINTER(Stats)]),
        "pr_run_static": (I32, [P, I32, D, C.POINTER(Stats)]),
        "pr_get_ranks": (I32, [P, P, U64]),
        "pr_topk": (I32, [P, U32, P, P, P, C.POINTER(U32)]),
        "pr_write_top_page": (I32, [P, C.c_char_p]),
        "pr_write_rank_dump": (I32, [P, C.c_char_p]),
        "pr_id_string": (I32, [P, U32, C.c_char_p, SZ, C.POINTER(SZ)]),
        "pr_pair": (I32, [P, U64, C.POINTER(U32), C.c_char_p, SZ, C.POINTER(SZ)]),
        "pr_get_degrees": (I32, [P, P, P, P, U64]),
        "pr_edge_digest": (I32, [P, P]),
        "pr_export_csr": (I32, [P, P, P, P, P, C.POINTER(U64), C.POINTER(U64)]),
        "pr_format_double": (I32, [D, C.c_char_p, SZ]),
        "pr_set_ranks": (I32, [P, P, U64, I32]),
        "pr_checkpoint_save": (I32, [P, C.c_char_p]),
        "pr_checkpoint_load": (I32, [P, C.c_char_p]),
        "pr_tfidf_ingest_buffer": (I32, [P, C.c_char_p, SZ]),
        "pr_tfidf_ingest_file": (I32, [P, C.c_char_p]),
        "pr_tfidf_info": (I32, [P, C.POINTER(U64), C.POINTER(U64), C.POINTER(U64), C.POINTER(U64)]),
        "pr_tfidf_lookup": (I32, [P, C.c_char_p, SZ, U32, P, P, C.POINTER(U32)]),
        "pr_tfidf_title": (I32, [P, U32, C.c_char_p, SZ, C.POINTER(SZ)]),
        "pr_tfidf_write_output": (I32, [P, C.c_char_p, C.c_char_p]),
    }
    for name, (rt, args) in sig.items():
        f = getattr(L, name)
        f.restype = rt
        f.argtypes = args
    _lib = L
    return L


def build_id() -> str:
    """Source hash the loaded library was built from (``pr_build_id``)."""
    return lib().pr_build_id().decode()


def source_hash() -> str:
    """Hash of the checked-out engine sources (what a fresh build would report)."""
    import source_hash as _sh
    return _sh.source_hash()


def _ptr(a: Optional[np.ndarray]):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def format_double(v: float) -> str:
    """Java ``Double.toString`` as the engine prints it into topPage."""
    buf = C.create_string_buffer(64)
    n = lib().pr_format_double(float(v), buf, 64)
    return buf.raw[:n].decode()


def layout_map(n_ranks: int, rank: int, n_a: int, n_b: int, n_c: int, ids):
    """The engine's row deal and x layout on the host (``pr_layout_map``): for internal vertex
    ids returns (owner rank, local row, x position) arrays and the dims dict."""
    k = np.ascontiguousarray(ids, np.uint32)
    owner = np.zeros(len(k), np.uint32)
    local = np.zeros(len(k), np.uint32)
    xp = np.zeros(len(k), np.uint64)
    dims = np.zeros(4, np.uint64)
    rc = lib().pr_layout_map(n_ranks, rank, n_a, n_b, n_c, len(k), _ptr(k), _ptr(owner),
                             _ptr(local), _ptr(xp), _ptr(dims))
    if rc:
        raise PageRankError(rc, f"pr_layout_map failed ({rc})")
    return owner, local, xp, {"max_a": int(dims[0]), "x_len": int(dims[1]),
                              "local_rows": int(dims[2]), "local_a": int(dims[3])}


def comm_unique_id() -> bytes:
    buf = C.create_string_buffer(128)
    rc = lib().pr_comm_unique_id(buf)
    if rc:
        raise PageRankError(rc, "pr_comm_unique_id failed")
    return buf.raw[:128]


class Engine:
    """One engine context (one process, one GPU) -- SparkContext + the job's RDDs."""

    def __init__(self, device: int = PR_DEVICE_FROM_RANK, n_ranks: int = 1, rank: int = 0,
                 topk: int = 100, flags: int = 0):
        L = lib()
        o = Opts()
        L.pr_opts_default(C.byref(o))
        o.device, o.n_ranks, o.rank, o.topk, o.flags = device, n_ranks, rank, topk, flags
        h = C.c_void_p()
        rc = L.pr_create(C.byref(h), C.byref(o))
        if rc:
            raise PageRankError(rc, f"pr_create failed ({rc}): no usable HIP device?")
        self._h = h
        self.n_ranks, self.rank = n_ranks, rank

    def close(self):
        if getattr(self, "_h", None):
            lib().pr_destroy(self._h)
            self._h = None

    __del__ = close

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def _check(self, rc: int):
        if rc:
            msg = (lib().pr_last_error(self._h) or b"").decode(errors="replace")
            raise _EXC.get(rc, PageRankError)(rc, msg or f"error {rc}")

    # ---- comm ----
    def comm_init(self, uid: bytes):
        self._check(lib().pr_comm_init(self._h, uid))

    def comm_init_external(self):
        """Exchange rounds through the caller (pr_ext_*), e.g. a torch.distributed group."""
        self._check(lib().pr_comm_init_external(self._h))

    def progress(self) -> Tuple[int, int]:
        """(rounds enqueued, rounds finished) of the running or last round loop; safe to call
        from another thread while ``run`` blocks."""
        enq, done = C.c_int32(0), C.c_int32(0)
        h = self._h
        if not h:
            return 0, 0
        lib().pr_progress(h, C.byref(enq), C.byref(done))
        return enq.value, done.value

    def selftest_sum_order(self, cases: int = 64, launches: int = 20) -> Dict[str, int]:
        """Bit-compare the LDS double-add order of the row launch over many waves and launches
        (pr_selftest_sum_order)."""
        a, b, c = C.c_uint64(0), C.c_uint64(0), C.c_uint64(0)
        self._check(lib().pr_selftest_sum_order(self._h, cases, launches, C.byref(a), C.byref(b),
                                                C.byref(c)))
        return {"copies": a.value, "differing": b.value, "lane_order_cases": c.value, "cases": cases}

    def comm_query(self) -> Dict[str, object]:
        """Transport of this context and, for RCCL, the communicator's own rank count."""
        tr, n, r = C.c_int32(0), C.c_int32(0), C.c_int32(0)
        self._check(lib().pr_comm_query(self._h, C.byref(tr), C.byref(n), C.byref(r)))
        return {"transport": ("none", "rccl", "local-group", "external")[tr.value],
                "comm_ranks": n.value, "comm_rank": r.value}

    def run_external(self, iterations: int, allgather, tol: float = 0.0) -> Dict[str, float]:
        """The round loop with a caller-supplied all-gather: ``allgather(send) -> recv`` takes
        this rank's uint8 unit and returns the p units in rank order (one uint8 array)."""
        unit = C.c_uint64(0)
        self._check(lib().pr_ext_begin(self._h, iterations, tol, C.byref(unit)))
        send = np.zeros(unit.value, np.uint8)
        stop = C.c_int32(0)
        for t in range(1, iterations + 1):
            self._check(lib().pr_ext_round(self._h, t, _ptr(send)))
            recv = np.ascontiguousarray(allgather(send), np.uint8)
            if recv.size != unit.value * self.n_ranks:
                raise ValueError(f"allgather returned {recv.size} bytes, expected "
                                 f"{unit.value} x {self.n_ranks} ranks")
            self._check(lib().pr_ext_complete(self._h, t, _ptr(recv), C.byref(stop)))
            if stop.value:
                break
        st = Stats()
        self._check(lib().pr_ext_end(self._h, C.byref(st)))
        return st.as_dict()

    # ---- input ----
    def ingest_files(self, arcs_path: str, mapping_path: str):
        self._check(lib().pr_ingest_files(self._h, arcs_path.encode(), mapping_path.encode()))

    def ingest_buffers(self, arcs: bytes, mapping: bytes):
        self._check(lib().pr_ingest_buffers(self._h, arcs, len(arcs), mapping, len(mapping)))

    def load_edges(self, src, dst, n: int, mapw=None, n_tot: int = 0):
        src = np.ascontiguousarray(src, np.uint32)
        dst = np.ascontiguousarray(dst, np.uint32)
        mw = None if mapw is None else np.ascontiguousarray(mapw, np.uint32)
        self._check(lib().pr_load_edges(self._h, _ptr(src), _ptr(dst), len(src), n, _ptr(mw),
                                        n_tot))

    def generate_rmat(self, scale: int, edge_factor: int, seed: int):
        self._check(lib().pr_generate_rmat(self._h, scale, edge_factor, seed))

    def info(self) -> Dict[str, float]:
        gi = GraphInfo()
        self._check(lib().pr_graph_get_info(self._h, C.byref(gi)))
        return gi.as_dict()

    # ---- the loop ----
    def run(self, iterations: int = 10, tol: float = 0.0) -> Dict[str, float]:
        st = Stats()
        rc = lib().pr_run(self._h, iterations, tol, C.byref(st))
        self._check(rc)
        return st.as_dict()

    def run_static(self, iterations: int = 10, tol: float = 0.0) -> Dict[str, float]:
        """``pr_run`` with the per-round scratch in the library's static device array: no
        allocation during the call (single-GPU contexts, bounded graph size)."""
        st = Stats()
        rc = lib().pr_run_static(self._h, iterations, tol, C.byref(st))
        self._check(rc)
        return st.as_dict()

    # ---- output ----
    def ranks(self) -> np.ndarray:
        n = int(self.info()["n_vertices"])
        out = np.zeros(n, np.float64)
        self._check(lib().pr_get_ranks(self._h, _ptr(out), n))
        return out

    def topk(self, k: int = 100) -> List[Tuple[int, int, float]]:
        pair = np.zeros(max(k, 1), np.uint64)
        vid = np.zeros(max(k, 1), np.uint32)
        rk = np.zeros(max(k, 1), np.float64)
        cnt = C.c_uint32(0)
        self._check(lib().pr_topk(self._h, k, _ptr(pair), _ptr(vid), _ptr(rk), C.byref(cnt)))
        return [(int(pair[i]), int(vid[i]), float(rk[i])) for i in range(cnt.value)]

    # ---- resume ----
    def set_ranks(self, ranks: Optional[np.ndarray], rounds_done: int = 0):
        """Seed later runs with ranks (by vertex id) reached after rounds_done rounds;
        None clears the seed."""
        if ranks is None:
            self._check(lib().pr_set_ranks(self._h, None, 0, 0))
            return
        r = np.ascontiguousarray(ranks, np.float64)
        self._check(lib().pr_set_ranks(self._h, _ptr(r), len(r), rounds_done))

    def checkpoint_save(self, path: str):
        self._check(lib().pr_checkpoint_save(self._h, path.encode()))

    def checkpoint_load(self, path: str):
        self._check(lib().pr_checkpoint_load(self._h, path.encode()))

    # ---- TF-IDF job (Spark.java) ----
    def tfidf_ingest(self, data: bytes):
        self._check(lib().pr_tfidf_ingest_buffer(self._h, data, len(data)))

    def tfidf_info(self) -> Dict[str, int]:
        v = [C.c_uint64(0) for _ in range(4)]
        self._check(lib().pr_tfidf_info(self._h, *[C.byref(x) for x in v]))
        return dict(zip(("docs", "words", "pairs", "tokens"), (x.value for x in v)))

    def tfidf_title(self, t: int) -> bytes:
        ln = C.c_size_t(0)
        self._check(lib().pr_tfidf_title(self._h, t, None, 0, C.byref(ln)))
        buf = C.create_string_buffer(max(ln.value, 1))
        self._check(lib().pr_tfidf_title(self._h, t, buf, ln.value, C.byref(ln)))
        return buf.raw[:ln.value]

    def tfidf_lookup(self, word: bytes, k: int = 100) -> List[Tuple[bytes, float]]:
        t = np.zeros(max(k, 1), np.uint32)
        v = np.zeros(max(k, 1), np.float64)
        cnt = C.c_uint32(0)
        self._check(lib().pr_tfidf_lookup(self._h, word, len(word), k, _ptr(t), _ptr(v),
                                          C.byref(cnt)))
        return [(self.tfidf_title(int(t[i])), float(v[i])) for i in range(cnt.value)]

    def tfidf_write_output(self, word: Optional[bytes] = None, path: str = "./output"):
        self._check(lib().pr_tfidf_write_output(self._h, word, path.encode()))

    def write_top_page(self, path: str = "./topPage"):
        self._check(lib().pr_write_top_page(self._h, path.encode()))

    def write_rank_dump(self, path: str):
        """Every ranked page by id: `id \\t title \\t rank` lines (pr_write_rank_dump)."""
        self._check(lib().pr_write_rank_dump(self._h, path.encode()))

    def id_string(self, v: int) -> bytes:
        ln = C.c_size_t(0)
        self._check(lib().pr_id_string(self._h, v, None, 0, C.byref(ln)))
        buf = C.create_string_buffer(max(ln.value, 1))
        self._check(lib().pr_id_string(self._h, v, buf, ln.value, C.byref(ln)))
        return buf.raw[:ln.value]

    def pair(self, i: int) -> Tuple[int, bytes]:
        ln = C.c_size_t(0)
        vid = C.c_uint32(0)
        self._check(lib().pr_pair(self._h, i, C.byref(vid), None, 0, C.byref(ln)))
        buf = C.create_string_buffer(max(ln.value, 1))
        self._check(lib().pr_pair(self._h, i, C.byref(vid), buf, ln.value, C.byref(ln)))
        return vid.value, buf.raw[:ln.value]

    def degrees(self) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
        n = int(self.info()["n_vertices"])
        o, i, w = (np.zeros(n, np.uint32) for _ in range(3))
        self._check(lib().pr_get_degrees(self._h, _ptr(o), _ptr(i), _ptr(w), n))
        return o, i, w

    def edge_digest(self) -> Tuple[int, int]:
        d = np.zeros(2, np.uint64)
        self._check(lib().pr_edge_digest(self._h, _ptr(d)))
        return int(d[0]), int(d[1])

    def export_csr(self):
        n, nnz = C.c_uint64(0), C.c_uint64(0)
        self._check(lib().pr_export_csr(self._h, None, None, None, None, C.byref(n), C.byref(nnz)))
        rp = np.zeros(n.value + 1, np.uint64)
        col = np.zeros(max(nnz.value, 1), np.uint32)
        od = np.zeros(max(n.value, 1), np.uint32)
        dw = np.zeros(max(n.value, 1), np.uint32)
        self._check(lib().pr_export_csr(self._h, _ptr(rp), _ptr(col), _ptr(od), _ptr(dw),
                                        C.byref(n), C.byref(nnz)))
        return rp, col[:nnz.value], od[:n.value], dw[:n.value]


class LocalGroup:
    """n engine contexts in this process acting as ranks 0..n-1 (device copies replace RCCL)."""

    def __init__(self, n: int, devices: Optional[Sequence[int]] = None, flags: int = 0):
        devs = list(devices) if devices is not None else [0] * n
        self.members = [Engine(device=devs[i], n_ranks=n, rank=i, flags=flags) for i in range(n)]
        self._arr = (C.c_void_p * n)(*[m._h for m in self.members])
        rc = lib().pr_comm_init_local(self._arr, n)
        if rc:
            raise PageRankError(rc, "pr_comm_init_local failed")

    def each(self, fn, *args):
        for m in self.members:
            getattr(m, fn)(*args)

    def run(self, iterations: int = 10, tol: float = 0.0) -> Dict[str, float]:
        st = Stats()
        rc = lib().pr_run_group(self._arr, len(self.members), iterations, tol, C.byref(st))
        self.members[0]._check(rc)
        return st.as_dict()

    def close(self):
        for m in self.members:
            m.close()


class PageRank:
    """Mirror of ``public class PageRank`` (PageRank.java:20)."""

    DEFAULT_ARCS = "./wikipedia_arcs"          # basename of s3n://.../wikipedia_arcs (:27)
    DEFAULT_MAPPING = "./wikipedia_mapping"    # basename of s3n://.../wikipedia_mapping (:30)

    @staticmethod
    def main(args: Sequence[str] = (), out: str = "./topPage", topk: int = 100,
             tol: float = 0.0) -> Dict[str, float]:
        """``PageRank.main(args)``: ``[arcs mapping [iterations]]``; writes ``out``.

        Raises ArrayIndexOutOfBoundsException / UnsupportedOperationException exactly where
        the reference job dies; an IOException while writing topPage is printed and
        swallowed like the reference's ``e.printStackTrace()`` (:201-204)."""
        args = list(args)
        arcs = args[0] if len(args) > 0 else PageRank.DEFAULT_ARCS
        mapping = args[1] if len(args) > 1 else PageRank.DEFAULT_MAPPING
        iterations = int(args[2]) if len(args) > 2 else 10          # :92
        with Engine(topk=topk) as eng:
            eng.ingest_files(arcs, mapping)
            stats = eng.run(iterations, tol)
            try:
                eng.write_top_page(out)
            except IOException as e:                                # :201-204
                import sys
                print(e, file=sys.stderr)
            return stats
