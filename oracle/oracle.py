"""TEST INFRASTRUCTURE ONLY -- ctypes binding of the C oracle (``oracle/pagerank_oracle.c``).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this module.  Parity status: *parity unpinned* against Spark (see
``pagerank_oracle.c`` header and DESIGN.md); pinned by Appendix-B KATs and by bit-exact
agreement with ``pagerank_literal.py``.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from typing import Dict, List, Optional, Tuple

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "liborc.so")
_lib = None

ORC_E_PARSE = -2
ORC_E_EMPTY_DANGLING = -3


def build() -> str:
    """Compile the oracle (gcc, seconds).  Safe to call repeatedly."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = C.CDLL(_LIB_PATH)
        P, U32, U64, I32, D = C.c_void_p, C.c_uint32, C.c_uint64, C.c_int, C.c_double
        L.orc_from_text.restype = P
        L.orc_from_text.argtypes = [C.c_char_p, C.c_size_t, C.c_char_p, C.c_size_t]
        L.orc_from_edges.restype = P
        L.orc_from_edges.argtypes = [P, P, U64, U32, P, U64]
        L.orc_from_rmat.restype = P
        L.orc_from_rmat.argtypes = [I32, I32, U64]
        L.orc_rmat_edges.restype = None
        L.orc_rmat_edges.argtypes = [U64, I32, U64, U64, P, P]
        L.orc_error.restype = I32
        L.orc_error.argtypes = [P, C.POINTER(C.c_int64)]
        for f, rt in (("orc_num_vertices", U32), ("orc_nnz", U64), ("orc_raw_edges", U64),
                      ("orc_n_tot", U64), ("orc_num_pairs", U64)):
            getattr(L, f).restype = rt
            getattr(L, f).argtypes = [P]
        L.orc_degrees.restype = None
        L.orc_degrees.argtypes = [P, P, P, P]
        L.orc_row_ptr.restype = C.POINTER(U64)
        L.orc_row_ptr.argtypes = [P]
        L.orc_col.restype = C.POINTER(U32)
        L.orc_col.argtypes = [P]
        L.orc_id_bytes.restype = C.POINTER(C.c_char)
        L.orc_id_bytes.argtypes = [P, U32, C.POINTER(C.c_size_t)]
        L.orc_pair.restype = None
        L.orc_pair.argtypes = [P, U64, C.POINTER(U32), C.POINTER(C.POINTER(C.c_char)),
                               C.POINTER(C.c_size_t)]
        L.orc_edge_digest.restype = None
        L.orc_edge_digest.argtypes = [P, P]
        L.orc_pagerank_csr.restype = I32
        L.orc_pagerank_csr.argtypes = [U32, P, P, P, P, U64, I32, I32, I32, D, P,
                                       C.POINTER(D), C.POINTER(I32), C.POINTER(D)]
        L.orc_run.restype = I32
        L.orc_run.argtypes = [P, I32, I32, I32, D, P, C.POINTER(D), C.POINTER(I32), C.POINTER(D)]
        L.orc_run_ex.restype = I32
        L.orc_run_ex.argtypes = [P, I32, I32, I32, D, I32, P, P, C.POINTER(D), C.POINTER(I32),
                                 C.POINTER(D)]
        L.orc_exact_dot_u32.restype = D
        L.orc_exact_dot_u32.argtypes = [P, P, U64]
        L.orc_free.restype = None
        L.orc_free.argtypes = [P]
        _lib = L
    return _lib


def _ptr(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


class OracleError(Exception):
    def __init__(self, code: int, line: int = 0):
        super().__init__(f"oracle error {code} (line {line})")
        self.code, self.line = code, line


class Graph:
    """A graph ingested by the oracle (text files or in-memory / R-MAT edges)."""

    def __init__(self, handle):
        self._h = handle
        L = lib()
        ln = C.c_int64(0)
        self.err = L.orc_error(handle, C.byref(ln))
        self.err_line = ln.value

    @classmethod
    def from_text(cls, arcs: bytes, mapping: bytes) -> "Graph":
        return cls(lib().orc_from_text(arcs, len(arcs), mapping, len(mapping)))

    @classmethod
    def from_edges(cls, src, dst, n: int, mapw=None, n_tot: Optional[int] = None) -> "Graph":
        src = np.ascontiguousarray(src, dtype=np.uint32)
        dst = np.ascontiguousarray(dst, dtype=np.uint32)
        mapw = np.ones(n, np.uint32) if mapw is None else np.ascontiguousarray(mapw, np.uint32)
        n_tot = n if n_tot is None else n_tot
        return cls(lib().orc_from_edges(_ptr(src), _ptr(dst), len(src), n, _ptr(mapw), n_tot))

    @classmethod
    def from_rmat(cls, scale: int, edge_factor: int, seed: int) -> "Graph":
        return cls(lib().orc_from_rmat(scale, edge_factor, seed))

    def __del__(self):
        if getattr(self, "_h", None):
            lib().orc_free(self._h)
            self._h = None

    def check(self):
        if self.err:
            raise OracleError(self.err, self.err_line)

    # ---- sizes / structure ----
    @property
    def n(self) -> int:
        return lib().orc_num_vertices(self._h)

    @property
    def nnz(self) -> int:
        return lib().orc_nnz(self._h)

    @property
    def raw_edges(self) -> int:
        return lib().orc_raw_edges(self._h)

    @property
    def n_tot(self) -> int:
        return lib().orc_n_tot(self._h)

    def degrees(self) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
        """(outdeg, indeg, dangling weight) per dense id."""
        n = self.n
        o, i, w = (np.zeros(n, np.uint32) for _ in range(3))
        lib().orc_degrees(self._h, _ptr(o), _ptr(i), _ptr(w))
        return o, i, w

    def csr(self) -> Tuple[np.ndarray, np.ndarray]:
        n, nnz = self.n, self.nnz
        rp = np.ctypeslib.as_array(lib().orc_row_ptr(self._h), shape=(n + 1,)).copy()
        col = (np.ctypeslib.as_array(lib().orc_col(self._h), shape=(nnz,)).copy()
               if nnz else np.zeros(0, np.uint32))
        return rp, col

    def edge_digest(self) -> Tuple[int, int]:
        out = np.zeros(2, np.uint64)
        lib().orc_edge_digest(self._h, _ptr(out))
        return int(out[0]), int(out[1])

    def id_bytes(self, v: int) -> bytes:
        ln = C.c_size_t(0)
        p = lib().orc_id_bytes(self._h, v, C.byref(ln))
        return C.string_at(p, ln.value) if ln.value else b""

    def ids(self) -> List[bytes]:
        return [self.id_bytes(v) for v in range(self.n)]

    def pairs(self) -> List[Tuple[int, bytes]]:
        out = []
        L = lib()
        for i in range(L.orc_num_pairs(self._h)):
            vid, tp, ln = C.c_uint32(0), C.POINTER(C.c_char)(), C.c_size_t(0)
            L.orc_pair(self._h, i, C.byref(vid), C.byref(tp), C.byref(ln))
            out.append((vid.value, C.string_at(tp, ln.value)))
        return out

    # ---- the job ----
    def run(self, iterations: int = 10, exact: bool = True, threads: int = 0,
            tol: float = 0.0, normalized: bool = False, r_init=None) -> Dict[str, object]:
        """normalized: r^0 = 1/N_tot and base 0.15/N_tot; r_init: resume from these ranks."""
        self.check()
        r = np.zeros(self.n, np.float64)
        spi, done, resid = C.c_double(0), C.c_int(0), C.c_double(0)
        if normalized or r_init is not None:
            ri = None if r_init is None else np.ascontiguousarray(r_init, np.float64)
            rc = lib().orc_run_ex(self._h, iterations, int(exact), threads, tol, int(normalized),
                                  _ptr(ri), _ptr(r), C.byref(spi), C.byref(done), C.byref(resid))
        else:
            rc = lib().orc_run(self._h, iterations, int(exact), threads, tol, _ptr(r),
                               C.byref(spi), C.byref(done), C.byref(resid))
        if rc:
            raise OracleError(rc, done.value)
        return {"ranks": r, "sec_per_iter": spi.value, "iterations": done.value,
                "residual": resid.value}


def pagerank_csr(row_ptr, col, outdeg, dang_w, n_tot: int, iterations: int, exact: bool = False,
                 threads: int = 0, tol: float = 0.0) -> Dict[str, object]:
    """Run the dense iteration on a caller-supplied pull CSR (used by the CPU baseline)."""
    n = len(outdeg)
    row_ptr = np.ascontiguousarray(row_ptr, np.uint64)
    col = np.ascontiguousarray(col, np.uint32)
    outdeg = np.ascontiguousarray(outdeg, np.uint32)
    dang_w = np.ascontiguousarray(dang_w, np.uint32)
    r = np.zeros(n, np.float64)
    spi, done, resid = C.c_double(0), C.c_int(0), C.c_double(0)
    rc = lib().orc_pagerank_csr(n, _ptr(row_ptr), _ptr(col), _ptr(outdeg), _ptr(dang_w), n_tot,
                                iterations, int(exact), threads, tol, _ptr(r), C.byref(spi),
                                C.byref(done), C.byref(resid))
    if rc:
        raise OracleError(rc, done.value)
    return {"ranks": r, "sec_per_iter": spi.value, "iterations": done.value,
            "residual": resid.value}


def rmat_edges(scale: int, edge_factor: int, seed: int, first: int = 0, count: Optional[int] = None):
    m = (edge_factor << scale) if count is None else count
    s = np.zeros(m, np.uint32)
    d = np.zeros(m, np.uint32)
    lib().orc_rmat_edges(seed, scale, first, m, _ptr(s), _ptr(d))
    return s, d


def exact_dot(v, w=None) -> float:
    v = np.ascontiguousarray(v, np.float64)
    wp = None
    if w is not None:
        w = np.ascontiguousarray(w, np.uint32)
        wp = _ptr(w)
    return lib().orc_exact_dot_u32(_ptr(v), wp, len(v))


def top_pages(graph: Graph, ranks: np.ndarray, k: int = 100):
    """(title, rank) rows of ranks.join(mappings) sorted descending (PageRank.java:167-189);
    ties broken by (title, id) so the oracle is deterministic."""
    rows = [(float(ranks[v]), t, v) for (v, t) in graph.pairs() if ranks[v] > 0.0]
    rows.sort(key=lambda r: (-r[0], r[1], r[2]))
    return [(t, r) for (r, t, _v) in rows[:k]]
