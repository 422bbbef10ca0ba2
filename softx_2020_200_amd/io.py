"""Drop-in I/O surface over the C-ABI (csrc/gls_io.cpp): deal.II parameter files,
ParsedFunction expressions (muParser semantics) and VTU/PVTU/PVD output with the reference's
fields (navier_stokes_base.cc:998-1086, post_processors.h:27-171)."""
from __future__ import annotations

import ctypes as C

import numpy as np

from .native import GLSError, MeshDesc, check, load

GLS_ENOTFOUND = -7


def _bind():
    L = load()
    if getattr(L, "_io_bound", False):
        return L
    vp, cp, i64, d = C.c_void_p, C.c_char_p, C.c_int64, C.POINTER(C.c_double)
    L.gls_prm_parse.argtypes = [cp, C.c_int, C.POINTER(vp)]
    L.gls_prm_get.argtypes = [vp, cp, C.c_char_p, C.c_int]
    L.gls_prm_n_entries.argtypes = [vp]
    L.gls_prm_entry.argtypes = [vp, C.c_int, C.c_char_p, C.c_int, C.c_char_p, C.c_int]
    L.gls_prm_destroy.argtypes = [vp]
    L.gls_prm_destroy.restype = None
    L.gls_expr_create.argtypes = [cp, cp, cp, C.POINTER(vp)]
    L.gls_expr_n_components.argtypes = [vp]
    L.gls_expr_eval.argtypes = [vp, i64, d, d]
    L.gls_expr_destroy.argtypes = [vp]
    L.gls_expr_destroy.restype = None
    L.gls_vtu_write.argtypes = [cp, C.POINTER(MeshDesc), d, C.c_int, C.c_int, C.c_int]
    L.gls_pvtu_write.argtypes = [cp, C.c_int, C.c_int, C.c_int, C.POINTER(cp)]
    L.gls_pvd_write.argtypes = [cp, C.c_int, d, C.POINTER(cp)]
    L._io_bound = True
    return L


class Prm:
    """Parsed parameter file; entries addressed "subsection/.../key"."""

    def __init__(self, text=None, path=None):
        self.L = _bind()
        h = C.c_void_p()
        src = path if path is not None else text
        check(self.L.gls_prm_parse(src.encode(), 1 if path is not None else 0, C.byref(h)), "gls_prm_parse")
        self.h = h

    def __del__(self):
        if getattr(self, "h", None):
            self.L.gls_prm_destroy(self.h)
            self.h = None

    def get(self, path, default=None):
        n = self.L.gls_prm_get(self.h, path.encode(), None, 0)
        if n == GLS_ENOTFOUND:
            return default
        check(n, "gls_prm_get")
        buf = C.create_string_buffer(n + 1)
        self.L.gls_prm_get(self.h, path.encode(), buf, n + 1)
        return buf.value.decode()

    def items(self):
        out = []
        for i in range(self.L.gls_prm_n_entries(self.h)):
            kb, vb = C.create_string_buffer(4096), C.create_string_buffer(65536)
            check(self.L.gls_prm_entry(self.h, i, kb, 4096, vb, 65536), "gls_prm_entry")
            out.append((kb.value.decode(), vb.value.decode()))
        return out


class Expr:
    """deal.II ParsedFunction: ';'-separated components over variables (default x,y,z,t)."""

    def __init__(self, expression, variables="x,y,z,t", constants=""):
        self.L = _bind()
        h = C.c_void_p()
        check(self.L.gls_expr_create(expression.encode(), variables.encode(), (constants or "").encode(), C.byref(h)),
              "gls_expr_create")
        self.h = h
        self.n_vars = len([v for v in variables.split(",") if v.strip()])
        self.n_components = self.L.gls_expr_n_components(h)

    def __del__(self):
        if getattr(self, "h", None):
            self.L.gls_expr_destroy(self.h)
            self.h = None

    def __call__(self, values):
        """values: [n_points, n_vars] -> [n_points, n_components]"""
        v = np.ascontiguousarray(values, dtype=np.float64).reshape(-1, self.n_vars)
        out = np.zeros((v.shape[0], self.n_components))
        check(self.L.gls_expr_eval(self.h, v.shape[0], v.ctypes.data_as(C.POINTER(C.c_double)),
                                   out.ctypes.data_as(C.POINTER(C.c_double))), "gls_expr_eval")
        return out


def write_vtu(filename, mesh, solution, subdivision=1, subdomain=0, binary=True, srf=False, omega=(0., 0., 0.)):
    """One VTU piece of a host solution vector on a mesh dict (softx_2020_200_amd.hyper_cube layout)."""
    L = _bind()
    dim, k, kp = mesh["dim"], mesh["k"], mesh["kp"]
    cv = np.ascontiguousarray(mesh["cell_vnodes"], dtype=np.int32)
    cpn = mesh.get("cell_pnodes") if kp != k else None
    cpn = np.ascontiguousarray(cpn, dtype=np.int32) if cpn is not None else None
    x0 = np.ascontiguousarray(mesh["cell_x0"], dtype=np.float64)
    h = np.ascontiguousarray(mesh["cell_h"], dtype=np.float64)
    sol = np.ascontiguousarray(solution, dtype=np.float64)
    if sol.size != dim * mesh["n_vnodes"] + mesh["n_pnodes"]:
        raise GLSError("solution length %d does not match the mesh" % sol.size)
    md = MeshDesc()
    md.dim, md.k, md.kp, md.nq1d = dim, k, kp, 0
    md.n_cells, md.n_vnodes, md.n_pnodes = cv.shape[0], mesh["n_vnodes"], mesh["n_pnodes"]
    md.cell_vnodes = cv.ctypes.data_as(C.POINTER(C.c_int32))
    md.cell_pnodes = cpn.ctypes.data_as(C.POINTER(C.c_int32)) if cpn is not None else None
    md.cell_x0 = x0.ctypes.data_as(C.POINTER(C.c_double))
    md.cell_h = h.ctypes.data_as(C.POINTER(C.c_double))
    md.srf = 1 if srf else 0
    md.omega = (C.c_double * 3)(*omega)
    check(L.gls_vtu_write(filename.encode(), C.byref(md), sol.ctypes.data_as(C.POINTER(C.c_double)), int(subdivision),
                          int(subdomain), 1 if binary else 0), "gls_vtu_write")


def write_pvtu(filename, dim, pieces, srf=False):
    L = _bind()
    arr = (C.c_char_p * len(pieces))(*[p.encode() for p in pieces])
    check(L.gls_pvtu_write(filename.encode(), dim, 1 if srf else 0, len(pieces), arr), "gls_pvtu_write")


def write_pvd(filename, times_and_files):
    L = _bind()
    t = np.ascontiguousarray([tf[0] for tf in times_and_files], dtype=np.float64)
    arr = (C.c_char_p * len(times_and_files))(*[tf[1].encode() for tf in times_and_files])
    check(L.gls_pvd_write(filename.encode(), len(times_and_files), t.ctypes.data_as(C.POINTER(C.c_double)), arr),
          "gls_pvd_write")
