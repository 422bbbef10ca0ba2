"""ctypes binding of libgls_native.so (include/gls_native.h).

The product path: every operator call goes to the HIP kernels in libgls_native.so.
There is no CPU fallback — if the extension is missing or no HIP device is present,
``load()`` / ``GLSContext`` raise.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GLS_NATIVE_LIB") or os.path.join(HERE, "libgls_native.so")  # override: experiments only

GLS_OK, GLS_EINVAL, GLS_EHIP, GLS_ENOMEM, GLS_ENOCONV, GLS_EIO, GLS_ECOMM = 0, -1, -2, -3, -4, -5, -6

SCHEMES = {
    "steady": 0, "bdf1": 1, "bdf2": 2, "bdf3": 3, "sdirk2": 4, "sdirk2_1": 5, "sdirk2_2": 6,
    "sdirk3": 7, "sdirk3_1": 8, "sdirk3_2": 9, "sdirk3_3": 10,
}

# every symbol declared in include/gls_native.h (checked by tests/test_native_abi.py)
EXPORTS = [
    "gls_last_error", "gls_version", "gls_create", "gls_destroy", "gls_set_stream", "gls_n_dofs", "gls_set_force",
    "gls_set_viscosity", "gls_set_time", "gls_set_state", "gls_residual", "gls_jacobian_apply",
    "gls_jacobian_apply_f32",
    "gls_jacobian_diagonal", "gls_set_dirichlet", "gls_apply_dirichlet", "gls_solve_linear", "gls_newton_solve",
    "gls_bdf_coefficients", "gls_sdirk_coefficients", "gls_newton_selftest", "gls_mesh_hyper_cube_sizes",
    "gls_mesh_hyper_cube", "gls_timing_reset", "gls_timing_get", "gls_timing_enable", "gls_uses_brick_kernels",
    "gls_part_create", "gls_part_sizes", "gls_part_get", "gls_part_destroy", "gls_dist_attach", "gls_dist_import", "gls_rccl_unique_id", "gls_rccl_create", "gls_rccl_destroy", "gls_rccl_info", "gls_mg_smoother_apply", "gls_mg_attach_replica",
    "gls_dist_attach_rccl",
    "gls_mg_attach", "gls_mg_detach", "gls_mg_set_coarse_replica", "gls_residual_and_diagonal", "gls_octree_set_periodic", "gls_ilu_attach", "gls_ilu_detach", "gls_ilu_info", "gls_ilu_matrix", "gls_ilu_factors", "gls_ilu_set_options", "gls_iluk_pattern", "gls_cuthill_mckee", "gls_section_timing", "gls_section_get", "gls_dist_attach_dofs", "gls_dist_attach_dofs_rccl", "gls_gpart_create", "gls_gpart_sizes", "gls_gpart_get", "gls_gpart_map_dofs", "gls_gpart_destroy", "gls_dpart_create", "gls_set_lattice", "gls_apply_preconditioner", "gls_mg_transfer",
    "gls_prm_parse", "gls_prm_get", "gls_prm_n_entries", "gls_prm_entry", "gls_prm_destroy",
    "gls_expr_create", "gls_expr_n_components", "gls_expr_eval", "gls_expr_destroy",
    "gls_vtu_write", "gls_pvtu_write", "gls_pvd_write",
    "gls_set_hanging", "gls_mesh_refined_create", "gls_mesh_refined_destroy", "gls_octree_create", "gls_octree_destroy", "gls_octree_info",
    "gls_octree_cells", "gls_octree_adapt", "gls_octree_prepare", "gls_octree_mesh", "gls_octree_mesh_destroy", "gls_octree_transfer", "gls_octree_faces", "gls_kelly_estimate_faces",
    "gls_kelly_estimate", "gls_refine_fixed_number", "gls_mesh_refined_interpolate", "gls_refine_pd", "gls_refine_coarsen_pd",
    "gls_freeze_jacobian", "gls_skip_newton_selftest", "gls_quadrature_points",
    "gls_umesh_generate", "gls_umesh_read_gmsh", "gls_umesh_set_manifold", "gls_umesh_boundary_manifold",
    "gls_umesh_refine_global", "gls_umesh_info", "gls_umesh_destroy", "gls_umesh_fe_space", "gls_fe_space_destroy",
    "gls_fe_space_transfer", "gls_umesh_prepare", "gls_umesh_adapt", "gls_umesh_set_periodic", "gls_fe_space_kelly_faces",
    "gls_kelly_estimate_mapped", "gls_fe_space_boundary_normals", "gls_fe_space_boundary_normal_sets",
    "gls_octree_coarsen_to", "gls_octree_mg_transfer", "gls_mg_attach_transfers", "gls_umesh_coarsen_to",
    "gls_fe_space_mg_transfer", "gls_forest_bricks",
]


class GLSError(RuntimeError):
    pass


class MeshDesc(C.Structure):
    _fields_ = [
        ("dim", C.c_int), ("k", C.c_int), ("kp", C.c_int), ("nq1d", C.c_int), ("n_cells", C.c_int),
        ("n_vnodes", C.c_int), ("n_pnodes", C.c_int),
        ("cell_vnodes", C.POINTER(C.c_int32)), ("cell_pnodes", C.POINTER(C.c_int32)),
        ("cell_x0", C.POINTER(C.c_double)), ("cell_h", C.POINTER(C.c_double)),
        ("vnode_mask", C.POINTER(C.c_uint8)),
        ("viscosity", C.c_double), ("srf", C.c_int), ("omega", C.c_double * 3),
        ("force_q", C.POINTER(C.c_double)),
        ("map_degree", C.c_int), ("cell_support", C.POINTER(C.c_double)),
    ]


class FESpace(C.Structure):
    _fields_ = [("dim", C.c_int), ("k", C.c_int), ("kp", C.c_int),
                ("n_cells", C.c_int64), ("n_vnodes", C.c_int64), ("n_pnodes", C.c_int64),
                ("cell_vnodes", C.POINTER(C.c_int32)), ("cell_pnodes", C.POINTER(C.c_int32)),
                ("vnode_x", C.POINTER(C.c_double)), ("pnode_x", C.POINTER(C.c_double)),
                ("vnode_bid", C.POINTER(C.c_uint32)), ("pnode_bid", C.POINTER(C.c_uint32)),
                ("cell_support", C.POINTER(C.c_double)), ("cell_mapping", C.POINTER(C.c_int32)),
                ("cell_measure", C.POINTER(C.c_double)), ("volume", C.c_double),
                ("cell_level", C.POINTER(C.c_int32)),
                ("n_vhang", C.c_int64), ("vhang_node", C.POINTER(C.c_int64)), ("vhang_off", C.POINTER(C.c_int64)),
                ("vhang_master", C.POINTER(C.c_int64)), ("vhang_w", C.POINTER(C.c_double)),
                ("n_phang", C.c_int64), ("phang_node", C.POINTER(C.c_int64)), ("phang_off", C.POINTER(C.c_int64)),
                ("phang_master", C.POINTER(C.c_int64)), ("phang_w", C.POINTER(C.c_double)),
                ("impl_", C.c_void_p)]


class LinearParams(C.Structure):
    _fields_ = [("max_iterations", C.c_int), ("restart", C.c_int), ("relative_residual", C.c_double),
                ("minimum_residual", C.c_double), ("iterations", C.c_int), ("final_residual", C.c_double),
                ("method", C.c_int), ("orthogonalization", C.c_int), ("true_residual", C.c_int)]


LIN_METHODS = {"gmres": 0, "bicgstab": 1}
ORTHO = {"gram": 0, "cgs2": 1}


class MGParams(C.Structure):
    _fields_ = [("n_levels", C.c_int), ("levels", C.POINTER(C.c_void_p)), ("pre_smooth", C.c_int),
                ("post_smooth", C.c_int), ("coarse_sweeps", C.c_int), ("omega", C.c_double),
                ("coarse_omega", C.c_double), ("coarse_direct", C.c_int), ("mixed_precision", C.c_int),
                ("level_sweeps", C.POINTER(C.c_int)), ("smoother", C.c_int), ("smoother_operator", C.c_int)]


class RefinedMesh(C.Structure):
    _fields_ = [("dim", C.c_int), ("k", C.c_int), ("kp", C.c_int),
                ("n_cells", C.c_int64), ("n_vnodes", C.c_int64), ("n_pnodes", C.c_int64),
                ("cell_vnodes", C.POINTER(C.c_int32)), ("cell_pnodes", C.POINTER(C.c_int32)),
                ("cell_level", C.POINTER(C.c_int32)),
                ("cell_x0", C.POINTER(C.c_double)), ("cell_h", C.POINTER(C.c_double)),
                ("vnode_x", C.POINTER(C.c_double)), ("pnode_x", C.POINTER(C.c_double)),
                ("n_vhang", C.c_int64), ("vhang_node", C.POINTER(C.c_int64)), ("vhang_off", C.POINTER(C.c_int64)),
                ("vhang_master", C.POINTER(C.c_int64)), ("vhang_w", C.POINTER(C.c_double)),
                ("n_phang", C.c_int64), ("phang_node", C.POINTER(C.c_int64)), ("phang_off", C.POINTER(C.c_int64)),
                ("phang_master", C.POINTER(C.c_int64)), ("phang_w", C.POINTER(C.c_double)),
                ("impl_", C.c_void_p)]


class NewtonParams(C.Structure):
    _fields_ = [("tolerance", C.c_double), ("max_iterations", C.c_int), ("verbosity", C.c_int),
                ("lin", LinearParams), ("newton_iterations", C.c_int), ("linear_iterations", C.c_int),
                ("residual_evaluations", C.c_int), ("final_residual", C.c_double),
                ("solver", C.c_int), ("skip_iterations", C.c_int), ("is_initial_step", C.c_int),
                ("force_matrix_renewal", C.c_int), ("linear_failures", C.c_int)]


_lib = None


def load():
    """Load the HIP extension; raise loudly if it has not been built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise GLSError("HIP extension %s is missing — run `python -m softx_2020_200_amd.build` "
                       "(or __graft_entry__.build()); there is no CPU fallback" % LIB_PATH)
    L = C.CDLL(LIB_PATH)
    vp, d, i64 = C.c_void_p, C.POINTER(C.c_double), C.c_int64
    L.gls_last_error.restype = C.c_char_p
    L.gls_version.restype = C.c_char_p
    L.gls_create.argtypes = [C.POINTER(MeshDesc), C.POINTER(vp)]
    L.gls_destroy.argtypes = [vp]
    L.gls_set_stream.argtypes = [vp, vp]
    L.gls_n_dofs.argtypes = [vp, C.POINTER(i64)]
    L.gls_set_force.argtypes = [vp, d]
    L.gls_set_viscosity.argtypes = [vp, C.c_double]
    L.gls_set_time.argtypes = [vp, C.c_int, d]
    L.gls_set_state.argtypes = [vp, vp, vp, vp, vp]
    L.gls_residual.argtypes = [vp, vp]
    L.gls_jacobian_apply.argtypes = [vp, vp, vp]
    L.gls_jacobian_apply_f32.argtypes = [vp, vp, vp]
    L.gls_jacobian_diagonal.argtypes = [vp, vp]
    L.gls_residual_and_diagonal.argtypes = [vp, vp, vp]
    L.gls_set_dirichlet.argtypes = [vp, i64, C.POINTER(i64), d]
    L.gls_apply_dirichlet.argtypes = [vp, vp]
    L.gls_solve_linear.argtypes = [vp, vp, vp, C.POINTER(LinearParams)]
    L.gls_newton_solve.argtypes = [vp, vp, vp, vp, vp, C.POINTER(NewtonParams)]
    L.gls_bdf_coefficients.argtypes = [C.c_int, d, C.c_int, d]
    L.gls_sdirk_coefficients.argtypes = [C.c_int, C.c_double, d]
    L.gls_newton_selftest.argtypes = [d]
    L.gls_skip_newton_selftest.argtypes = [C.c_int, d]
    L.gls_freeze_jacobian.argtypes = [vp, C.c_int]
    L.gls_mesh_hyper_cube_sizes.argtypes = [C.c_int] * 5 + [C.POINTER(i64)] * 3
    L.gls_mesh_hyper_cube.argtypes = [C.c_int] * 4 + [C.c_double, C.c_double, C.c_int,
                                                      C.POINTER(C.c_int32), C.POINTER(C.c_int32), d, d]
    L.gls_timing_reset.argtypes = [vp]
    L.gls_timing_get.argtypes = [vp, C.c_int, d, C.POINTER(i64)]
    L.gls_timing_enable.argtypes = [vp, C.c_int]
    L.gls_uses_brick_kernels.argtypes = [vp]
    L.gls_mg_attach.argtypes = [vp, C.POINTER(MGParams)]
    L.gls_mg_detach.argtypes = [vp]
    L.gls_mg_set_coarse_replica.argtypes = [vp, vp, i64, C.POINTER(i64)]
    L.gls_mg_attach_transfers.argtypes = [vp, C.POINTER(MGParams), C.POINTER(C.POINTER(i64)),
                                          C.POINTER(C.POINTER(C.c_int32)), C.POINTER(C.POINTER(C.c_double)),
                                          C.POINTER(C.POINTER(i64))]
    L.gls_octree_coarsen_to.argtypes = [vp, C.c_int, C.POINTER(vp)]
    L.gls_umesh_coarsen_to.argtypes = [vp, C.c_int, C.POINTER(vp)]
    L.gls_forest_bricks.argtypes = [vp]
    L.gls_fe_space_mg_transfer.argtypes = [C.POINTER(FESpace), C.POINTER(FESpace), C.POINTER(i64), vp, vp, vp, vp]
    L.gls_octree_mg_transfer.argtypes = [C.POINTER(RefinedMesh), C.POINTER(RefinedMesh), C.POINTER(i64), vp, vp, vp, vp]
    L.gls_set_lattice.argtypes = [vp, C.c_int, C.POINTER(i64)]
    L.gls_apply_preconditioner.argtypes = [vp, vp, vp]
    L.gls_mg_smoother_apply.argtypes = [vp, vp, vp]
    L.gls_mg_attach_replica.argtypes = [vp, C.POINTER(MGParams), vp, C.POINTER(C.c_int64), C.POINTER(C.c_int32),
                                        C.POINTER(C.c_double), C.POINTER(C.c_int64)]
    L.gls_mg_transfer.argtypes = [vp, C.c_int, C.c_int, vp, vp]
    P64 = C.POINTER(i64)
    L.gls_set_hanging.argtypes = [vp, i64, P64, P64, P64, d]
    L.gls_mesh_refined_create.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.c_double, C.c_double,
                                          C.POINTER(C.c_int32), C.POINTER(C.POINTER(RefinedMesh))]
    L.gls_mesh_refined_destroy.argtypes = [C.POINTER(RefinedMesh)]
    L.gls_kelly_estimate.argtypes = [vp, vp, C.c_int, vp]
    L.gls_refine_fixed_number.argtypes = [i64, C.POINTER(C.c_float), C.c_double, C.POINTER(C.c_int32)]
    L.gls_refine_pd.argtypes = [i64, C.POINTER(C.c_float), C.c_int, C.c_int, C.c_double, i64,
                                C.POINTER(C.c_int32), C.POINTER(C.c_double)]
    L.gls_mesh_refined_interpolate.argtypes = [C.POINTER(RefinedMesh), C.c_int, C.c_double, C.c_double,
                                               C.POINTER(C.c_double), C.POINTER(C.c_double)]
    L.gls_quadrature_points.argtypes = [vp, d]
    L.gls_umesh_generate.argtypes = [C.c_int, C.c_char_p, C.c_char_p, C.POINTER(vp)]
    L.gls_umesh_read_gmsh.argtypes = [C.c_int, C.c_char_p, C.POINTER(vp)]
    L.gls_umesh_set_manifold.argtypes = [vp, C.c_int, C.c_int, d, d]
    L.gls_umesh_boundary_manifold.argtypes = [vp, C.c_int, C.c_int]
    L.gls_umesh_refine_global.argtypes = [vp, C.c_int]
    L.gls_umesh_info.argtypes = [vp, C.POINTER(i64), C.POINTER(i64), d]
    L.gls_umesh_destroy.argtypes = [vp]
    L.gls_umesh_destroy.restype = None
    L.gls_umesh_fe_space.argtypes = [vp, C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_int32),
                                     C.POINTER(C.POINTER(FESpace))]
    L.gls_fe_space_destroy.argtypes = [C.POINTER(FESpace)]
    L.gls_fe_space_transfer.argtypes = [C.POINTER(FESpace), C.POINTER(FESpace), d, d]
    pi32 = C.POINTER(C.c_int32)
    L.gls_umesh_prepare.argtypes = [vp, pi32, pi32]
    L.gls_umesh_adapt.argtypes = [vp, pi32, pi32]
    L.gls_umesh_set_periodic.argtypes = [vp, C.c_int, pi32]
    L.gls_fe_space_kelly_faces.argtypes = [C.POINTER(FESpace), C.c_int, C.POINTER(i64), pi32, pi32, d, d, d, d]
    L.gls_fe_space_boundary_normals.argtypes = [C.POINTER(FESpace), C.c_int, d]
    L.gls_fe_space_boundary_normal_sets.argtypes = [C.POINTER(FESpace), C.c_int, C.POINTER(C.c_int32), d]
    L.gls_kelly_estimate_mapped.argtypes = [vp, vp, C.c_int, i64, C.c_int, pi32, pi32, d, d, d, d, vp]
    _lib = L
    return L


def check(rc, what=""):
    if rc < 0:
        msg = load().gls_last_error().decode()
        raise GLSError("%s failed (%d): %s" % (what, rc, msg))
    return rc


def _dp(a):
    return a.ctypes.data_as(C.POINTER(C.c_double)) if a is not None else C.POINTER(C.c_double)()


# ---------------------------------------------------------------------------------------------
# host-only helpers (no GPU needed)
# ---------------------------------------------------------------------------------------------
def bdf_coefficients(order, dts):
    dts = np.ascontiguousarray(dts, dtype=np.float64)
    out = np.zeros(order + 1)
    check(load().gls_bdf_coefficients(order, _dp(dts), len(dts), _dp(out)), "gls_bdf_coefficients")
    return out


def sdirk_coefficients(order, dt):
    out = np.zeros(order * (order + 1))
    check(load().gls_sdirk_coefficients(order, dt, _dp(out)), "gls_sdirk_coefficients")
    return out.reshape(order, order + 1)


def newton_selftest():
    out = np.zeros(2)
    check(load().gls_newton_selftest(_dp(out)), "gls_newton_selftest")
    return out


def skip_newton_selftest(skip_iterations=1):
    out = np.zeros(2)
    check(load().gls_skip_newton_selftest(int(skip_iterations), _dp(out)), "gls_skip_newton_selftest")
    return out


def hyper_cube(dim, n, k, kp=None, lo=-1.0, hi=1.0, periodic=()):
    """GridGenerator::hyper_cube + refine_global through the C++ mesh builder (Morton cells)."""
    kp = k if kp is None else kp
    L = load()
    pm = sum(1 << d for d in periodic)
    nc, nv, npn = C.c_int64(), C.c_int64(), C.c_int64()
    check(L.gls_mesh_hyper_cube_sizes(dim, n, k, kp, pm, C.byref(nc), C.byref(nv), C.byref(npn)), "mesh sizes")
    nc, nv, npn = nc.value, nv.value, npn.value
    cv = np.zeros((nc, (k + 1) ** dim), dtype=np.int32)
    cp = np.zeros((nc, (kp + 1) ** dim), dtype=np.int32)
    x0 = np.zeros((nc, dim))
    h = np.zeros((nc, dim))
    check(L.gls_mesh_hyper_cube(dim, n, k, kp, lo, hi, pm, cv.ctypes.data_as(C.POINTER(C.c_int32)),
                                cp.ctypes.data_as(C.POINTER(C.c_int32)), _dp(x0), _dp(h)), "gls_mesh_hyper_cube")
    return dict(dim=dim, k=k, kp=kp, n_cells=nc, n_vnodes=nv, n_pnodes=npn, cell_vnodes=cv, cell_pnodes=cp,
                cell_x0=x0, cell_h=h)


def refined_cube(dim, n, k, kp=None, refine=None, lo=-1.0, hi=1.0):
    """hyper_cube(lo, hi) with n^dim cells, the flagged cells (refine[n^dim], lexicographic) split
    once more; hanging-node constraint lines per node (C++ builder, gls_mesh_refined_create)."""
    kp = k if kp is None else kp
    L = load()
    nc = n ** dim
    flags = np.zeros(nc, dtype=np.int32) if refine is None else np.ascontiguousarray(refine, dtype=np.int32)
    if flags.size != nc:
        raise GLSError("refine must hold n^dim flags")
    pm = C.POINTER(RefinedMesh)()
    check(L.gls_mesh_refined_create(dim, n, k, kp, lo, hi, flags.ctypes.data_as(C.POINTER(C.c_int32)),
                                    C.byref(pm)), "gls_mesh_refined_create")
    try:
        return _refined_mesh_dict(pm, dim, k, kp)
    finally:
        L.gls_mesh_refined_destroy(pm)


def _refined_mesh_dict(pm, dim, k, kp):
    """Copy a gls_refined_mesh (cells, node coordinates, node-level hanging lines) into numpy arrays."""
    if True:
        m = pm.contents

        def take(ptr, count, dt, shape=None):
            a = np.ctypeslib.as_array(ptr, shape=(int(count),)).astype(dt, copy=True) if count else np.zeros(0, dt)
            return a.reshape(shape) if shape is not None else a

        ncl = int(m.n_cells)
        out = dict(dim=dim, k=k, kp=kp, n_cells=ncl, n_vnodes=int(m.n_vnodes), n_pnodes=int(m.n_pnodes),
                   cell_vnodes=take(m.cell_vnodes, ncl * (k + 1) ** dim, np.int32, (ncl, (k + 1) ** dim)),
                   cell_pnodes=take(m.cell_pnodes, ncl * (kp + 1) ** dim, np.int32, (ncl, (kp + 1) ** dim)),
                   cell_level=take(m.cell_level, ncl, np.int32),
                   cell_x0=take(m.cell_x0, ncl * dim, np.float64, (ncl, dim)),
                   cell_h=take(m.cell_h, ncl * dim, np.float64, (ncl, dim)),
                   vnode_x=take(m.vnode_x, m.n_vnodes * dim, np.float64, (int(m.n_vnodes), dim)),
                   pnode_x=take(m.pnode_x, m.n_pnodes * dim, np.float64, (int(m.n_pnodes), dim)))
        for tag, nh in (("v", int(m.n_vhang)), ("p", int(m.n_phang))):
            offs = take(getattr(m, tag + "hang_off"), nh + 1, np.int64)
            nm = int(offs[-1]) if nh else 0
            out[tag + "hang"] = (take(getattr(m, tag + "hang_node"), nh, np.int64), offs,
                                 take(getattr(m, tag + "hang_master"), nm, np.int64),
                                 take(getattr(m, tag + "hang_w"), nm, np.float64))
        return out


class Octree:
    """Multi-level adaptive hyper_cube (gls_octree_*): p4est-style refine / coarsen with vertex 2:1
    balance; mesh(k, kp) gives the refined_cube-style dict with closed hanging-node lines."""

    def __init__(self, dim, n, lo=-1.0, hi=1.0):
        self.L = load()
        self.L.gls_octree_create.argtypes = [C.c_int, C.c_int, C.POINTER(C.c_void_p)]
        self.L.gls_octree_destroy.argtypes = [C.c_void_p]
        self.L.gls_octree_set_periodic.argtypes = [C.c_void_p, C.c_int]
        self.L.gls_octree_info.argtypes = [C.c_void_p, C.POINTER(C.c_int64), C.POINTER(C.c_int)]
        self.L.gls_octree_cells.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_double, C.c_double]
        self.L.gls_octree_adapt.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int]
        self.L.gls_octree_mesh.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_double, C.c_double,
                                           C.POINTER(C.POINTER(RefinedMesh))]
        self.L.gls_octree_mesh_destroy.argtypes = [C.POINTER(RefinedMesh)]
        self.L.gls_octree_transfer.argtypes = [C.POINTER(RefinedMesh), C.POINTER(RefinedMesh), C.c_void_p, C.c_void_p]
        self.dim, self.n, self.lo, self.hi = dim, n, lo, hi
        self.h = C.c_void_p()
        check(self.L.gls_octree_create(dim, n, C.byref(self.h)), "gls_octree_create")

    def __del__(self):
        if getattr(self, "h", None):
            self.L.gls_octree_destroy(self.h)

    def coarsen_to(self, level):
        """The forest with every leaf finer than `level` replaced by its ancestor on `level`
        (gls_octree_coarsen_to): a level mesh of the multigrid on the refinement hierarchy."""
        out = Octree.__new__(Octree)
        out.L, out.dim, out.n, out.lo, out.hi = self.L, self.dim, self.n, self.lo, self.hi
        out.h = C.c_void_p()
        check(self.L.gls_octree_coarsen_to(self.h, int(level), C.byref(out.h)), "gls_octree_coarsen_to")
        return out

    def set_periodic(self, mask):
        """periodic directions (bit d), before adapting: neighbourhoods wrap, mesh() identifies the faces"""
        check(self.L.gls_octree_set_periodic(self.h, int(mask)), "gls_octree_set_periodic")

    @property
    def n_cells(self):
        nc, ml = C.c_int64(), C.c_int()
        check(self.L.gls_octree_info(self.h, C.byref(nc), C.byref(ml)), "gls_octree_info")
        return nc.value

    @property
    def max_level(self):
        nc, ml = C.c_int64(), C.c_int()
        check(self.L.gls_octree_info(self.h, C.byref(nc), C.byref(ml)), "gls_octree_info")
        return ml.value

    def cells(self):
        nc = self.n_cells
        lev = np.zeros(nc, dtype=np.int32)
        x0 = np.zeros((nc, self.dim))
        h = np.zeros((nc, self.dim))
        check(self.L.gls_octree_cells(self.h, lev.ctypes.data, x0.ctypes.data, h.ctypes.data, self.lo, self.hi),
              "gls_octree_cells")
        return lev, x0, h

    def adapt(self, refine=None, coarsen=None, max_level=30, min_level=0):
        nc = self.n_cells
        r = np.zeros(nc, np.int32) if refine is None else np.ascontiguousarray(refine, dtype=np.int32)
        c = np.zeros(nc, np.int32) if coarsen is None else np.ascontiguousarray(coarsen, dtype=np.int32)
        check(self.L.gls_octree_adapt(self.h, r.ctypes.data, c.ctypes.data, int(max_level), int(min_level)),
              "gls_octree_adapt")

    def prepare(self, refine, coarsen):
        """Triangulation::prepare_coarsening_and_refinement with the reference's mesh smoothing
        (gls_octree_prepare; navier_stokes_base.cc:55-60, 682). Returns (refine, coarsen, loops)."""
        nc = self.n_cells
        r = np.array(refine, dtype=np.int32).reshape(nc)
        c = np.array(coarsen, dtype=np.int32).reshape(nc)
        self.L.gls_octree_prepare.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
        loops = self.L.gls_octree_prepare(self.h, r.ctypes.data, c.ctypes.data)
        check(min(loops, 0), "gls_octree_prepare")
        return r, c, loops

    def mesh_handle(self, k, kp=None):
        """Owned gls_refined_mesh pointer (free with free_mesh_handle)."""
        kp = k if kp is None else kp
        pm = C.POINTER(RefinedMesh)()
        check(self.L.gls_octree_mesh(self.h, k, kp, self.lo, self.hi, C.byref(pm)), "gls_octree_mesh")
        return pm

    def free_mesh_handle(self, pm):
        self.L.gls_octree_mesh_destroy(pm)

    def faces(self, k=1, kp=None):
        """Interior face pieces for Kelly (gls_octree_faces): (fa, fb, fdir, rect_a, rect_b)."""
        pm = self.mesh_handle(k, kp)
        try:
            self.L.gls_octree_faces.argtypes = [C.POINTER(RefinedMesh), C.POINTER(C.c_int64)] + [C.c_void_p] * 5
            n = C.c_int64()
            check(self.L.gls_octree_faces(pm, C.byref(n), None, None, None, None, None), "gls_octree_faces")
            fa, fb, fd = (np.zeros(n.value, np.int32) for _ in range(3))
            ra, rb = np.zeros((n.value, 4)), np.zeros((n.value, 4))
            check(self.L.gls_octree_faces(pm, C.byref(n), fa.ctypes.data, fb.ctypes.data, fd.ctypes.data, ra.ctypes.data,
                                          rb.ctypes.data), "gls_octree_faces")
            return fa, fb, fd, ra, rb
        finally:
            self.free_mesh_handle(pm)

    def mesh(self, k, kp=None):
        kp = k if kp is None else kp
        pm = self.mesh_handle(k, kp)
        try:
            return _refined_mesh_dict(pm, self.dim, k, kp)
        finally:
            self.free_mesh_handle(pm)


def octree_mg_transfer(fine_handle, coarse_handle):
    """Prolongation CSR (off, col, w) over the fine DoFs and the state injection (coarse DoF -> fine DoF)
    between two nested octree meshes (gls_octree_mg_transfer; handles from Octree.mesh_handle)."""
    L = load()
    nnz = C.c_int64()
    check(L.gls_octree_mg_transfer(fine_handle, coarse_handle, C.byref(nnz), None, None, None, None),
          "gls_octree_mg_transfer")
    f, c = fine_handle.contents, coarse_handle.contents
    nf = f.dim * f.n_vnodes + f.n_pnodes
    nc = c.dim * c.n_vnodes + c.n_pnodes
    off = np.zeros(nf + 1, np.int64)
    col = np.zeros(max(nnz.value, 1), np.int32)
    w = np.zeros(max(nnz.value, 1))
    inj = np.zeros(nc, np.int64)
    check(L.gls_octree_mg_transfer(fine_handle, coarse_handle, C.byref(nnz), off.ctypes.data, col.ctypes.data,
                                   w.ctypes.data, inj.ctypes.data), "gls_octree_mg_transfer")
    return off, col[:nnz.value], w[:nnz.value], inj


def octree_transfer(old_handle, new_handle, vec, n_new):
    """SolutionTransfer between two octree meshes (gls_octree_transfer; host vectors)."""
    L = load()
    src = np.ascontiguousarray(vec, dtype=np.float64)
    out = np.zeros(n_new)
    check(L.gls_octree_transfer(old_handle, new_handle, src.ctypes.data, out.ctypes.data), "gls_octree_transfer")
    return out


def refine_fixed_number(criteria, top_fraction):
    """GridRefinement::refine_and_coarsen_fixed_number, refinement flags (gls_refine_fixed_number)."""
    c = np.ascontiguousarray(criteria, dtype=np.float32)
    flags = np.zeros(c.size, dtype=np.int32)
    rc = load().gls_refine_fixed_number(c.size, c.ctypes.data_as(C.POINTER(C.c_float)), float(top_fraction),
                                        flags.ctypes.data_as(C.POINTER(C.c_int32)))
    check(min(rc, 0), "gls_refine_fixed_number")
    return flags


def refine_pd(criteria, dim, top_fraction, fraction_type="number", max_n_cells=100000000):
    """parallel::distributed::GridRefinement::refine_and_coarsen_fixed_number / _fixed_fraction,
    refinement flags (gls_refine_pd; navier_stokes_base.cc:654-667). Returns (flags, threshold)."""
    c = np.ascontiguousarray(criteria, dtype=np.float32)
    flags = np.zeros(c.size, dtype=np.int32)
    thr = C.c_double(0.0)
    ft = {"number": 0, "fraction": 1}[fraction_type]
    rc = load().gls_refine_pd(c.size, c.ctypes.data_as(C.POINTER(C.c_float)), int(dim), ft, float(top_fraction),
                              int(max_n_cells), flags.ctypes.data_as(C.POINTER(C.c_int32)), C.byref(thr))
    check(min(rc, 0), "gls_refine_pd")
    return flags, thr.value


def refine_coarsen_pd(criteria, dim, top_fraction, bottom_fraction, fraction_type="number", max_n_cells=100000000):
    """parallel::distributed::GridRefinement::refine_and_coarsen_fixed_number / _fixed_fraction with
    coarsening (gls_refine_coarsen_pd; navier_stokes_base.cc:654-667). Returns (refine, coarsen,
    (top threshold, bottom threshold))."""
    c = np.ascontiguousarray(criteria, dtype=np.float32)
    r, k = np.zeros(c.size, dtype=np.int32), np.zeros(c.size, dtype=np.int32)
    th = (C.c_double * 2)()
    ft = {"number": 0, "fraction": 1}[fraction_type]
    L = load()
    L.gls_refine_coarsen_pd.argtypes = [C.c_int64, C.c_void_p, C.c_int, C.c_int, C.c_double, C.c_double, C.c_int64,
                                        C.c_void_p, C.c_void_p, C.c_void_p]
    rc = L.gls_refine_coarsen_pd(c.size, c.ctypes.data, int(dim), ft, float(top_fraction), float(bottom_fraction),
                                 int(max_n_cells), r.ctypes.data, k.ctypes.data, th)
    check(min(rc, 0), "gls_refine_coarsen_pd")
    return r, k, (th[0], th[1])


def refined_interpolate(dim, n, k, kp, refine, coarse, lo=-1.0, hi=1.0):
    """SolutionTransfer::interpolate of a hyper_cube(n) solution onto refined_cube(dim, n, k, kp,
    refine) (gls_mesh_refined_interpolate; host arrays)."""
    L = load()
    flags = np.ascontiguousarray(refine, dtype=np.int32)
    pm = C.POINTER(RefinedMesh)()
    check(L.gls_mesh_refined_create(dim, n, k, kp, lo, hi, flags.ctypes.data_as(C.POINTER(C.c_int32)),
                                    C.byref(pm)), "gls_mesh_refined_create")
    try:
        m = pm.contents
        fine = np.zeros(dim * int(m.n_vnodes) + int(m.n_pnodes))
        src = np.ascontiguousarray(coarse, dtype=np.float64)
        check(L.gls_mesh_refined_interpolate(pm, n, lo, hi, _dp(src), _dp(fine)), "gls_mesh_refined_interpolate")
        return fine
    finally:
        L.gls_mesh_refined_destroy(pm)


def hanging_dof_lines(mesh):
    """node-level hanging lines of refined_cube -> DoF-level CSR (dofs, offsets, masters, weights):
    velocity DoF node*dim + c per component, pressure DoF dim*n_vnodes + node."""
    dim, nv = mesh["dim"], mesh["n_vnodes"]
    dofs, offs, mas, ws = [], [0], [], []
    vn, vo, vm, vw = mesh["vhang"]
    for i, nd in enumerate(vn):
        sl = slice(vo[i], vo[i + 1])
        for c in range(dim):
            dofs.append(nd * dim + c)
            mas.extend((vm[sl] * dim + c).tolist())
            ws.extend(vw[sl].tolist())
            offs.append(len(mas))
    pn, po, pmas, pw = mesh["phang"]
    for i, nd in enumerate(pn):
        sl = slice(po[i], po[i + 1])
        dofs.append(dim * nv + nd)
        mas.extend((dim * nv + pmas[sl]).tolist())
        ws.extend(pw[sl].tolist())
        offs.append(len(mas))
    return (np.array(dofs, dtype=np.int64), np.array(offs, dtype=np.int64), np.array(mas, dtype=np.int64),
            np.array(ws, dtype=np.float64))


# ---------------------------------------------------------------------------------------------
# device context
# ---------------------------------------------------------------------------------------------
def _ptr(t):
    if t is None:
        return None
    import torch
    if not isinstance(t, torch.Tensor) or not t.is_cuda or t.dtype != torch.float64 or not t.is_contiguous():
        raise GLSError("expected a contiguous float64 CUDA (HIP) tensor")
    return C.c_void_p(t.data_ptr())


class GLSContext:
    """Owner of one gls_ctx (one GPU). Vectors are torch float64 tensors on cuda."""

    def __init__(self, dim, k, kp, cell_vnodes, cell_pnodes, cell_h, n_vnodes, n_pnodes, viscosity=1.0,
                 cell_x0=None, vnode_mask=None, force_q=None, srf=False, omega=(0.0, 0.0, 0.0), nq1d=0,
                 stream=None, map_degree=0, cell_support=None):
        import torch
        if not torch.cuda.is_available():
            raise GLSError("no HIP device visible: the GLS operators run only on the GPU")
        self.L = load()
        self.dim, self.k, self.kp = dim, k, kp
        keep = []

        def arr(a, dt):
            if a is None:
                return None
            a = np.ascontiguousarray(a, dtype=dt)
            keep.append(a)
            return a

        cv = arr(cell_vnodes, np.int32)
        cp = arr(cell_pnodes, np.int32) if (cell_pnodes is not None and kp != k) else None
        if cp is None and kp != k:
            raise GLSError("cell_pnodes required for kp != k")
        hh = arr(cell_h, np.float64)
        x0 = arr(cell_x0, np.float64)
        vm = arr(vnode_mask, np.uint8)
        fq = arr(force_q, np.float64)
        D = MeshDesc()
        D.dim, D.k, D.kp, D.nq1d = dim, k, kp, nq1d
        D.n_cells = cv.shape[0]
        D.n_vnodes, D.n_pnodes = int(n_vnodes), int(n_pnodes)
        D.cell_vnodes = cv.ctypes.data_as(C.POINTER(C.c_int32))
        D.cell_pnodes = cp.ctypes.data_as(C.POINTER(C.c_int32)) if cp is not None else C.POINTER(C.c_int32)()
        D.cell_x0 = _dp(x0)
        D.cell_h = _dp(hh)
        D.vnode_mask = vm.ctypes.data_as(C.POINTER(C.c_uint8)) if vm is not None else C.POINTER(C.c_uint8)()
        D.viscosity = viscosity
        D.srf = 1 if srf else 0
        for i in range(3):
            D.omega[i] = omega[i]
        D.force_q = _dp(fq)
        if map_degree:  # mapped (curved / unstructured) cells: MappingQ support points per cell
            D.map_degree = int(map_degree)
            D.cell_support = _dp(arr(cell_support, np.float64))
        h = C.c_void_p()
        check(self.L.gls_create(C.byref(D), C.byref(h)), "gls_create")
        self.h = h
        n = C.c_int64()
        check(self.L.gls_n_dofs(self.h, C.byref(n)), "gls_n_dofs")
        self.n_dofs = n.value
        self.n_cells = D.n_cells
        self.n_vnodes, self.n_pnodes = D.n_vnodes, D.n_pnodes
        # stream-ordered with torch: run on the caller's current torch stream unless told otherwise
        if stream is None:
            stream = torch.cuda.current_stream().cuda_stream
        self.stream = stream
        check(self.L.gls_set_stream(self.h, C.c_void_p(stream)), "gls_set_stream")
        self._state = None
        self.nq = (nq1d or (k + 1)) ** dim

    def quadrature_points(self):
        """physical QGauss points [n_cells, nq, dim] (gls_quadrature_points; mapped for curved cells)"""
        out = np.zeros((self.n_cells, self.nq, self.dim))
        check(self.L.gls_quadrature_points(self.h, _dp(out)), "gls_quadrature_points")
        return out

    def close(self):
        if getattr(self, "h", None):
            self.L.gls_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def uses_brick_kernels(self):
        return bool(self.L.gls_uses_brick_kernels(self.h))

    def zeros(self):
        import torch
        return torch.zeros(self.n_dofs, dtype=torch.float64, device="cuda")

    def set_time(self, scheme, time_steps=(1.0, 1.0, 1.0, 1.0)):
        ts = np.zeros(4)
        ts[:len(time_steps)] = time_steps[:4]
        check(self.L.gls_set_time(self.h, SCHEMES[scheme] if isinstance(scheme, str) else scheme, _dp(ts)),
              "gls_set_time")

    def set_state(self, u, u1=None, u2=None, u3=None):
        self._state = (u, u1, u2, u3)  # keep tensors alive while borrowed
        check(self.L.gls_set_state(self.h, _ptr(u), _ptr(u1), _ptr(u2), _ptr(u3)), "gls_set_state")

    def forest_bricks(self):
        """sibling-group bricks of an adapted forest that run the pencil kernel (gls_forest_bricks)"""
        return int(self.L.gls_forest_bricks(self.h))

    def set_hanging(self, dofs, offsets, masters, weights):
        """Hanging-node constraint lines (gls_set_hanging): DoF dofs[i] = sum w * masters."""
        arrs = [np.ascontiguousarray(a, dtype=t) for a, t in ((dofs, np.int64), (offsets, np.int64),
                                                               (masters, np.int64), (weights, np.float64))]
        P64 = C.POINTER(C.c_int64)
        check(self.L.gls_set_hanging(self.h, len(arrs[0]), arrs[0].ctypes.data_as(P64), arrs[1].ctypes.data_as(P64),
                                     arrs[2].ctypes.data_as(P64), _dp(arrs[3])), "gls_set_hanging")

    def set_force(self, force_q):
        f = None if force_q is None else np.ascontiguousarray(force_q, dtype=np.float64)
        check(self.L.gls_set_force(self.h, _dp(f)), "gls_set_force")

    def set_viscosity(self, nu):
        check(self.L.gls_set_viscosity(self.h, nu), "gls_set_viscosity")

    def residual(self, out=None):
        out = self.zeros() if out is None else out
        check(self.L.gls_residual(self.h, _ptr(out)), "gls_residual")
        return out

    def jacobian_apply(self, v, out=None):
        out = self.zeros() if out is None else out
        check(self.L.gls_jacobian_apply(self.h, _ptr(v), _ptr(out)), "gls_jacobian_apply")
        return out

    def jacobian_apply_f32(self, v, out=None):
        """J.v in FP32 arithmetic (the mixed-precision V-cycle's operator); FP64 in/out vectors."""
        out = self.zeros() if out is None else out
        check(self.L.gls_jacobian_apply_f32(self.h, _ptr(v), _ptr(out)), "gls_jacobian_apply_f32")
        return out

    def residual_and_diagonal(self, out=None, diag=None):
        """assemble_matrix_and_rhs: the residual and the Jacobian diagonal at the current state (one
        fused launch on the Q2 brick path); returns (residual, diagonal)."""
        out = self.zeros() if out is None else out
        diag = self.zeros() if diag is None else diag
        check(self.L.gls_residual_and_diagonal(self.h, _ptr(out), _ptr(diag)), "gls_residual_and_diagonal")
        return out, diag

    def jacobian_diagonal(self, out=None):
        out = self.zeros() if out is None else out
        check(self.L.gls_jacobian_diagonal(self.h, _ptr(out)), "gls_jacobian_diagonal")
        return out

    def set_dirichlet(self, dofs, values):
        dofs = np.ascontiguousarray(dofs, dtype=np.int64)
        vals = np.ascontiguousarray(values, dtype=np.float64)
        self._dir = (dofs, vals)
        check(self.L.gls_set_dirichlet(self.h, len(dofs), dofs.ctypes.data_as(C.POINTER(C.c_int64)), _dp(vals)),
              "gls_set_dirichlet")

    def apply_dirichlet(self, x):
        check(self.L.gls_apply_dirichlet(self.h, _ptr(x)), "gls_apply_dirichlet")
        return x

    def solve_linear(self, rhs, x=None, max_iterations=1000, restart=30, relative_residual=1e-4,
                     minimum_residual=1e-12, method="gmres", orthogonalization="gram", true_residual=False):
        """solve_system_GMRES / solve_system_BiCGStab (method="bicgstab") with the attached preconditioner.
        orthogonalization: GMRES's "gram" (Gram-corrected single pass) or "cgs2"; true_residual: report
        ||b - A x|| at convergence instead of the Krylov recurrence estimate."""
        x = self.zeros() if x is None else x
        p = LinearParams(max_iterations, restart, relative_residual, minimum_residual, 0, 0.0,
                         LIN_METHODS[method], ORTHO[orthogonalization], int(bool(true_residual)))
        rc = self.L.gls_solve_linear(self.h, _ptr(rhs), _ptr(x), C.byref(p))
        if rc < 0 and rc != GLS_ENOCONV:
            check(rc, "gls_solve_linear")
        return x, p.iterations, p.final_residual, rc == GLS_OK

    def newton(self, present, u1=None, u2=None, u3=None, tolerance=1e-8, max_iterations=10, verbosity=0,
               lin_max_iterations=1000, restart=30, relative_residual=1e-4, minimum_residual=1e-12,
               solver="newton", skip_iterations=1, is_initial_step=False, force_matrix_renewal=False,
               lin_method="gmres", orthogonalization="gram"):
        """NewtonNonLinearSolver::solve / SkipNewtonNonLinearSolver::solve (solver="skip_newton");
        lin_method: the linear solver ("gmres" | "bicgstab")."""
        self._state = (present, u1, u2, u3)
        lp = LinearParams(lin_max_iterations, restart, relative_residual, minimum_residual, 0, 0.0,
                          LIN_METHODS[lin_method], ORTHO[orthogonalization], 0)
        p = NewtonParams(tolerance, max_iterations, verbosity, lp, 0, 0, 0, 0.0,
                         {"newton": 0, "skip_newton": 1}[solver], int(skip_iterations), int(is_initial_step),
                         int(force_matrix_renewal), 0)
        check(self.L.gls_newton_solve(self.h, _ptr(present), _ptr(u1), _ptr(u2), _ptr(u3), C.byref(p)),
              "gls_newton_solve")
        return dict(newton_iterations=p.newton_iterations, linear_iterations=p.linear_iterations,
                    residual_evaluations=p.residual_evaluations, final_residual=p.final_residual,
                    linear_failures=p.linear_failures)

    def freeze_jacobian(self, freeze=True):
        """Keep the Jacobian operators at the current state (skip_newton matrix reuse)."""
        check(self.L.gls_freeze_jacobian(self.h, 1 if freeze else 0), "gls_freeze_jacobian")

    def attach_multigrid(self, coarse_levels, pre_smooth=2, post_smooth=2, coarse_sweeps=30, omega=0.6,
                         coarse_omega=0.0, coarse_direct=0, mixed_precision=0, level_sweeps=None, smoother_operator=0):
        """GMRES right preconditioner = geometric multigrid V-cycle over [self] + coarse_levels
        (GLSContext objects of the same problem on hyper_cube(n/2^l)). Keeps references alive.
        level_sweeps: optional {level: (pre, post)} overriding pre_smooth / post_smooth per level
        (negative level indices count from the coarsest). smoother_operator=1: the FP32 smoothing J.v
        applies the Oseen (Picard) linearization (gls_mg_params.smoother_operator)."""
        levels = [self] + list(coarse_levels)
        arr = (C.c_void_p * len(levels))(*[lv.h for lv in levels])
        ls = None
        if level_sweeps:
            pre0 = pre_smooth if pre_smooth > 0 else (0 if pre_smooth < 0 else 2)
            post0 = post_smooth if post_smooth >= 0 else 2
            flat = [pre0, post0] * len(levels)
            for lv, (a, b) in level_sweeps.items():
                flat[2 * (lv % len(levels))], flat[2 * (lv % len(levels)) + 1] = a, b
            ls = (C.c_int * len(flat))(*flat)
        p = MGParams(len(levels), C.cast(arr, C.POINTER(C.c_void_p)), pre_smooth, post_smooth, coarse_sweeps, omega,
                     coarse_omega, coarse_direct, int(mixed_precision), ls, 0, int(smoother_operator))
        check(self.L.gls_mg_attach(self.h, C.byref(p)), "gls_mg_attach")
        self._mg_levels = levels

    def attach_multigrid_transfers(self, coarse_levels, transfers, pre_smooth=2, post_smooth=2, coarse_sweeps=30,
                                   omega=0.6, coarse_omega=0.0, coarse_direct=0, level_sweeps=None, smoother="jacobi",
                                   mixed_precision=0):
        """The V-cycle on a general hierarchy (gls_mg_attach_transfers): levels [self] + coarse_levels
        (hanging lines set on each), transfers[l] = (off, col, w, inject) from level l+1 to level l
        (octree_mg_transfer). Smoothing: damped Jacobi, or smoother="ilu" (ILU(0) per level); mixed_precision=1:
        the levels' forest bricks apply the pencil J.v in FP32 (the other cells stay FP64)."""
        levels = [self] + list(coarse_levels)
        if len(transfers) != len(levels) - 1:
            raise GLSError("attach_multigrid_transfers: one transfer per level pair")
        arr = (C.c_void_p * len(levels))(*[lv.h for lv in levels])
        ls = None
        if level_sweeps:
            pre0 = pre_smooth if pre_smooth > 0 else (0 if pre_smooth < 0 else 2)
            post0 = post_smooth if post_smooth >= 0 else 2
            flat = [pre0, post0] * len(levels)
            for lv, (a, b) in level_sweeps.items():
                flat[2 * (lv % len(levels))], flat[2 * (lv % len(levels)) + 1] = a, b
            ls = (C.c_int * len(flat))(*flat)
        keep = [(np.ascontiguousarray(o, np.int64), np.ascontiguousarray(c, np.int32), np.ascontiguousarray(w, np.float64),
                 np.ascontiguousarray(j, np.int64)) for o, c, w, j in transfers]
        P64, P32, PD = C.POINTER(C.c_int64), C.POINTER(C.c_int32), C.POINTER(C.c_double)
        offs = (P64 * len(keep))(*[k[0].ctypes.data_as(P64) for k in keep])
        cols = (P32 * len(keep))(*[k[1].ctypes.data_as(P32) for k in keep])
        ws = (PD * len(keep))(*[k[2].ctypes.data_as(PD) for k in keep])
        injs = (P64 * len(keep))(*[k[3].ctypes.data_as(P64) for k in keep])
        p = MGParams(len(levels), C.cast(arr, C.POINTER(C.c_void_p)), pre_smooth, post_smooth, coarse_sweeps, omega,
                     coarse_omega, coarse_direct, int(mixed_precision), ls, {"jacobi": 0, "ilu": 1, "ilu-coarse": 2}[smoother])
        check(self.L.gls_mg_attach_transfers(self.h, C.byref(p), offs, cols, ws, injs), "gls_mg_attach_transfers")
        self._mg_levels = levels

    def attach_multigrid_replica(self, replica, p_off, p_col, p_w, inject_local, pre_smooth=2, post_smooth=2,
                                 omega=0.6, smoother="jacobi", coarse_direct=0):
        """The refinement-hierarchy V-cycle across ranks (gls_mg_attach_replica): this distributed fine
        context smooths its rows, `replica` (a single-rank context of the whole level-1 mesh with its own
        hierarchy attached) runs the coarser levels on every rank; P on the local fine rows (replica columns),
        inject_local = the local fine DoF a replica DoF's state comes from where this rank owns it, else -1;
        coarse_direct=1 with a replica without its own hierarchy: the exact solve on it (two-level cycle)."""
        keep = (np.ascontiguousarray(p_off, np.int64), np.ascontiguousarray(p_col, np.int32),
                np.ascontiguousarray(p_w, np.float64), np.ascontiguousarray(inject_local, np.int64))
        arr = (C.c_void_p * 1)(self.h)
        p = MGParams(1, C.cast(arr, C.POINTER(C.c_void_p)), pre_smooth, post_smooth, 0, omega, 0.0, int(coarse_direct), 0,
                     None, {"jacobi": 0, "ilu": 1}[smoother], 0)
        check(self.L.gls_mg_attach_replica(self.h, C.byref(p), replica.h, keep[0].ctypes.data_as(C.POINTER(C.c_int64)),
                                           keep[1].ctypes.data_as(C.POINTER(C.c_int32)),
                                           keep[2].ctypes.data_as(C.POINTER(C.c_double)),
                                           keep[3].ctypes.data_as(C.POINTER(C.c_int64))), "gls_mg_attach_replica")
        self._mg_replica = (replica, keep)

    def set_coarse_replica(self, replica, local_to_replica):
        """Multi-GPU V-cycle below the coarsest distributed level = the single-GPU one, run redundantly on
        every rank by `replica` (a single-rank GLSContext of that level's whole mesh with its own
        attach_multigrid hierarchy); local_to_replica: replica row of each local row of that level."""
        m = np.ascontiguousarray(local_to_replica, dtype=np.int64)
        check(self.L.gls_mg_set_coarse_replica(self.h, replica.h, len(m), m.ctypes.data_as(C.POINTER(C.c_int64))),
              "gls_mg_set_coarse_replica")
        self._coarse_replica = replica

    def mg_smoother_apply(self, v, out=None):
        """y = A_s v with the operator the attached V-cycle smooths this level with (gls_mg_smoother_apply)."""
        out = self.zeros() if out is None else out
        check(self.L.gls_mg_smoother_apply(self.h, _ptr(v), _ptr(out)), "gls_mg_smoother_apply")
        return out

    def apply_preconditioner(self, v, out=None):
        out = self.zeros() if out is None else out
        check(self.L.gls_apply_preconditioner(self.h, _ptr(v), _ptr(out)), "gls_apply_preconditioner")
        return out

    def kelly_estimate(self, sol, variable=0, out=None):
        """Kelly error indicator per cell (gls_kelly_estimate): variable 0 velocity, 1 pressure."""
        import torch
        out = torch.empty(self.n_cells, dtype=torch.float64, device=sol.device) if out is None else out
        check(self.L.gls_kelly_estimate(self.h, _ptr(sol), int(variable), _ptr(out)), "gls_kelly_estimate")
        return out

    def kelly_estimate_faces(self, sol, variable, faces, out=None):
        """Kelly indicator on a mesh with hanging faces (gls_kelly_estimate_faces); faces from
        Octree.faces()."""
        import torch
        fa, fb, fd, ra, rb = faces
        out = torch.empty(self.n_cells, dtype=torch.float64, device=sol.device) if out is None else out
        self.L.gls_kelly_estimate_faces.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int64] + [C.c_void_p] * 6
        check(self.L.gls_kelly_estimate_faces(self.h, _ptr(sol), int(variable), len(fa), fa.ctypes.data, fb.ctypes.data,
                                              fd.ctypes.data, ra.ctypes.data, rb.ctypes.data, _ptr(out)),
              "gls_kelly_estimate_faces")
        return out

    def kelly_estimate_mapped(self, sol, variable, faces, out=None):
        """Kelly indicator on a mapped mesh (gls_kelly_estimate_mapped); faces from
        FESpaceHandle.kelly_faces(n_q + 1)."""
        import torch
        out = torch.empty(self.n_cells, dtype=torch.float64, device=sol.device) if out is None else out
        f = {k: np.ascontiguousarray(v) for k, v in faces.items() if isinstance(v, np.ndarray)}
        p32 = lambda a: a.ctypes.data_as(C.POINTER(C.c_int32))  # noqa: E731
        check(self.L.gls_kelly_estimate_mapped(self.h, _ptr(sol), int(variable), len(f["ca"]), int(faces["nqf"]),
                                               p32(f["ca"]), p32(f["cb"]), _dp(f["xi"]), _dp(f["g"]), _dp(f["jxw"]),
                                               _dp(f["diam"]), _ptr(out)), "gls_kelly_estimate_mapped")
        return out

    def mg_transfer(self, level, direction, v, out):
        """Restrict (direction 0: level -> level+1) or prolongate (1: level+1 -> level) a device vector."""
        check(self.L.gls_mg_transfer(self.h, int(level), int(direction), _ptr(v), _ptr(out)), "gls_mg_transfer")
        return out

    def set_lattice(self, n1d, local_to_global):
        """Declare the (rank-local) nodes as a box of the global n1d^3 hyper_cube node lattice."""
        l2g = np.ascontiguousarray(local_to_global, dtype=np.int64)
        check(self.L.gls_set_lattice(self.h, int(n1d), l2g.ctypes.data_as(C.POINTER(C.c_int64))), "gls_set_lattice")

    def detach_multigrid(self):
        check(self.L.gls_mg_detach(self.h), "gls_mg_detach")
        self._mg_levels = None

    def attach_ilu(self, athresh=1e-8, rthresh=1.0, fill=0, block_dofs=0, ordering="cm"):
        """Assembled ILU(fill) preconditioner (the reference's ILU-preconditioned GMRES, setup_ILU); the
        Jacobian is probed from the device operator; ordering "cm" (the reference's Cuthill-McKee) or
        "multicolor"; block_dofs > 0: block-Jacobi subdomains of that size (gls_ilu_set_options).
        Returns (nnz of the ILU pattern, n_probes)."""
        self.L.gls_ilu_set_options.argtypes = [C.c_void_p, C.c_int, C.c_int64]
        check(self.L.gls_ilu_set_options(self.h, {"cm": 0, "multicolor": 1}[ordering], int(block_dofs)),
              "gls_ilu_set_options")
        self.L.gls_ilu_attach.argtypes = [C.c_void_p, C.c_int, C.c_double, C.c_double]
        check(self.L.gls_ilu_attach(self.h, int(fill), float(athresh), float(rthresh)), "gls_ilu_attach")
        nnz, npr = C.c_int64(), C.c_int()
        self.L.gls_ilu_info.argtypes = [C.c_void_p, C.POINTER(C.c_int64), C.POINTER(C.c_int)]
        check(self.L.gls_ilu_info(self.h, C.byref(nnz), C.byref(npr)), "gls_ilu_info")
        return nnz.value, npr.value

    def ilu_factors(self):
        """(perm, scipy CSR of the factored ILU) in the factorization numbering: perm[dof] = its row;
        strictly lower part = L (unit diagonal), upper part with the diagonal = U."""
        import scipy.sparse as sp
        nnz, _ = C.c_int64(), C.c_int()
        self.L.gls_ilu_info.argtypes = [C.c_void_p, C.POINTER(C.c_int64), C.POINTER(C.c_int)]
        check(self.L.gls_ilu_info(self.h, C.byref(nnz), C.byref(_)), "gls_ilu_info")
        perm = np.zeros(self.n_dofs, dtype=np.int32)
        rowp = np.zeros(self.n_dofs + 1, dtype=np.int32)
        col = np.zeros(nnz.value, dtype=np.int32)
        val = np.zeros(nnz.value)
        self.L.gls_ilu_factors.argtypes = [C.c_void_p] * 5
        check(self.L.gls_ilu_factors(self.h, perm.ctypes.data, rowp.ctypes.data, col.ctypes.data, val.ctypes.data),
              "gls_ilu_factors")
        return perm, sp.csr_matrix((val, col, rowp), shape=(self.n_dofs, self.n_dofs))

    def ilu_matrix(self):
        """The probed operator matrix (scipy CSR) behind the attached ILU, before perturbation/factoring."""
        import scipy.sparse as sp
        nnz, _ = C.c_int64(), C.c_int()
        self.L.gls_ilu_info.argtypes = [C.c_void_p, C.POINTER(C.c_int64), C.POINTER(C.c_int)]
        check(self.L.gls_ilu_info(self.h, C.byref(nnz), C.byref(_)), "gls_ilu_info")
        rowp = np.zeros(self.n_dofs + 1, dtype=np.int32)
        col = np.zeros(nnz.value, dtype=np.int32)
        val = np.zeros(nnz.value)
        self.L.gls_ilu_matrix.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
        check(self.L.gls_ilu_matrix(self.h, rowp.ctypes.data, col.ctypes.data, val.ctypes.data), "gls_ilu_matrix")
        return sp.csr_matrix((val, col, rowp), shape=(self.n_dofs, self.n_dofs))

    def detach_ilu(self):
        self.L.gls_ilu_detach.argtypes = [C.c_void_p]
        check(self.L.gls_ilu_detach(self.h), "gls_ilu_detach")

    # profiling
    def timing(self, enable=True):
        check(self.L.gls_timing_enable(self.h, 1 if enable else 0), "gls_timing_enable")
        check(self.L.gls_timing_reset(self.h), "gls_timing_reset")

    def timing_get(self, which):
        ms, n = C.c_double(), C.c_int64()
        check(self.L.gls_timing_get(self.h, which, C.byref(ms), C.byref(n)), "gls_timing_get")
        return ms.value, n.value


# ---------------------------------------------------------------------------------------------
# unstructured / curved meshes (host side, gls_umesh_* / gls_fe_space_*)
# ---------------------------------------------------------------------------------------------
MANIFOLD_TYPES = {"flat": 0, "spherical": 1, "cylindrical": 2}


class UMesh:
    """Owner of a gls_umesh: GridGenerator grids (hyper_cube, hyper_rectangle,
    subdivided_hyper_rectangle, hyper_shell, cylinder, cylinder_shell) or a gmsh file, manifolds,
    global refinement. fe_space() discretizes it (numpy arrays, see gls_fe_space)."""

    def __init__(self, dim, grid_type=None, grid_arguments="", gmsh=None):
        self.L = load()
        self.dim = dim
        h = C.c_void_p()
        if gmsh is not None:
            check(self.L.gls_umesh_read_gmsh(dim, str(gmsh).encode(), C.byref(h)), "gls_umesh_read_gmsh")
        else:
            check(self.L.gls_umesh_generate(dim, grid_type.encode(), grid_arguments.encode(), C.byref(h)),
                  "gls_umesh_generate")
        self.h = h

    def __del__(self):
        try:
            if getattr(self, "h", None):
                self.L.gls_umesh_destroy(self.h)
                self.h = None
        except Exception:
            pass

    def set_manifold(self, manifold_id, kind, center=(0.0, 0.0, 0.0), axis=(0.0, 0.0, 1.0)):
        c = np.ascontiguousarray(list(center) + [0.0] * (3 - len(center)), dtype=np.float64)
        a = np.ascontiguousarray(list(axis) + [0.0] * (3 - len(axis)), dtype=np.float64)
        check(self.L.gls_umesh_set_manifold(self.h, int(manifold_id), MANIFOLD_TYPES[kind], _dp(c), _dp(a)),
              "gls_umesh_set_manifold")

    def boundary_manifold(self, boundary_id, manifold_id):
        check(self.L.gls_umesh_boundary_manifold(self.h, int(boundary_id), int(manifold_id)),
              "gls_umesh_boundary_manifold")

    def refine_global(self, times=1):
        check(self.L.gls_umesh_refine_global(self.h, int(times)), "gls_umesh_refine_global")

    def info(self):
        nc, nv, vol = C.c_int64(), C.c_int64(), C.c_double()
        check(self.L.gls_umesh_info(self.h, C.byref(nc), C.byref(nv), C.byref(vol)), "gls_umesh_info")
        return nc.value, nv.value, vol.value

    def fe_space(self, k, kp=None, qmapping_all=False, periodic=()):
        """FE_Q(k)^dim x FE_Q(kp) on this mesh -> dict of numpy arrays (gls_umesh_fe_space)."""
        return self.fe_space_handle(k, kp, qmapping_all, periodic).data

    def fe_space_handle(self, k, kp=None, qmapping_all=False, periodic=()):
        """The same as a live FESpaceHandle (transfers, Kelly face pieces)."""
        kp = k if kp is None else kp
        per = np.ascontiguousarray(np.array(periodic, dtype=np.int32).reshape(-1))
        pm = C.POINTER(FESpace)()
        check(self.L.gls_umesh_fe_space(self.h, int(k), int(kp), 1 if qmapping_all else 0, len(per) // 3,
                                        per.ctypes.data_as(C.POINTER(C.c_int32)), C.byref(pm)), "gls_umesh_fe_space")
        return FESpaceHandle(self.L, pm)

    def set_periodic(self, periodic):
        """Periodic pairs (id a, id b, direction) of the triangulation (gls_umesh_set_periodic): the mesh
        smoothing and the 2:1 balance see across them."""
        per = np.ascontiguousarray(np.array(periodic, dtype=np.int32).reshape(-1))
        check(self.L.gls_umesh_set_periodic(self.h, len(per) // 3, per.ctypes.data_as(C.POINTER(C.c_int32))),
              "gls_umesh_set_periodic")

    def coarsen_to(self, level):
        """A copy with every active cell finer than `level` replaced by its ancestor (gls_umesh_coarsen_to):
        a level mesh of the multigrid on the refinement hierarchy."""
        out = UMesh.__new__(UMesh)
        out.L, out.dim = self.L, self.dim
        out.h = C.c_void_p()
        check(self.L.gls_umesh_coarsen_to(self.h, int(level), C.byref(out.h)), "gls_umesh_coarsen_to")
        return out

    def prepare(self, refine, coarsen):
        """prepare_coarsening_and_refinement with the reference's smoothing (gls_umesh_prepare);
        returns the smoothed (refine, coarsen) flags over the active cells."""
        r = np.ascontiguousarray(refine, dtype=np.int32).copy()
        c = np.ascontiguousarray(coarsen, dtype=np.int32).copy()
        check(self.L.gls_umesh_prepare(self.h, r.ctypes.data_as(C.POINTER(C.c_int32)),
                                       c.ctypes.data_as(C.POINTER(C.c_int32))), "gls_umesh_prepare")
        return r, c

    def adapt(self, refine, coarsen=None):
        """execute_coarsening_and_refinement (gls_umesh_adapt) with per-active-cell flags."""
        r = np.ascontiguousarray(refine, dtype=np.int32)
        c = np.ascontiguousarray(np.zeros_like(r) if coarsen is None else coarsen, dtype=np.int32)
        check(self.L.gls_umesh_adapt(self.h, r.ctypes.data_as(C.POINTER(C.c_int32)),
                                     c.ctypes.data_as(C.POINTER(C.c_int32))), "gls_umesh_adapt")


class FESpaceHandle:
    """A live gls_fe_space: .data (numpy dict), transfer_from (SolutionTransfer from an earlier space
    of the same mesh), kelly_faces (face pieces with MappingQ geometry)."""

    def __init__(self, L, ptr):
        self.L, self.ptr = L, ptr
        self.data = _fe_space_dict(ptr.contents)

    def __del__(self):
        try:
            if getattr(self, "ptr", None):
                self.L.gls_fe_space_destroy(self.ptr)
                self.ptr = None
        except Exception:
            pass

    def mg_transfer_from(self, coarse):
        """Prolongation CSR (off, col, w) from the space `coarse` of a coarser level of the same hierarchy and
        the state injection (gls_fe_space_mg_transfer)."""
        nnz = C.c_int64()
        check(self.L.gls_fe_space_mg_transfer(self.ptr, coarse.ptr, C.byref(nnz), None, None, None, None),
              "gls_fe_space_mg_transfer")
        d, c = self.data, coarse.data
        nf = d["dim"] * d["n_vnodes"] + d["n_pnodes"]
        nc = c["dim"] * c["n_vnodes"] + c["n_pnodes"]
        off = np.zeros(nf + 1, np.int64)
        col = np.zeros(max(nnz.value, 1), np.int32)
        w = np.zeros(max(nnz.value, 1))
        inj = np.zeros(nc, np.int64)
        check(self.L.gls_fe_space_mg_transfer(self.ptr, coarse.ptr, C.byref(nnz), off.ctypes.data, col.ctypes.data,
                                              w.ctypes.data, inj.ctypes.data), "gls_fe_space_mg_transfer")
        return off, col[:nnz.value], w[:nnz.value], inj

    def transfer_from(self, old, vec):
        vec = np.ascontiguousarray(vec, dtype=np.float64)
        out = np.zeros(self.data["dim"] * self.data["n_vnodes"] + self.data["n_pnodes"])
        check(self.L.gls_fe_space_transfer(old.ptr, self.ptr, _dp(vec), _dp(out)), "gls_fe_space_transfer")
        return out

    def boundary_normals(self, boundary_id):
        out = np.zeros((self.data["n_vnodes"], self.data["dim"]))
        check(self.L.gls_fe_space_boundary_normals(self.ptr, int(boundary_id), _dp(out)), "gls_fe_space_boundary_normals")
        return out

    def boundary_normal_sets(self, boundary_id):
        """(rank per node, grouped unit normals [n_vnodes][3][dim]) of a slip boundary's edges / corners"""
        nv, dim = self.data["n_vnodes"], self.data["dim"]
        cnt, out = np.zeros(nv, np.int32), np.zeros((nv, 3, dim))
        check(self.L.gls_fe_space_boundary_normal_sets(self.ptr, int(boundary_id), cnt.ctypes.data_as(C.POINTER(C.c_int32)),
                                                       _dp(out)), "gls_fe_space_boundary_normal_sets")
        return cnt, out

    def kelly_faces(self, nq):
        n = C.c_int64()
        z32 = C.POINTER(C.c_int32)()
        zd = C.POINTER(C.c_double)()
        check(self.L.gls_fe_space_kelly_faces(self.ptr, int(nq), C.byref(n), z32, z32, zd, zd, zd, zd),
              "gls_fe_space_kelly_faces")
        dim, ne = self.data["dim"], int(n.value)
        nqf = nq ** (dim - 1)
        ca, cb = np.zeros(ne, np.int32), np.zeros(ne, np.int32)
        xi, g = np.zeros((ne, nqf, 2, dim)), np.zeros((ne, nqf, 2, dim))
        jxw, diam = np.zeros((ne, nqf)), np.zeros(self.data["n_cells"])
        p32 = lambda a: a.ctypes.data_as(C.POINTER(C.c_int32))  # noqa: E731
        check(self.L.gls_fe_space_kelly_faces(self.ptr, int(nq), C.byref(n), p32(ca), p32(cb), _dp(xi), _dp(g),
                                              _dp(jxw), _dp(diam)), "gls_fe_space_kelly_faces")
        return dict(ca=ca, cb=cb, xi=xi, g=g, jxw=jxw, diam=diam, nqf=nqf)


def _fe_space_dict(m):
    dim, k, kp = m.dim, m.k, m.kp
    nc, nv, npn = int(m.n_cells), int(m.n_vnodes), int(m.n_pnodes)
    nl, npl = (k + 1) ** dim, (kp + 1) ** dim

    def take(ptr, count, dt, shape):
        return np.ctypeslib.as_array(ptr, shape=(int(count),)).astype(dt, copy=True).reshape(shape)

    return dict(dim=dim, k=k, kp=kp, n_cells=nc, n_vnodes=nv, n_pnodes=npn,
                cell_vnodes=take(m.cell_vnodes, nc * nl, np.int32, (nc, nl)),
                cell_pnodes=take(m.cell_pnodes, nc * npl, np.int32, (nc, npl)),
                vnode_x=take(m.vnode_x, nv * dim, np.float64, (nv, dim)),
                pnode_x=take(m.pnode_x, npn * dim, np.float64, (npn, dim)),
                vnode_bid=take(m.vnode_bid, nv, np.uint32, (nv,)),
                pnode_bid=take(m.pnode_bid, npn, np.uint32, (npn,)),
                cell_support=take(m.cell_support, nc * nl * dim, np.float64, (nc, nl, dim)),
                cell_mapping=take(m.cell_mapping, nc, np.int32, (nc,)),
                cell_measure=take(m.cell_measure, nc, np.float64, (nc,)), volume=float(m.volume),
                cell_level=take(m.cell_level, nc, np.int32, (nc,)),
                vhang=_hang_lines(m.n_vhang, m.vhang_node, m.vhang_off, m.vhang_master, m.vhang_w),
                phang=_hang_lines(m.n_phang, m.phang_node, m.phang_off, m.phang_master, m.phang_w))


def _hang_lines(n, node, off, master, w):
    """hanging lines as {node: [(master, weight), ...]}"""
    n = int(n)
    if n == 0:
        return {}
    node = np.ctypeslib.as_array(node, shape=(n,)).copy()
    off = np.ctypeslib.as_array(off, shape=(n + 1,)).copy()
    nm = int(off[-1])
    master = np.ctypeslib.as_array(master, shape=(nm,)).copy()
    w = np.ctypeslib.as_array(w, shape=(nm,)).copy()
    return {int(node[i]): [(int(master[j]), float(w[j])) for j in range(off[i], off[i + 1])] for i in range(n)}


def iluk_pattern(A, fill):
    """Host-only ILU(fill) level-of-fill pattern of the square CSR graph A (scipy sparse): returns
    (rowp, col, level) of the pattern, diagonal included, rows sorted (gls_iluk_pattern)."""
    L = load()
    A = A.tocsr()
    A.sort_indices()
    n = A.shape[0]
    rowp = np.ascontiguousarray(A.indptr, dtype=np.int32)
    col = np.ascontiguousarray(A.indices, dtype=np.int32)
    nnz = C.c_int64()
    L.gls_iluk_pattern.argtypes = [C.c_int64, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p,
                                   C.c_int64, C.POINTER(C.c_int64)]
    check(L.gls_iluk_pattern(n, rowp.ctypes.data, col.ctypes.data, int(fill), None, None, None, 0, C.byref(nnz)),
          "gls_iluk_pattern")
    orow = np.zeros(n + 1, dtype=np.int32)
    ocol = np.zeros(nnz.value, dtype=np.int32)
    olev = np.zeros(nnz.value, dtype=np.int32)
    check(L.gls_iluk_pattern(n, rowp.ctypes.data, col.ctypes.data, int(fill), orow.ctypes.data, ocol.ctypes.data,
                             olev.ctypes.data, nnz.value, C.byref(nnz)), "gls_iluk_pattern")
    return orow, ocol, olev


def cuthill_mckee(adj_off, adj, dof_off, dofs):
    """Host-only DoF renumbering of gls_ilu_attach (deal.II Cuthill_McKee on a node graph): returns
    order[new index] = DoF (gls_cuthill_mckee)."""
    L = load()
    a = [np.ascontiguousarray(x, dtype=np.int64) for x in (adj_off, adj, dof_off, dofs)]
    order = np.zeros(len(a[3]), dtype=np.int64)
    L.gls_cuthill_mckee.argtypes = [C.c_int64] + [C.c_void_p] * 5
    check(L.gls_cuthill_mckee(len(a[0]) - 1, *(x.ctypes.data for x in a), order.ctypes.data), "gls_cuthill_mckee")
    return order
