"""softx_2020_200_amd — MI355X-native GLS (SUPG/PSPG) Navier–Stokes hot path.

Drop-in for Lethe's GLSNavierStokesSolver assembly + linear solve path
(LMNS3d/SOFTX_2020_200 source/solvers/gls_navier_stokes.cc). The compute runs in
hand-written HIP kernels for gfx950 (libgls_native.so, C-ABI in include/gls_native.h);
this package is the thin Python front-end over that ABI.
"""
from .native import (GLSContext, GLSError, Octree, SCHEMES, bdf_coefficients, hanging_dof_lines, hyper_cube,  # noqa: F401
                     load, newton_selftest, octree_mg_transfer, skip_newton_selftest, refine_fixed_number, refine_pd, refine_coarsen_pd, refined_cube, refined_interpolate,
                     sdirk_coefficients)
from .problem import CavityProblem, build_context  # noqa: F401

__all__ = ["GLSContext", "GLSError", "SCHEMES", "bdf_coefficients", "sdirk_coefficients", "hyper_cube", "load",
           "newton_selftest", "skip_newton_selftest", "CavityProblem", "build_context", "refined_cube", "hanging_dof_lines",
           "refine_fixed_number", "refine_pd", "refine_coarsen_pd", "refined_interpolate", "octree_mg_transfer"]
