/* gls_native.h — C-ABI of the MI355X-native GLS Navier–Stokes hot path.
 *
 * Drop-in boundary for Lethe's GLSNavierStokesSolver assembly + linear-solve path.
 * Every entry point below names the reference interface it replaces
 * (paths relative to the reference tree, LMNS3d/SOFTX_2020_200).
 *
 * Conventions
 *   - Plain C types only: pointers, sizes, doubles. No torch / HIP types in signatures
 *     (streams are passed as void*; NULL = the context's own stream).
 *   - Return 0 on success or a negative GLS_E* code; gls_last_error() gives the text
 *     (thread-local). No C++ exception ever crosses this boundary
 *     (the reference throws std::runtime_error, gls_navier_stokes.cc:825, :1158).
 *   - Vectors are FP64, global layout [velocity node-major, comps interleaved | pressure]:
 *       dof(vnode, c) = vnode*dim + c,  dof(pnode) = dim*n_vnodes + pnode.
 *   - Operator entry points take DEVICE pointers (hipMalloc / torch cuda tensors); calls are
 *     stream-ordered on the context stream. Host-pointer entry points say so.
 *   - One context per GPU; the multi-GPU context (gls_dist_*) wraps RCCL.
 */
#ifndef GLS_NATIVE_H
#define GLS_NATIVE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GLS_OK 0
#define GLS_EINVAL -1   /* bad argument / unsupported configuration */
#define GLS_EHIP -2     /* HIP runtime error */
#define GLS_ENOMEM -3   /* device allocation failed */
#define GLS_ENOCONV -4  /* linear solver did not converge (informational) */
#define GLS_EIO -5      /* file / parse error */
#define GLS_ECOMM -6    /* RCCL error */
#define GLS_ENOTFOUND -7 /* parameter entry absent (gls_prm_get; the caller applies the default) */

/* TimeSteppingMethod, same order as include/core/parameters.h:56-69 */
enum gls_scheme {
  GLS_STEADY = 0, GLS_BDF1, GLS_BDF2, GLS_BDF3, GLS_SDIRK2, GLS_SDIRK2_1, GLS_SDIRK2_2,
  GLS_SDIRK3, GLS_SDIRK3_1, GLS_SDIRK3_2, GLS_SDIRK3_3
};

const char *gls_last_error(void);
const char *gls_version(void);

/* ------------------------------------------------------------------------------------------
 * Mesh / DoF map description (host pointers, copied at gls_create).
 * Replaces NavierStokesBase ctor FESystem(FE_Q(k)^dim, FE_Q(kp)) + QGauss(k+1)
 * (source/solvers/navier_stokes_base.cc:62,70) and GLSNavierStokesSolver::setup_dofs
 * (source/solvers/gls_navier_stokes.cc:55-228): cell->DoF map, zero_constraints mask.
 * Cells are axis-aligned boxes (hyper_cube / subdivided meshes, MappingQ affine on them).
 * ------------------------------------------------------------------------------------------ */
typedef struct {
  int dim;                      /* 2 or 3 */
  int k;                        /* velocity degree (1..3) */
  int kp;                       /* pressure degree (1..k) */
  int nq1d;                     /* QGauss points per direction, 0 = k+1 (navier_stokes_base.cc:70, :93-94) */
  int n_cells;
  int n_vnodes, n_pnodes;
  const int32_t *cell_vnodes;   /* [n_cells*(k+1)^dim], lexicographic local node order (x fastest) */
  const int32_t *cell_pnodes;   /* [n_cells*(kp+1)^dim]; NULL when kp==k and pressure nodes == velocity nodes */
  const double *cell_x0;        /* [n_cells*dim] lower corner (used by the SRF source term); may be NULL */
  const double *cell_h;         /* [n_cells*dim] extents */
  const uint8_t *vnode_mask;    /* [n_vnodes] bit c set = velocity comp c is in zero_constraints; NULL = none */
  double viscosity;             /* physical properties/kinematic viscosity */
  int srf;                      /* velocity source = srf (parameters.h:511-515) */
  double omega[3];
  const double *force_q;        /* [n_cells*nq*dim] forcing at quadrature points; NULL = NoForce */
  /* General (curved / unstructured) cells: MappingQ(map_degree) of FEValues (gls_navier_stokes.cc:
   * 245-252). 0 = axis-aligned boxes given by cell_x0 / cell_h (the brick fast path). > 0: the
   * cells' mapping support points, lexicographic on the equidistant (map_degree+1)^dim lattice
   * (Q1 cells of a MappingQ(k, qmapping_all = false) mesh are passed as their exact Qk embedding).
   * Jacobians, JxW, the Hessian mapping correction and the quadrature points are derived per
   * quadrature point at gls_create; cell->measure() (h of tau) from the cell's corner vertices. */
  int map_degree;
  const double *cell_support;   /* [n_cells][(map_degree+1)^dim][dim] */
} gls_mesh_desc;

typedef struct gls_ctx gls_ctx;

/* setup_dofs equivalent: uploads the DoF map, geometry, tabulated 1D bases. */
int gls_create(const gls_mesh_desc *desc, gls_ctx **out);
int gls_destroy(gls_ctx *ctx);
int gls_set_stream(gls_ctx *ctx, void *hip_stream);
int gls_n_dofs(const gls_ctx *ctx, int64_t *n_dofs);
/* Physical quadrature points QGauss(nq1d) of every cell (HOST array [n_cells][nq][dim]): where the
 * caller evaluates forcing (gls_set_force) and analytical functions; the mapped points for
 * general cells. */
int gls_quadrature_points(const gls_ctx *ctx, double *xq);
/* 1 when the context runs the sum-factorized brick kernels (3D Qk-Qk on Morton 2x2x2 bricks),
 * 0 for the general per-cell kernels. GLS_DISABLE_BRICK=1 in the environment forces 0. */
int gls_uses_brick_kernels(const gls_ctx *ctx);
/* Rewrite the forcing at quadrature points (host pointer, [n_cells*nq*dim]) or clear it (NULL). */
int gls_set_force(gls_ctx *ctx, const double *force_q);
int gls_set_viscosity(gls_ctx *ctx, double viscosity);

/* Time-stepping state for the next assembly (replaces the top of assembleGLS,
 * gls_navier_stokes.cc:295-329: time_steps_vector -> bdf_coefficients / sdirk_coefficients). */
int gls_set_time(gls_ctx *ctx, int scheme, const double time_steps[4]);

/* Evaluation point and history (DEVICE pointers, borrowed until the next call):
 * evaluation_point, solution_m1..m3 of PhysicsSolver (include/core/physics_solver.h:107-111).
 * u1..u3 may be NULL when the scheme does not read them. The state is captured here: the
 * Jacobian diagonal and the J.v linearization (per quadrature point) are cached until the next
 * gls_set_state / gls_set_time / gls_set_viscosity / gls_set_force, so changing the vectors'
 * contents in place requires calling gls_set_state again. */
int gls_set_state(gls_ctx *ctx, const double *u, const double *u1, const double *u2, const double *u3);

/* assemble_rhs (gls_navier_stokes.cc:1023-1128 -> assembleGLS<false,...>):
 * rhs = -R(u) with zero_constraints (constrained rows 0). DEVICE pointer, length n_dofs. */
int gls_residual(gls_ctx *ctx, double *rhs);

/* Matrix-free action of the reference's assembled Jacobian (assembleGLS<true,...>,
 * gls_navier_stokes.cc:519-625, distributed with zero_constraints :758-765):
 * Jv = P J P v + D_c v, D_c = sum over cells of |local(i,i)| on constrained DoFs (deal.II rule).
 * Replaces system_matrix.vmult inside Trilinos GMRES (gls_navier_stokes.cc:1276-1279). */
int gls_jacobian_apply(gls_ctx *ctx, const double *v, double *Jv);

/* The same operator evaluated in FP32 arithmetic from an FP32 copy of the linearization (3D
 * Qk-Qk brick path only; v, Jv are FP64 DEVICE vectors): the operator the mixed-precision
 * multigrid V-cycle smooths with (gls_mg_params.mixed_precision). Not a reference interface: a
 * preconditioner-internal operator, exposed for parity tests (relative error ~1e-6). */
int gls_jacobian_apply_f32(gls_ctx *ctx, const double *v, double *Jv);

/* Hanging-node constraints (DoF level), after the Dirichlet mask of gls_create:
 *   DoF dofs[i] = sum_{j in [offsets[i], offsets[i+1])} weights[j] * DoF masters[j]
 * (DoFTools::make_hanging_node_constraints, gls_navier_stokes.cc:84, 143; host arrays). Hanging
 * DoFs must not carry a Dirichlet mask bit (deal.II: interpolate_boundary_values skips DoFs that
 * are already constrained) and may not be masters; Dirichlet masters drop out of the operators
 * (closed zero_constraints). The operators then are those of the reference's condensed system
 * (AffineConstraints::distribute_local_to_global): residual and J.v rows of hanging DoFs are
 * condensed onto their masters, the hanging rows themselves are 0 / D_c v; gls_apply_dirichlet
 * also distributes the hanging values (nonzero_constraints.distribute). The diagonal returned by
 * gls_jacobian_diagonal stays the element-diagonal sum on unconstrained rows (a Jacobi scaling,
 * not the condensed diagonal). Single GPU, per-cell kernels (no bricks, no multigrid). */
int gls_set_hanging(gls_ctx *ctx, int64_t n_lines, const int64_t *dofs, const int64_t *offsets,
                    const int64_t *masters, const double *weights);

/* Adapted forests (after gls_set_hanging on 3D Q2-Q2 box cells): the number of complete sibling groups
 * of leaves (8 consecutive cells forming a 2x2x2 brick) whose J.v / diagonal run the sum-factorised pencil
 * kernel (cached linearization, element-vector output summed with the per-cell kernel's); 0 = per-cell
 * kernels only (GLS_OCT_BRICKS=0 in the environment forces it). */
int gls_forest_bricks(const gls_ctx *ctx);

/* Diagonal of that assembled Jacobian (DEVICE pointer). */
int gls_jacobian_diagonal(gls_ctx *ctx, double *diag);

/* assemble_matrix_and_rhs (gls_navier_stokes.cc:917-1000, assembleGLS<true>: the matrix and the rhs in
 * one pass over the cells): the residual into rhs (as gls_residual) and the Jacobian's diagonal (as
 * gls_jacobian_diagonal; diag may be NULL) at the current state, with the J.v linearization cached.
 * On the 3D Q2 brick path one fused launch computes all three; the values equal those of the separate
 * calls bitwise. DEVICE pointers. */
int gls_residual_and_diagonal(gls_ctx *ctx, double *rhs, double *diag);

/* Apply nonzero_constraints.distribute to a DEVICE vector: x[dof] = value for listed DoFs
 * (PhysicsSolver::apply_constraints, physics_solver.h:98-102). Host arrays, copied. */
int gls_set_dirichlet(gls_ctx *ctx, int64_t n, const int64_t *dofs, const double *values);
int gls_apply_dirichlet(gls_ctx *ctx, double *x);

/* ------------------------------------------------------------------------------------------
 * Linear solve: replaces solve_system_GMRES + setup_ILU (gls_navier_stokes.cc:1242-1289,
 * :1161-1176). Right-preconditioned restarted GMRES on the matrix-free operator with a
 * Jacobi (diagonal) preconditioner; tolerance = max(rel*||rhs||, abs) as the reference.
 * x and rhs are DEVICE pointers. Returns GLS_OK or GLS_ENOCONV (x holds the last iterate).
 * ------------------------------------------------------------------------------------------ */
#define GLS_LIN_GMRES 0     /* solve_system_GMRES (gls_navier_stokes.cc:1242-1289) */
#define GLS_LIN_BICGSTAB 1  /* solve_system_BiCGStab (gls_navier_stokes.cc:1293-1340): right-preconditioned
                               BiCGStab, same preconditioner and tolerance rule; an iteration = one
                               BiCGStab step (two operator applications), as AztecOO counts them */
#define GLS_ORTHO_GRAM 0    /* GMRES: Gram-corrected single-pass classical Gram-Schmidt (default) */
#define GLS_ORTHO_CGS2 1    /* GMRES: classical Gram-Schmidt + DGKS re-orthogonalisation pass */
typedef struct {
  int max_iterations;     /* linear solver/max iters */
  int restart;            /* GMRES restart (deal.II default 30) */
  double relative_residual, minimum_residual;
  int iterations;         /* out */
  double final_residual;  /* out */
  int method;             /* GLS_LIN_GMRES (0, default) | GLS_LIN_BICGSTAB ('linear solver/method',
                             parameters.cc:519-532; 'amg' is GMRES with the caller's preconditioner) */
  int orthogonalization;  /* GMRES only: GLS_ORTHO_GRAM (0) | GLS_ORTHO_CGS2; the environment variable
                             GLS_GMRES_CGS2=1 forces CGS2 for every call */
  int true_residual;      /* in: 1 = on convergence recompute ||b - A x|| into final_residual (one extra
                             operator application); 0 = the Krylov recurrence estimate (deal.II) */
} gls_linear_params;
int gls_solve_linear(gls_ctx *ctx, const double *rhs, double *x, gls_linear_params *prm);

/* Geometric multigrid preconditioner (matrix-free, monolithic), replacing the Jacobi default of
 * gls_solve_linear (the reference's ILU / ML-AMG setup, gls_navier_stokes.cc:1161-1240).
 * levels[0] = ctx; levels[l] = caller-created contexts of the same problem on the nested
 * hyper_cube with n/2^l cells per direction (same k, same boundary conditions and Dirichlet
 * lists). Each V-cycle: damped-Jacobi smoothing with the level's own matrix-free GLS Jacobian at
 * the injected state, exact Qk restriction/prolongation. 3D Q1-Q1 / Q2-Q2. The coarse levels are
 * switched to ctx's stream (and follow later gls_set_stream calls on ctx).
 * Multi-GPU: every level is a distributed context (gls_dist_attach on the partition of its own
 * hyper_cube; nested partitions: rank r's coarse cells are the parents of its fine cells) that
 * also declared its lattice embedding with gls_set_lattice. Restriction sums owned fine rows and
 * export-adds the coarse ghost rows; prolongation imports the coarse ghosts first. */
typedef struct {
  int n_levels;
  gls_ctx **levels;
  int pre_smooth, post_smooth, coarse_sweeps;  /* pre: 0 -> 2, < 0 -> none (x = 0, residual = rhs);
                                                  post: < 0 -> 2, 0 -> none; coarse: 0 -> 30 */
  double omega;                               /* damped-Jacobi weight of the smoother, 0 -> 0.6 */
  double coarse_omega;                        /* weight of the coarsest-level sweeps, 0 -> omega */
  int coarse_direct;                          /* coarsest level: 0 auto (exact solve when on one GPU
                                                 with <= 2048 DoFs), 1 direct solve (<= 40000 DoFs;
                                                 a gls_mg_attach_replica level <= 8192),
                                                 -1 Jacobi sweeps. The direct solve probes the coarsest
                                                 Jacobian and factors it by rocSOLVER LU with the
                                                 first pressure DoF pinned (the enclosed-flow gauge).
                                                 Up to 8192 DoFs FP64: unpivoted by default, the
                                                 inverse checked by max|A (A^-1 e) - e| and finiteness;
                                                 a zero pivot or a failed check refactors with partial
                                                 pivoting (GLS_MG_COARSE_SOLVER=lu: always pivoted).
                                                 Above: FP32 unpivoted (sgetrf_npvt by a library worker
                                                 thread on a side stream, overlapping the finer levels'
                                                 setup), applied by blocked triangular solves; checked
                                                 by |A x - 1| / |1|: < 1e-2 as it is, < 0.5 with one
                                                 refinement step against the FP64 matrix, else pivoted
                                                 FP32 LU + explicit inverse */
  int mixed_precision;                        /* 1: the V-cycle's smoothing / residual J.v run in FP32
                                                 arithmetic from an FP32 copy of the linearization
                                                 (brick path; vectors, transfers and the outer GMRES
                                                 operator stay FP64). 0: all FP64 (an FP32 copy of the
                                                 ILU smoothers' factors measured slower:
                                                 profiles/r06_ab_ilu_fp32_factors.txt) */
  const int *level_sweeps;                    /* optional (NULL: uniform): 2*n_levels ints, the
                                                 pre / post sweep counts of each level (the entries of
                                                 the coarsest level are ignored) */
  int smoother;                               /* 0: damped Jacobi (omega); 1: ILU(0) of each level's
                                                 probed Jacobian, undamped (the smoother Trilinos ML
                                                 uses under the reference's AMG, gls_navier_stokes.cc:
                                                 1208-1226); levels with hanging nodes only
                                                 (gls_mg_attach_transfers); 2: ILU(0) on the coarser
                                                 levels, damped Jacobi on the finest (its FP32 brick
                                                 J.v with mixed_precision) */
  int smoother_operator;                      /* 0: the levels' Newton Jacobian; 1: its Oseen (Picard)
                                                 linearization on the FP32 brick levels (no (grad u) v
                                                 terms, no SUPG tau (v . grad phi) R_s term): cheaper
                                                 smoothing J.v; the outer GMRES operator is the exact
                                                 Jacobian either way */
} gls_mg_params;
int gls_mg_attach(gls_ctx *ctx, const gls_mg_params *prm);
/* The same V-cycle on a general level hierarchy with the caller's grid transfers: levels of an adaptive
 * (octree) mesh with hanging-node constraints (gls_set_hanging before attaching), e.g. the global
 * coarsening gls_octree_coarsen_to / gls_octree_mg_transfer builds. For l = 0 .. n_levels-2:
 * p_off[l] (n_dofs(l)+1), p_col[l], p_w[l] = the prolongation from level l+1 to level l as CSR (rows of
 * constrained fine DoFs may be empty), inject[l] (n_dofs(l+1)) = the level-l DoF whose value the
 * level-(l+1) state takes (hanging values are then distributed from their lines). Restriction = P^T;
 * the V-cycle zeroes constrained rows (Dirichlet and hanging) after each transfer. Smoothing: damped
 * Jacobi with each level's own operator (per-cell kernels on hanging levels, FP64). One GPU. Host arrays
 * (copied). The levels may differ in element degree (h-p hierarchies: a Q2-Q1 level above Q1-Q1 ones, the
 * p-level pairs of gls_fe_space_mg_transfer), not in dimension. */
int gls_mg_attach_transfers(gls_ctx *ctx, const gls_mg_params *prm, const int64_t *const *p_off,
                            const int32_t *const *p_col, const double *const *p_w, const int64_t *const *inject);
/* The refinement-hierarchy V-cycle ACROSS RANKS on general meshes (the reference's AMG is global,
 * gls_navier_stokes.cc:1180-1240): ctx is the rank-local fine context (distributed with
 * gls_dist_attach_dofs[_rccl]); every coarser level runs as a REPLICA on every rank: `replica` is a
 * single-rank context of the level-1 mesh (the whole of it) with its own hierarchy attached (e.g.
 * gls_mg_attach_transfers), so the N-rank V-cycle is the one-rank V-cycle up to the fine level's smoother.
 * p_off (n_local + 1) / p_col / p_w: the prolongation from level 1 (replica DoFs) onto the rank's local fine
 * DoFs, owned and ghost rows; inject (replica n_dofs): the local fine DoF whose value the replica's state
 * takes, on the one rank that owns it (-1 elsewhere). The restriction sums P^T over each rank's owned rows
 * and all-reduces in the replica numbering. prm: pre / post smooth, omega, smoother (0 damped Jacobi, 1
 * ILU(0) per rank = Ifpack additive Schwarz, overlap 0); coarse_direct > 0 with a replica WITHOUT a hierarchy
 * of its own (two-level case): the replica level is solved exactly (probed, LU-inverted, <= 8192 DoFs) on
 * every rank; levels / other coarse entries are not used. Host arrays. */
int gls_mg_attach_replica(gls_ctx *ctx, const gls_mg_params *prm, gls_ctx *replica, const int64_t *p_off,
                          const int32_t *p_col, const double *p_w, const int64_t *inject);
/* z = M^-1 v with the preconditioner gls_solve_linear uses at the current state (the V-cycle when
 * attached, else Jacobi): the reference's preconditioner vmult (DEVICE pointers, no aliasing). */
int gls_apply_preconditioner(gls_ctx *ctx, const double *v, double *z);
/* y = A_s v: the operator the attached V-cycle smooths this level with (the Jacobian, in FP32 with
 * gls_mg_params.mixed_precision, its Oseen part with smoother_operator = 1); DEVICE pointers. */
int gls_mg_smoother_apply(gls_ctx *ctx, const double *v, double *y);
/* Multigrid grid transfer between levels `level` and `level`+1 of the attached hierarchy (DEVICE
 * pointers): direction 0 restricts a level-`level` vector into level `level`+1 (transpose of the
 * Qk interpolation, the reference's MGTransfer restrict_and_add into a zeroed vector), direction 1
 * prolongates a level-`level`+1 vector onto level `level` (exact Qk interpolation). Constrained
 * rows are not touched here; the V-cycle zeroes them. */
int gls_mg_transfer(gls_ctx *ctx, int level, int direction, const double *in, double *out);
/* Lattice embedding of a (rank-local) mesh: its velocity nodes are a subset of the global n1d^3
 * Qk node lattice of hyper_cube in canonical numbering (global id = x + n1d*(y + n1d*z)), local
 * node i being global node local_to_global[i] (host array, n_vnodes entries). The local nodes
 * must fill an axis-aligned box (Morton partitions of a 2^m-cube over 2^j ranks do). */
int gls_set_lattice(gls_ctx *ctx, int n1d, const int64_t *local_to_global);
int gls_mg_detach(gls_ctx *ctx);
/* Multi-GPU: the V-cycle below the coarsest DISTRIBUTED level is the single-GPU one, computed
 * redundantly on every rank. replica = a single-rank context of that level's WHOLE mesh (same problem
 * and boundary data) with its own gls_mg_attach hierarchy below it (e.g. the exact LU level of the
 * one-GPU cycle); local_to_replica[i] = the replica row of the coarsest level's local row i (n_local =
 * its n_dofs). The coarsest level's correction becomes: all-reduce its owned right-hand-side rows into
 * the replica numbering, apply the replica's preconditioner, take back the local rows. Its state, time
 * data and viscosity follow the hierarchy's (gathered at every Jacobian state). With the replica the
 * N-rank cycle performs the operations of the 1-rank cycle (bench.py --gpus N). */
int gls_mg_set_coarse_replica(gls_ctx *ctx, gls_ctx *replica, int64_t n_local, const int64_t *local_to_replica);
/* Assembled ILU(fill) preconditioner for GMRES (replaces setup_ILU, gls_navier_stokes.cc:1161-1176:
 * Trilinos PreconditionILU(ilu_fill, ilu_atol, ilu_rtol, overlap 0) = Ifpack ILU(k), the reference's
 * 'linear solver/method = gmres' with 'ilu preconditioner fill / absolute / relative tolerance',
 * parameters.cc:546-560). The Jacobian is probed from the device operator into CSR with
 * distance-2-colored unit vectors once per Jacobian state; its graph is the reference's system
 * sparsity (constrained rows / columns hold the diagonal only, lines couple their masters). DoFs are
 * renumbered like DoFRenumbering::Cuthill_McKee; the ILU(fill) level-of-fill pattern (Ifpack_IlukGraph:
 * level(i,j) = min_k level(i,k) + level(k,j) + 1 <= fill) is inserted with explicit zeros, the
 * diagonal perturbed like Ifpack (a_ii <- rthresh a_ii + sign(a_ii) athresh) and factored by rocSPARSE
 * (multicolor order: by the color-by-color device factorization, same IKJ update order).
 * fill outside 0..GLS_ILU_MAX_FILL is rejected (GLS_EINVAL). Single rank, no multigrid. */
#define GLS_ILU_MAX_FILL 10
int gls_ilu_attach(gls_ctx *ctx, int fill, double athresh, double rthresh);
int gls_ilu_detach(gls_ctx *ctx);
/* Options of the next gls_ilu_attach.
 * ordering: GLS_ILU_ORDER_CM (default) = DoFRenumbering::Cuthill_McKee as the reference factors;
 *   GLS_ILU_ORDER_MULTICOLOR = DoFs grouped by a distance-1 coloring of the matrix's node graph
 *   (Cuthill-McKee inside a color): a different ILU (weaker, more GMRES iterations) whose triangular
 *   solves have a dependency chain of ~colors x DoFs per node instead of ~the matrix bandwidth.
 * block_dofs: block-Jacobi subdomains: the cells (in their space-filling order) are cut into
 *   ceil(n_dofs / block_dofs) contiguous ranges, couplings between the ranges are dropped and every
 *   block is factored on its own -- Ifpack's additive Schwarz with overlap 0, which is what the
 *   reference's setup_ILU gives with one block per MPI rank. 0 (default): one block. */
#define GLS_ILU_ORDER_CM 0
#define GLS_ILU_ORDER_MULTICOLOR 1
int gls_ilu_set_options(gls_ctx *ctx, int ordering, int64_t block_dofs);
int gls_ilu_info(const gls_ctx *ctx, int64_t *nnz, int *n_probes);
int gls_ilu_matrix(gls_ctx *ctx, int32_t *rowp, int32_t *col, double *val); /* probed CSR (tests) */
/* factored values in the factorization numbering (perm[dof] = row), for tests */
int gls_ilu_factors(gls_ctx *ctx, int32_t *perm, int32_t *rowp, int32_t *col, double *val);
/* Host only (no device): the ILU(fill) level-of-fill pattern of an n x n CSR graph (diagonal always
 * included, rows sorted), with each entry's level. Call with out_rowp / out_col / out_level all NULL
 * to get out_nnz; capacity = length of out_col / out_level. */
int gls_iluk_pattern(int64_t n, const int32_t *rowp, const int32_t *col, int fill, int32_t *out_rowp,
                     int32_t *out_col, int32_t *out_level, int64_t capacity, int64_t *out_nnz);
/* Host only: the DoF renumbering gls_ilu_attach uses (deal.II DoFRenumbering::Cuthill_McKee,
 * gls_navier_stokes.cc:70) on a node graph: node x's row nodes adj[adj_off[x] .. adj_off[x+1]) (itself
 * included), its DoFs dofs[dof_off[x] .. dof_off[x+1]) (old order = position in dofs);
 * order[new index] = DoF. */
int gls_cuthill_mckee(int64_t n_nodes, const int64_t *adj_off, const int64_t *adj, const int64_t *dof_off,
                      const int64_t *dofs, int64_t *order);

/* ------------------------------------------------------------------------------------------
 * Nonlinear solve: NewtonNonLinearSolver::solve (include/core/newton_non_linear_solver.h:74-139)
 * on device vectors: present (in/out, DEVICE, length n_dofs). History from gls_set_state's u1..u3
 * slots is given here explicitly.
 * ------------------------------------------------------------------------------------------ */
/* TimerOutput sections of the Newton / GMRES path (the reference's TimerOutput::Scope names,
 * gls_navier_stokes.cc:921 assemble_system, :1028 assemble_rhs, :1165 setup_ILU, :1182 setup_AMG (here
 * the geometric multigrid's setup), :1274 solve_linear_system): while enabled, gls_newton_solve
 * accumulates each section's host wall time (context stream drained at the section boundaries) and
 * call count. gls_section_timing(ctx, on) also zeroes the accumulators. */
#define GLS_SEC_ASSEMBLE_SYSTEM 0
#define GLS_SEC_ASSEMBLE_RHS 1
#define GLS_SEC_SETUP_ILU 2
#define GLS_SEC_SETUP_GMG 3
#define GLS_SEC_SOLVE_LINEAR 4
#define GLS_N_SECTIONS 5
int gls_section_timing(gls_ctx *ctx, int enable);
int gls_section_get(const gls_ctx *ctx, int section, double *seconds, int *calls);

#define GLS_NEWTON 0
#define GLS_SKIP_NEWTON 1
typedef struct {
  double tolerance;       /* non-linear solver/tolerance */
  int max_iterations;     /* non-linear solver/max iterations */
  int verbosity;          /* 0 quiet, 1 verbose (prints the reference's Newton lines) */
  gls_linear_params lin;
  int newton_iterations;  /* out */
  int linear_iterations;  /* out: total */
  int residual_evaluations; /* out */
  double final_residual;  /* out */
  int solver;             /* non-linear solver/solver: GLS_NEWTON | GLS_SKIP_NEWTON (parameters.cc:385-440) */
  int skip_iterations;    /* non-linear solver/skip iterations (skip_newton only; >= 1) */
  int is_initial_step;    /* solve_non_linear_system(method, first_iteration, force_matrix_renewal) */
  int force_matrix_renewal; /*   flags (physics_solver.h:92-96, navier_stokes_base.cc:461-590) */
  int linear_failures;    /* out: linear solves that stopped at max iterations (the reference's
                             SolverControl throws NoConvergence there; this library continues) */
} gls_newton_params;
/* Freeze (1) / release (0) the Jacobian at the current state: the skip_newton matrix reuse
 * (skip_newton_non_linear_solver.h:66-70, 126-130). While frozen, gls_jacobian_apply,
 * gls_jacobian_diagonal, the J.v linearization and the multigrid levels stay at the snapshot of
 * the state vectors and time coefficients taken here; gls_set_state / gls_set_time move only the
 * residual. gls_newton_solve with solver = GLS_SKIP_NEWTON drives this itself. */
int gls_freeze_jacobian(gls_ctx *ctx, int freeze);
int gls_newton_solve(gls_ctx *ctx, double *present, const double *u1, const double *u2, const double *u3,
                     gls_newton_params *prm);

/* ------------------------------------------------------------------------------------------
 * Multi-GPU (one process per GPU). Replaces the MPI domain decomposition of
 * parallel::distributed::Triangulation + Trilinos ghosted vectors (navier_stokes_base.cc:55-60,
 * gls_navier_stokes.cc:186-202) and compress(add) (:774-776).
 *   gls_part_*      : partition plan of a Morton brick mesh (host): rank-local mesh with owned
 *                     nodes first, ghosts after; import/export lists per neighbour rank.
 *   gls_dist_attach : turns a context built on the rank-local mesh into a distributed one.
 *                     Ghost import (before residual / J.v / set_state) and export-add (after)
 *                     pack into caller-owned DEVICE buffers (4 doubles per node: u,v,w,p) and call
 *                     xchg(user, 0 = import: send send_buf segments to neighbours, receive into
 *                     recv_buf | 1 = export: send recv_buf segments, receive into send_buf);
 *                     dot products sum owned DoFs and call allreduce(user, dev_buf, n) (sum).
 *                     The caller implements both with RCCL (torch.distributed "nccl") over xGMI.
 *                     Calls are made on the context stream's order; callbacks must return 0.
 * ------------------------------------------------------------------------------------------ */
typedef struct gls_part gls_part;
int gls_part_create(int n_cells, int nodes_per_cell, const int32_t *cell_vnodes, int n_vnodes, int rank, int world,
                    gls_part **out);
int gls_part_sizes(const gls_part *p, int64_t *cell_begin, int64_t *cell_end, int64_t *n_owned_nodes,
                   int64_t *n_local_nodes, int *n_nbrs, int64_t *n_send, int64_t *n_recv);
int gls_part_get(const gls_part *p, int32_t *local_cell_vnodes, int64_t *local_to_global, int *nbr_ranks,
                 int64_t *send_offsets, int32_t *send_nodes, int64_t *recv_offsets, int32_t *recv_nodes);
int gls_part_destroy(gls_part *p);

typedef int (*gls_exchange_fn)(void *user, int phase);
typedef int (*gls_allreduce_fn)(void *user, double *dev_buf, int n);
/* red_buf: a DEVICE buffer of at least GLS_RED_BUF_MIN doubles. Every reduction the library makes
 * through the callback goes through it in pieces of at most that many values (GMRES dots: restart+1
 * <= 256, the multigrid replica's right-hand side in chunks of 256). */
#define GLS_RED_BUF_MIN 256
int gls_dist_attach(gls_ctx *ctx, int64_t n_owned_nodes, int n_nbrs, const int64_t *send_offsets,
                    const int32_t *send_nodes, const int64_t *recv_offsets, const int32_t *recv_nodes, double *send_buf,
                    double *recv_buf, double *red_buf, gls_exchange_fn xchg, gls_allreduce_fn allreduce, void *user);
/* refresh ghost entries of a DEVICE vector (e.g. the history vectors once per time step) */
int gls_dist_import(gls_ctx *ctx, double *x);
/* In-library RCCL transport (replaces the callbacks above; the reference's Trilinos ghosted vectors
 * and compress(add), gls_navier_stokes.cc:186-202, 774-776): rank 0 calls gls_rccl_unique_id and
 * broadcasts the GLS_RCCL_ID_BYTES bytes by any means; every rank calls gls_rccl_create (one
 * communicator per process, shared by all contexts, e.g. every multigrid level), then
 * gls_dist_attach_rccl per context with the gls_part_get lists. Ghost import / export-add are
 * grouped ncclSend / ncclRecv and the dot products ncclAllReduce, all on the context stream. */
#define GLS_RCCL_ID_BYTES 128
typedef struct gls_rccl gls_rccl;
int gls_rccl_unique_id(unsigned char *id_out);
int gls_rccl_create(const unsigned char *id, int rank, int world, gls_rccl **out);
int gls_rccl_destroy(gls_rccl *comm);
/* the communicator's rank and size as RCCL reports them (ncclCommUserRank / ncclCommCount) */
int gls_rccl_info(const gls_rccl *comm, int *rank, int *world);
int gls_dist_attach_rccl(gls_ctx *ctx, gls_rccl *comm, int64_t n_owned_nodes, int n_nbrs, const int *nbr_ranks,
                         const int64_t *send_offsets, const int32_t *send_nodes, const int64_t *recv_offsets,
                         const int32_t *recv_nodes);

/* General meshes across ranks (adaptive / unstructured forests; the p::d triangulation partition,
 * navier_stokes_base.cc:55-60, 682-733, ghosted vectors gls_navier_stokes.cc:186-202): any dim,
 * Qk-Qk' with separate pressure nodes, hanging-node / slip lines (DoF level, global numbering:
 * velocity node*dim + c, pressure dim*n_vnodes + node). Every rank holds the same global mesh
 * (replicated host data) and calls gls_gpart_create with its rank: contiguous equal-count ranges of
 * the given cell order per rank, node ownership by the lowest touching rank, rank-local nodes
 * owned first then ghosts (ascending (owner, id)); ghosts include the masters of the lines on local
 * cells. The rank's context is created on the local cells (gls_gpart_get) and attached with
 * gls_dist_attach_dofs (callbacks, one double per exchanged DoF) or gls_dist_attach_dofs_rccl;
 * gls_gpart_map_dofs maps global DoF ids (Dirichlet rows, line DoFs and masters) to local ones
 * (-1 where not local). Hanging lines (gls_set_hanging) are then given in local ids. */
typedef struct gls_gpart gls_gpart;
int gls_gpart_create(int dim, int k, int kp, int64_t n_cells, const int32_t *cell_vnodes, const int32_t *cell_pnodes,
                     int64_t n_vnodes, int64_t n_pnodes, int64_t n_lines, const int64_t *line_dofs,
                     const int64_t *line_offsets, const int64_t *line_masters, int rank, int world, gls_gpart **out);
int gls_gpart_sizes(const gls_gpart *p, int64_t *cell_begin, int64_t *cell_end, int64_t *n_vnodes, int64_t *n_pnodes,
                    int64_t *n_owned_vnodes, int64_t *n_owned_pnodes, int *n_nbrs, int64_t *n_send, int64_t *n_recv);
int gls_gpart_get(const gls_gpart *p, int32_t *local_cell_vnodes, int32_t *local_cell_pnodes, int64_t *vnode_l2g,
                  int64_t *pnode_l2g, int *nbr_ranks, int64_t *send_offsets, int32_t *send_dofs, int64_t *recv_offsets,
                  int32_t *recv_dofs);
int gls_gpart_map_dofs(const gls_gpart *p, int64_t n, const int64_t *global_dofs, int64_t *local_dofs);
int gls_gpart_destroy(gls_gpart *p);
/* The same plan from the rank's LOCAL PART only (distributed forest: no rank holds the global mesh;
 * the p::d triangulation's locally relevant cells, navier_stokes_base.cc:55-60): the owned cells
 * (cell_owner == rank, in the given order) plus the ghost layer -- every cell sharing a node with an
 * owned cell, and every cell touching a MASTER node of a hanging line whose DoF lies on an owned cell
 * (e.g. the far corner / edge midpoints of a coarse face) -- each with its owner; the lines whose DoF
 * lies on a provided cell. A node is owned by the lowest rank among ALL cells touching it, so each node
 * the rank needs must come with every cell touching it: with a thinner layer (p4est's one-cell ghost
 * layer alone) two ranks can disagree on an owner and on the exchange lists. A needed master node that
 * lies on no provided cell is rejected (GLS_EINVAL); a missing cell of a provided node cannot be seen
 * locally -- dist.local_part() builds the layer by this rule. Nodes are 64-bit keys unique over
 * the forest (no global numbering needed); DoF keys are key * (dim + 1) + c with c = dim for pressure
 * (line_dofs / line_masters and gls_gpart_map_dofs use DoF keys). cell_pkeys = NULL for equal order.
 * vnode_l2g / pnode_l2g of gls_gpart_get return the local nodes' keys; the exchange lists are those of
 * gls_gpart_create for the same partition (identical arrays when the keys are the global node ids).
 * A global numbering, if wanted, is one exclusive scan of the owned counts plus one exchange. */
int gls_dpart_create(int dim, int k, int kp, int64_t n_cells, const int32_t *cell_owner, const int64_t *cell_vkeys,
                     const int64_t *cell_pkeys, int64_t n_lines, const int64_t *line_dofs, const int64_t *line_offsets,
                     const int64_t *line_masters, int rank, int world, gls_gpart **out);
int gls_dist_attach_dofs(gls_ctx *ctx, int64_t n_owned_vnodes, int64_t n_owned_pnodes, int n_nbrs,
                         const int64_t *send_offsets, const int32_t *send_dofs, const int64_t *recv_offsets,
                         const int32_t *recv_dofs, double *send_buf, double *recv_buf, double *red_buf,
                         gls_exchange_fn xchg, gls_allreduce_fn allreduce, void *user);
int gls_dist_attach_dofs_rccl(gls_ctx *ctx, gls_rccl *comm, int64_t n_owned_vnodes, int64_t n_owned_pnodes,
                              int n_nbrs, const int *nbr_ranks, const int64_t *send_offsets, const int32_t *send_dofs,
                              const int64_t *recv_offsets, const int32_t *recv_dofs);

/* ------------------------------------------------------------------------------------------
 * Host-side building blocks (host pointers).
 * ------------------------------------------------------------------------------------------ */
/* bdf_coefficients (source/core/bdf.cc:45-75): alpha[order+1] */
int gls_bdf_coefficients(int order, const double *dt, int n_dt, double *alpha);
/* sdirk_coefficients (source/core/sdirk.cc:11-44): out[order*(order+1)] row-major */
int gls_sdirk_coefficients(int order, double dt, double *out);
/* Newton driver KAT: the reference's fake physics x0^2+x1=0, 2x1+3=0
 * (tests/core/non_linear_test_system_01.h:50-129) through the same Newton template. */
int gls_newton_selftest(double x_out[2]);
/* SkipNewton KAT (tests/core/skip_newton_non_linear_solver_01.cc): same fake physics through the
 * SkipNewton template (skip_newton_non_linear_solver.h:54-131), tol 1e-8, 10 iterations. */
int gls_skip_newton_selftest(int skip_iterations, double x_out[2]);

/* hyper_cube mesh + canonical DoF numbering (GridGenerator::hyper_cube + refine_global,
 * source/core/grids.cc:12-60). Periodic directions identify the high face with the low face.
 * Cells are emitted in Morton (p4est z-)order. Arrays are allocated by the caller with the
 * sizes from gls_mesh_hyper_cube_sizes. boundary ids: colorize ? 2d / 2d+1 : 0. */
int gls_mesh_hyper_cube_sizes(int dim, int n, int k, int kp, int periodic_mask,
                              int64_t *n_cells, int64_t *n_vnodes, int64_t *n_pnodes);
int gls_mesh_hyper_cube(int dim, int n, int k, int kp, double lo, double hi, int periodic_mask,
                        int32_t *cell_vnodes, int32_t *cell_pnodes, double *cell_x0, double *cell_h);

/* Locally refined hyper_cube (one extra level): hyper_cube(lo, hi) with n^dim cells, the cells
 * flagged in refine[n^dim] (lexicographic, x fastest; NULL = none) split into 2^dim children
 * (execute_coarsening_and_refinement on a p4est forest, navier_stokes_base.cc:592-780). Nodes are
 * numbered lexicographically on the fine node lattice; hanging nodes are constrained to the
 * unrefined neighbour's nodes: value(node) = sum_j w_j value(master_j) (node level, for every
 * component; see gls_set_hanging for the DoF-level lines). Velocity FE_Q(k) and pressure
 * FE_Q(kp) spaces, 1 <= kp <= k <= 2. Owned storage, freed by gls_mesh_refined_destroy. */
typedef struct {
  int dim, k, kp;
  int64_t n_cells, n_vnodes, n_pnodes;
  const int32_t *cell_vnodes;   /* [n_cells][(k+1)^dim] lexicographic local order */
  const int32_t *cell_pnodes;   /* [n_cells][(kp+1)^dim] */
  const int32_t *cell_level;    /* [n_cells] 0 unrefined, 1 child of a refined cell */
  const double *cell_x0, *cell_h;  /* [n_cells][dim] */
  const double *vnode_x, *pnode_x; /* [n_vnodes][dim], [n_pnodes][dim] */
  int64_t n_vhang;              /* hanging velocity node vhang_node[i] = sum over j in           */
  const int64_t *vhang_node;    /*   [vhang_off[i], vhang_off[i+1]) of vhang_w[j] * node          */
  const int64_t *vhang_off;     /*   vhang_master[j]                                              */
  const int64_t *vhang_master;
  const double *vhang_w;
  int64_t n_phang;              /* the same for the pressure nodes */
  const int64_t *phang_node, *phang_off, *phang_master;
  const double *phang_w;
  void *impl_;                  /* owned storage (opaque) */
} gls_refined_mesh;
int gls_mesh_refined_create(int dim, int n, int k, int kp, double lo, double hi, const int32_t *refine,
                            gls_refined_mesh **out);
int gls_mesh_refined_destroy(gls_refined_mesh *mesh);
/* Multi-level adaptive refinement of a hyper_cube (the reference's p4est forest,
 * navier_stokes_base.cc:55-60, 592-780): an octree over n^dim level-0 cells, leaves in p4est's
 * depth-first Morton order. gls_octree_adapt refines flagged leaves (below max_level), coarsens
 * complete sibling groups that are all flagged (above min_level) when that keeps the vertex 2:1
 * balance, and restores the balance by refinement (limit_level_difference_at_vertices).
 * gls_octree_mesh builds the FE_Q(k) x FE_Q(kp) node spaces with hanging lines whose masters are
 * all unconstrained (make_hanging_node_constraints + close()), as a gls_refined_mesh (free it with
 * gls_octree_mesh_destroy); gls_octree_transfer is SolutionTransfer between two such meshes of the
 * same cube (host vectors, [velocity node-major | pressure]). */
typedef struct gls_octree gls_octree;
int gls_octree_create(int dim, int n, gls_octree **out);
void gls_octree_destroy(gls_octree *tree);
/* Periodic directions (bit d of mask; before adapting): the balance, the smoothing's neighbourhoods and
 * the Kelly faces wrap around them, and gls_octree_mesh identifies the max face's nodes with the min
 * face's, hanging lines included (periodicity under local refinement, gls_navier_stokes.cc:130-134,
 * 164-168: make_periodicity_constraints closed together with the hanging-node constraints). */
int gls_octree_set_periodic(gls_octree *tree, int mask);
int gls_octree_info(const gls_octree *tree, int64_t *n_cells, int *max_level);
int gls_octree_cells(const gls_octree *tree, int32_t *level, double *x0, double *h, double lo, double hi);
int gls_octree_adapt(gls_octree *tree, const int32_t *refine, const int32_t *coarsen, int max_level, int min_level);
/* Triangulation::prepare_coarsening_and_refinement with the reference's mesh smoothing
 * (smoothing_on_refinement | smoothing_on_coarsening, navier_stokes_base.cc:55-60, called at :682):
 * do_not_produce_unrefined_islands, eliminate_refined_inner/boundary_islands,
 * limit_level_difference_at_vertices, eliminate_unrefined_islands, no double refinement at faces,
 * complete-family coarsening that keeps the 2:1 rule (fix_coarsen_flags), iterated until the flags no
 * longer change. refine / coarsen: per-leaf flags in the tree's order, updated in place. Returns the
 * number of iterations. */
int gls_octree_prepare(const gls_octree *tree, int32_t *refine, int32_t *coarsen);
int gls_octree_mesh(const gls_octree *tree, int k, int kp, double lo, double hi, gls_refined_mesh **out);
int gls_octree_mesh_destroy(gls_refined_mesh *mesh);
int gls_octree_transfer(const gls_refined_mesh *old_mesh, const gls_refined_mesh *new_mesh, const double *old_vec,
                        double *new_vec);
/* Kelly error indicator per cell: KellyErrorEstimator<dim>::estimate as
 * refine_mesh_kelly calls it (navier_stokes_base.cc:612-652) — face rule QGauss<dim-1>(n_q + 1),
 * no Neumann boundaries (boundary faces add nothing), deal.II's default cell_diameter_over_24:
 * eta_K = sqrt(sum over interior faces F of K of diam(K)/24 * int_F sum_c [d u_c / dn]^2) over the
 * velocity components (variable 0) or the pressure (variable 1). Conforming meshes (no hanging
 * nodes). sol, eta: DEVICE pointers (eta: n_cells doubles; deal.II stores them as float). */
int gls_kelly_estimate(gls_ctx *ctx, const double *sol, int variable, double *eta);
/* The same on meshes with hanging faces (gls_octree_mesh): the face pieces from gls_octree_faces
 * (the fine side of a non-conforming face is one piece; deal.II integrates over the subfaces), the
 * integrals on the device, each piece counted for both of its cells. sol, eta: DEVICE pointers. */
int gls_kelly_estimate_faces(gls_ctx *ctx, const double *sol, int variable, int64_t n_faces, const int32_t *fa,
                             const int32_t *fb, const int32_t *fdir, const double *rect_a, const double *rect_b,
                             double *eta);
int gls_octree_faces(const gls_refined_mesh *mesh, int64_t *n_faces, int32_t *fa, int32_t *fb, int32_t *fdir,
                     double *rect_a, double *rect_b);
/* Level meshes of a geometric multigrid on the refinement hierarchy (global coarsening; the reference's
 * level hierarchy of the p4est forest, not a reference interface -- its GLS solver uses ILU / ML-AMG,
 * gls_navier_stokes.cc:1161-1240): a copy of the forest with every leaf finer than `level` replaced by
 * its ancestor on `level` (2:1 balance preserved). Free with gls_octree_destroy. */
int gls_octree_coarsen_to(const gls_octree *tree, int level, gls_octree **out);
/* Prolongation between two nested octree meshes (coarse = a coarsening of fine): DoF-level CSR over the
 * fine DoFs, fine DoF i = sum_j P_ij coarse DoF j = the conforming coarse field (hanging nodes from their
 * lines) interpolated at the fine node; rows of fine hanging DoFs are empty, columns are coarse masters.
 * off: n_dofs(fine)+1, col / w: nnz; inject: n_dofs(coarse), the fine DoF at each coarse DoF's position.
 * off == NULL: nnz only. Host arrays; non-periodic. */
int gls_octree_mg_transfer(const gls_refined_mesh *fine, const gls_refined_mesh *coarse, int64_t *nnz, int64_t *off,
                           int32_t *col, double *w, int64_t *inject);
/* The same on mapped (MappingQ) meshes, conforming or adapted: pieces and geometry from
 * gls_fe_space_kelly_faces with nq = n_q + 1 (nqf = nq^(dim-1) points per piece, host arrays),
 * the jump integrals on the device; eta (DEVICE, n_cells) = sqrt(cell_diam/24 * sum of pieces). */
int gls_kelly_estimate_mapped(gls_ctx *ctx, const double *sol, int variable, int64_t n_pieces, int nqf,
                              const int32_t *ca, const int32_t *cb, const double *xi, const double *g,
                              const double *jxw, const double *cell_diam, double *eta);
/* GridRefinement::refine_and_coarsen_fixed_number, refinement part (navier_stokes_base.cc:654-661;
 * serial deal.II rule): flags[i] = 1 for the int(top_fraction * n_cells) largest criteria (every
 * cell >= the threshold value). Returns the number of flagged cells. HOST arrays. */
int gls_refine_fixed_number(int64_t n_cells, const float *criteria, double top_fraction, int32_t *flags);
/* parallel::distributed::GridRefinement::refine_and_coarsen_fixed_number (fraction_type 0) and
 * refine_and_coarsen_fixed_fraction (fraction_type 1), refinement part — the calls refine_mesh_kelly
 * makes (navier_stokes_base.cc:654-667; deal.II 9.2 distributed/grid_refinement.cc): bisection for
 * the threshold (25 steps at most) between the widened extremes of the criteria, the target being
 * int(f * n_cells) cells (f = top_fraction capped by adjust_refine_and_coarsen_number_fraction<dim>
 * so the refined mesh has at most max_n_cells cells) or top_fraction of the summed criteria;
 * flags[i] = 1 where criteria[i] >= threshold. criteria >= 0 over ALL cells (gathered), HOST
 * arrays; threshold may be NULL. Returns the number of flagged cells. */
int gls_refine_pd(int64_t n_cells, const float *criteria, int dim, int fraction_type, double top_fraction,
                  int64_t max_n_cells, int32_t *flags, double *threshold);
/* The same with coarsening (fraction coarsening = bottom_fraction): adjust_refine_and_coarsen_
 * number_fraction<dim> caps both fractions (and coarsens (n - max) / (1 - 2^-dim) cells when the mesh
 * already has max_n_cells); the bottom threshold leaves int((1 - bottom) * n) cells (or that fraction
 * of the summed criteria) above it, the lowest float when bottom = 0; mark_cells: refine[i] = 1 where
 * criteria >= top (GridRefinement::refine), coarsen[i] = 1 where criteria <= bottom and not refine
 * (GridRefinement::coarsen). thresholds[2] = {top, bottom} (may be NULL). Returns the refined count. */
int gls_refine_coarsen_pd(int64_t n_cells, const float *criteria, int dim, int fraction_type, double top_fraction,
                          double bottom_fraction, int64_t max_n_cells, int32_t *refine, int32_t *coarsen,
                          double *thresholds);
/* SolutionTransfer::interpolate (navier_stokes_base.cc:689-733) for the first refinement of the
 * uniform hyper_cube(n, lo, hi) that `mesh` was built from: coarse in canonical lattice numbering
 * ([velocity node-major | pressure]), fine in the refined mesh's numbering. HOST arrays. */
int gls_mesh_refined_interpolate(const gls_refined_mesh *mesh, int n, double lo, double hi, const double *coarse,
                                 double *fine);

/* ------------------------------------------------------------------------------------------
 * Unstructured quadrilateral / hexahedral meshes, host side.
 * gls_umesh_generate: GridGenerator::generate_from_name_and_arguments (source/core/grids.cc:30-36)
 *   for hyper_cube ("lo : hi : colorize"), hyper_rectangle ("p1 : p2 : colorize"),
 *   subdivided_hyper_rectangle ("n1,n2[,n3] : p1 : p2 : colorize"), hyper_shell (2D,
 *   "center : inner : outer : n_cells : colorize"; inner boundary 0, outer 1; SphericalManifold on
 *   every object), cylinder (3D, "radius : half_length"; axis x, hull 0, x = -L 1, x = +L 2;
 *   CylindricalManifold on the hull) and cylinder_shell (3D, "length : inner : outer : n_radial :
 *   n_axial"; axis z, builder-defined colouring inner 0, outer 1, z = 0 2, z = length 3;
 *   CylindricalManifold on every object).
 * gls_umesh_read_gmsh: GridIn::read_msh (grids.cc:21-28), ASCII 2.2 / 4.0 / 4.1; quads (2D) or
 *   hexes (3D); boundary id = physical tag of the boundary element (the entity tag when none).
 * gls_umesh_set_manifold / gls_umesh_boundary_manifold: set_manifold + set_all_manifold_ids_on_
 *   boundary (source/core/manifolds.cc:226-247); type 0 flat, 1 spherical(center), 2 cylindrical
 *   (axis through center).
 * gls_umesh_refine_global: refine_global with deal.II 9.2's new-vertex placement (line midpoints
 *   on the line's manifold, quad / hex centres by transfinite-interpolation weights); cells stay
 *   parent-major (children of cell c are 2^dim c + lexicographic child index).
 * gls_umesh_fe_space: FE_Q(k)^dim x FE_Q(kp) nodes (1 <= kp <= k <= 2), MappingQ(k, qmapping_all)
 *   support points per cell, node support points, boundary-id bits per node (bit b: the node lies
 *   on a boundary face with id b), cell->measure(); periodic pairs (id_a, id_b, direction) triples
 *   identify the nodes of id_b with their translates on id_a (make_periodicity_constraints).
 * gls_fe_space_transfer: SolutionTransfer::interpolate across one global refinement (HOST vectors).
 * ------------------------------------------------------------------------------------------ */
typedef struct gls_umesh gls_umesh;
typedef struct {
  int dim, k, kp;
  int64_t n_cells, n_vnodes, n_pnodes;
  const int32_t *cell_vnodes, *cell_pnodes;   /* [n_cells][(k+1)^dim], [n_cells][(kp+1)^dim] lexicographic */
  const double *vnode_x, *pnode_x;            /* [n][dim] support points (mapped) */
  const uint32_t *vnode_bid, *pnode_bid;      /* boundary-id bits per node */
  const double *cell_support;                 /* [n_cells][(k+1)^dim][dim]: gls_mesh_desc.cell_support, map_degree = k */
  const int32_t *cell_mapping;                /* mapping degree used per cell (1 or k) */
  const double *cell_measure;                 /* cell->measure() */
  double volume;                              /* GridTools::volume (sum of measures) */
  const int32_t *cell_level;                  /* refinement level of each active cell */
  int64_t n_vhang;                            /* hanging velocity node vhang_node[i] = sum over j in    */
  const int64_t *vhang_node, *vhang_off;      /*   [vhang_off[i], vhang_off[i+1]) of vhang_w[j] * node   */
  const int64_t *vhang_master;                /*   vhang_master[j] (make_hanging_node_constraints +      */
  const double *vhang_w;                      /*   close(); masters unconstrained)                       */
  int64_t n_phang;                            /* the same for the pressure nodes */
  const int64_t *phang_node, *phang_off, *phang_master;
  const double *phang_w;
  void *impl_;
} gls_fe_space;
int gls_umesh_generate(int dim, const char *grid_type, const char *grid_arguments, gls_umesh **out);
int gls_umesh_read_gmsh(int dim, const char *path, gls_umesh **out);
int gls_umesh_set_manifold(gls_umesh *mesh, int manifold_id, int type, const double *center, const double *axis);
int gls_umesh_boundary_manifold(gls_umesh *mesh, int boundary_id, int manifold_id);
int gls_umesh_refine_global(gls_umesh *mesh, int times);
int gls_umesh_info(const gls_umesh *mesh, int64_t *n_cells, int64_t *n_vertices, double *volume);
void gls_umesh_destroy(gls_umesh *mesh);
int gls_umesh_fe_space(const gls_umesh *mesh, int k, int kp, int qmapping_all, int n_periodic,
                       const int32_t *periodic, gls_fe_space **out);
int gls_fe_space_destroy(gls_fe_space *space);
int gls_fe_space_transfer(const gls_fe_space *coarse, const gls_fe_space *fine, const double *coarse_vec,
                          double *fine_vec);
/* Local adaptation of the triangulation (the reference's p::d::Triangulation with
 * smoothing_on_refinement | smoothing_on_coarsening, navier_stokes_base.cc:55-60, 592-780), on any
 * mesh above (gmsh, generators, manifolds; new vertices placed as refine_global places them):
 *   gls_umesh_prepare: prepare_coarsening_and_refinement with that smoothing (the steps of
 *     gls_octree_prepare, neighbours through shared faces); refine / coarsen are per-active-cell
 *     flags in the order of gls_umesh_fe_space's cells, updated in place; returns the iterations.
 *   gls_umesh_adapt: execute_coarsening_and_refinement: flagged cells refined, complete flagged
 *     families coarsened when the vertex 2:1 balance allows, balance restored by refinement.
 * A space built afterwards carries the hanging-node lines (gls_fe_space.vhang_* / phang_*) and its
 * cells' levels; gls_fe_space_transfer then maps vectors from any earlier space of the same mesh
 * (refinement, coarsening, several levels). */
int gls_umesh_prepare(const gls_umesh *mesh, int32_t *refine, int32_t *coarsen);
/* Unit normals at the velocity nodes of the boundary faces with id boundary_id (the averaged face
 * normals VectorTools::compute_no_normal_flux_constraints uses for a slip boundary,
 * gls_navier_stokes.cc:100-110); [n_vnodes][dim], zero off that boundary. Host array. */
int gls_fe_space_boundary_normals(const gls_fe_space *space, int boundary_id, double *normals);
/* Edges and corners of a slip boundary (compute_no_normal_flux_constraints constrains as many
 * velocity components as independent normal directions meet at a node): the node's face normals
 * grouped by direction (groups within 60 degrees merge: a smooth curved wall gives one), count[v] =
 * the rank of the group means (0 off the boundary, 1, 2 = an edge in 3D, dim = all components);
 * normals: [n_vnodes][3][dim], row i = unit mean of group i (row 0 = the node normal when count = 1). */
int gls_fe_space_boundary_normal_sets(const gls_fe_space *space, int boundary_id, int32_t *count, double *normals);
int gls_umesh_adapt(gls_umesh *mesh, const int32_t *refine, const int32_t *coarsen);
/* Periodic boundary pairs of the triangulation (the reference's add_periodicity after
 * collect_periodic_faces, grids.cc:41-58): n_periodic triples (id a, id b, direction). gls_umesh_prepare
 * then treats the faces across them as neighbours (mesh smoothing) and gls_umesh_adapt / the vertex 2:1
 * balance identify the translated vertices, so refinement levels differ by at most one across a periodic
 * boundary. A space built with the same pairs (gls_umesh_fe_space) identifies the partnered nodes and
 * constrains the nodes of a finer face to the coarser face across the boundary
 * (make_periodicity_constraints, gls_navier_stokes.cc:128-134, 162-168), and its Kelly faces
 * (gls_fe_space_kelly_faces) include the periodic face pieces. */
int gls_umesh_set_periodic(gls_umesh *mesh, int n_periodic, const int32_t *periodic);
/* Level meshes of a geometric multigrid on the triangulation's refinement hierarchy (global coarsening):
 * a copy whose active cells are the current ones with every cell finer than `level` replaced by its
 * ancestor on `level` (free with gls_umesh_destroy). gls_fe_space_mg_transfer: the prolongation between
 * the FE spaces of two such levels (coarse = a coarsening of fine's triangulation) as a DoF-level CSR over
 * the fine DoFs -- FE_Q's embedding of the coarse cell's field (hanging nodes from their lines) at the fine
 * node's reference position, whatever the mapping; fine hanging rows empty, coarse masters as columns --
 * and inject (n_dofs(coarse)): the fine DoF at each coarse DoF's node. off == NULL: nnz only. Feed both to
 * gls_mg_attach_transfers (the reference preconditions these meshes with ILU / ML-AMG,
 * gls_navier_stokes.cc:1161-1240). A P-LEVEL PAIR -- the same active cells (two spaces of one triangulation, or
 * of copies with the same hierarchy), the coarse space of lower degree (Q2-Q1 -> Q1-Q1) -- gives the coarse
 * degree's interpolant at the fine nodes (FE_Q's embedding of the lower degree) and the injection at the
 * shared nodes (the fine degree a multiple of the coarse one); other degree mismatches are GLS_EINVAL. */
int gls_umesh_coarsen_to(const gls_umesh *mesh, int level, gls_umesh **out);
int gls_fe_space_mg_transfer(const gls_fe_space *fine, const gls_fe_space *coarse, int64_t *nnz, int64_t *off,
                             int32_t *col, double *w, int64_t *inject);
/* Face pieces for KellyErrorEstimator with MappingQ on such a space (conforming faces one piece,
 * a face with a refined neighbour one piece per child face; geometry on the coarse side as deal.II's
 * present cell): cells ca / cb, and per QGauss<dim-1>(nq) point q of piece e the reference
 * coordinates xi[e][q][side][dim] of both sides, g[e][q][side][dim] = J^-1 n, jxw[e][q];
 * cell_diam[n_cells] = cell->diameter(). Host arrays; call with ca == NULL for the count. */
int gls_fe_space_kelly_faces(const gls_fe_space *space, int nq, int64_t *n_pieces, int32_t *ca, int32_t *cb,
                             double *xi, double *g, double *jxw, double *cell_diam);

/* ------------------------------------------------------------------------------------------
 * Drop-in I/O surface, host side.
 * Parameter files: deal.II ParameterHandler text (`subsection`/`end`, `set key = value`, `#`
 * comments, `\` continuation) as read by Parameters::*::parse_parameters (source/core/
 * parameters.cc) and BoundaryConditions (boundary_conditions.h:130-425). Entries are addressed
 * "subsection/subsection/key" with deal.II's whitespace normalisation.
 * ------------------------------------------------------------------------------------------ */
typedef struct gls_prm gls_prm;
int gls_prm_parse(const char *text_or_path, int is_path, gls_prm **out);
int gls_prm_get(const gls_prm *prm, const char *path, char *buf, int cap); /* length, or GLS_ENOTFOUND */
int gls_prm_n_entries(const gls_prm *prm);
int gls_prm_entry(const gls_prm *prm, int i, char *path, int path_cap, char *value, int value_cap);
void gls_prm_destroy(gls_prm *prm);

/* Function expressions: deal.II Functions::ParsedFunction / FunctionParser over muParser
 * ("Function expression" = ';'-separated components, "Function constants" = "a=1, b=2",
 * variables "x,y,z,t"; pi/Pi predefined; deal.II's extra functions if/int/ceil/floor/cot/csc/
 * sec/pow/erfc and log = natural log). out[p*n_comp + c], values[p*n_vars + v] (HOST arrays). */
typedef struct gls_expr gls_expr;
int gls_expr_create(const char *expr, const char *vars, const char *constants, gls_expr **out);
int gls_expr_n_components(const gls_expr *e);
int gls_expr_eval(const gls_expr *e, int64_t n_points, const double *values, double *out);
void gls_expr_destroy(gls_expr *e);

/* Output: NavierStokesBase::write_output_results (navier_stokes_base.cc:998-1086) — one patch per
 * cell with `subdivision` intervals (Lagrange cells when k > 1), point data velocity, pressure,
 * subdomain, vorticity, q_criterion [, velocity_eulerian when mesh->srf]; solution is a HOST
 * vector in this library's layout. Master records: write_vtu_and_pvd (solutions_output.cc:14-59). */
int gls_vtu_write(const char *filename, const gls_mesh_desc *mesh, const double *solution, int subdivision,
                  int subdomain, int binary);
int gls_pvtu_write(const char *filename, int dim, int srf, int n_pieces, const char *const *piece_files);
int gls_pvd_write(const char *filename, int n, const double *times, const char *const *files);

/* ------------------------------------------------------------------------------------------
 * Profiling hooks: time the next operator launches on the context stream with HIP events.
 * ------------------------------------------------------------------------------------------ */
int gls_timing_reset(gls_ctx *ctx);
/* which: 0 residual, 1 jacobian_apply, 2 diagonal, 3 J.v linearization (once per state),
 * 4 FP32 J.v of the mixed-precision V-cycle, 5 brick-surface slab sums (after each brick launch);
 * returns total ms and launch count */
int gls_timing_get(gls_ctx *ctx, int which, double *total_ms, int64_t *count);
int gls_timing_enable(gls_ctx *ctx, int enable);

#ifdef __cplusplus
}
#endif
#endif
