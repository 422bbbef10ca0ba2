// gls_launch.hpp — host-side launch entry points of the device kernels.
#pragma once
#include "gls_common.hpp"

namespace gls {

// deterministic scatter of the per-cell kernels' element vectors (P.ev): y = per-node sums in slot order
hipError_t gather_element_vectors(double *y, const double *ev, const int64_t *voff, const int64_t *vslot, int64_t nv,
                                  const int64_t *poff, const int64_t *pslot, int64_t np, int dim, hipStream_t s);
hipError_t launch_cell_kernel(int dim, int k, int kp, int nq1d, int mode, const OpParams &P, const Tables1D &T,
                              hipStream_t s);
bool cell_kernel_supported(int dim, int k, int kp, int nq1d);
// sum-factorized J.v of 3D Q2-Q1 / Q2-Q2 cells from the linearization cache (gls_cell_sf.hip); hipErrorNotSupported
// when the launch is not its case (launch_cell_kernel then runs the dense kernel). GLS_CELL_SF=0: dense (A/B, tests)
hipError_t launch_cell_sf_jv(int dim, int k, int kp, int nq1d, const OpParams &P, const Tables1D &T, hipStream_t s);
bool cell_sf_enabled();
int cell_kernel_cells_per_block(int dim, int k, int nq1d, bool probe = false);  // cells per workgroup
// sum-factorized 3D Qk-Qk kernels on 2x2x2 Morton bricks (residual, J.v); k in {1,2}
hipError_t launch_brick_kernel(int k, int mode, const OpParams &P, const Tables1D &T, hipStream_t s);
size_t brick_qdata_size(int k, int n_cells);  // doubles of MODE_LIN storage
// J.v in FP32 arithmetic from P.qdf (FP32 linearization); v, y FP64 (multigrid smoother operator)
hipError_t launch_brick_jv_f32(int k, const OpParams &P, const Tables1D &T, hipStream_t s);
hipError_t vec_to_f32(const double *a, float *b, int64_t n, hipStream_t s);
hipError_t vec_from_f32(const float *a, double *b, int64_t n, hipStream_t s);
// Q2 brick J.v in the pencil dataflow (gls_brick_pencil.hip; FP64 from P.qd or FP32 from P.qdf), same
// contract as the lane-per-point MODE_JVQ launch with a slab; hipErrorNotSupported when not applicable
// (probing, colored launches, no slab). GLS_PENCIL=0 disables it.
hipError_t launch_pencil_jv(const OpParams &P, const Tables1D &T, hipStream_t s, bool f32);
hipError_t launch_pencil_residual(const OpParams &P, const Tables1D &T, hipStream_t s);  // MODE_RESIDUAL, FP64
hipError_t launch_pencil_lin(const OpParams &P, const Tables1D &T, hipStream_t s);  // MODE_LIN (+ diagonal into P.y)
// MODE_RESLIN: residual (res_y / res_slab) + linearization (qd, qdf) + diagonal (y / slab) in one pass
hipError_t launch_pencil_reslin(const OpParams &P, const Tables1D &T, hipStream_t s);
hipError_t launch_pencil_ev(int mode, const OpParams &P, const Tables1D &T, hipStream_t s, bool f32 = false);  // forest sibling-group bricks -> element vectors
bool pencil_enabled();
// persistent wave-per-brick versions (gls_brick_wave.hip), selected by the launchers above
hipError_t launch_brick_wave(int k, int mode, const OpParams &P, const Tables1D &T, hipStream_t s);
hipError_t launch_brick_wave_jv_f32(int k, const OpParams &P, const Tables1D &T, hipStream_t s);
hipError_t launch_brick_wave_probe(int k, const OpParams &P, const Tables1D &T, int64_t j0, int nprobe, hipStream_t s);
size_t brick_wave_qdata_size(int k, int n_cells);

int brick_boundary_nodes(int k);  // NBND: brick-lattice nodes on the 2x2x2 brick's surface
// y[nodes[i]] = sum_{j in [off[i], off[i+1])} slab[slots[j]] (4 fields per node)
hipError_t brick_slab_sum(const double *slab, const int32_t *nodes, const int32_t *off, const int32_t *slots,
                          int64_t n_sum, int64_t n_vnodes, double *y, hipStream_t s);
// the same with an FP32 slab (slabf != nullptr) and/or a fused damped-Jacobi sweep (jb != nullptr:
// y holds x and is updated x <- x + jomega (jb - A x) / jd, rows in vmask use (A x)_i = jd_i x_i)
hipError_t brick_slab_sum_ex(const double *slab, const float *slabf, const int32_t *nodes, const int32_t *off,
                             const int32_t *slots, int64_t n_sum, int64_t n_vnodes, double *y, const uint8_t *vmask,
                             const double *jb, const double *jd, double jomega, hipStream_t s,
                             const double *rb = nullptr);  // rb (no jb): y = rb - A x
// the same sums on the structured hyper_cube (nb1 bricks per direction, lexicographic nodes, Morton
// bricks, no periodic wrap): slots computed from the lattice coordinates, no index arrays
hipError_t brick_slab_sum_cube(int k, int nb1, const double *slab, const float *slabf, int64_t n_vnodes, double *y,
                               const uint8_t *vmask, const double *jb, const double *jd, double jomega, hipStream_t s,
                               const double *rb = nullptr, double *x0 = nullptr);  // x0: OpParams::jx0's surface nodes
bool brick_fused_jacobi_supported(int k);  // the selected brick kernel honours OpParams::jx and ::slabf
// batched probing: Y[(j - j0) * n_dofs + i] += (J_cell-sum e_j)_i for nprobe unit vectors (MODE_JVQ)
bool brick_colors_supported(int k);  // colored brick launches (OpParams::bricks) available
bool brick_subset_supported(int k);  // brick-subset launches (OpParams::subset) available
hipError_t launch_brick_probe(int k, const OpParams &P, const Tables1D &T, int64_t j0, int nprobe, hipStream_t s);

// ---- BLAS-1 style kernels on device vectors (gls_vector_kernels.hip)
hipError_t vec_fill(double *x, int64_t n, double a, hipStream_t s);
hipError_t vec_copy(double *y, const double *x, int64_t n, hipStream_t s);
hipError_t vec_axpy(double *y, double a, const double *x, int64_t n, hipStream_t s);          // y += a x
hipError_t vec_axpby(double *y, double a, const double *x, double b, int64_t n, hipStream_t s);  // y = a x + b y
hipError_t vec_scale(double *x, double a, int64_t n, hipStream_t s);
hipError_t vec_div(double *y, const double *x, const double *d, int64_t n, hipStream_t s);       // y = x / d
// partial dot products: out[k] = sum_i A[k][i] * w[i] for k < nk (A rows have stride lda),
// written as per-block partials into work, reduced into out (device) by a second kernel.
hipError_t vec_multidot(const double *A, int64_t lda, int nk, const double *w, int64_t n, double *out,
                        double *work, hipStream_t s);
hipError_t vec_multidot2(const double *A, int64_t lda, int nk, const double *w, int64_t n1, int64_t off2, int64_t n2,
                         double *out, double *work, hipStream_t s);  // sums over [0,n1) U [off2, off2+n2)
// ghost exchange packing: buf[j*4 + {0,1,2,3}] <-> (vel comps, pressure) of local node nodes[j]
hipError_t vec_pack_nodes(const double *x, const int32_t *nodes, int64_t m, int64_t voff, double *buf, hipStream_t s);
hipError_t vec_unpack_nodes(double *x, const int32_t *nodes, int64_t m, int64_t voff, const double *buf, int add,
                            hipStream_t s);
// w -= sum_k h[k] * A[k]  (h on device); zero_init: w starts at 0 (not read)
hipError_t vec_multiaxpy(double *w, const double *A, int64_t lda, int nk, const double *h, double sign, int64_t n,
                         hipStream_t s, bool zero_init = false);
// w = y + a x
hipError_t vec_waxpy(double *w, const double *y, double a, const double *x, int64_t n, hipStream_t s);
// w -= sign * sum_k h[k] A[k] (nk <= 8, h on device), fused with out[k] = A[k] . w_new (k < nk, when
// dots) and out[dots ? nk : 0] = ||w_new||^2, both over the owned rows [0, n1) U [off2, off2 + n2)
hipError_t vec_multiaxpy_dots(double *w, const double *A, int64_t lda, int nk, const double *h, double sign, int64_t n,
                              int64_t n1, int64_t off2, int64_t n2, bool dots, double scale, double *out,
                              double *work, hipStream_t s);
// hanging-node constraint lines (CSR): distribute x[dof] = sum w src[master]; condense onto masters
hipError_t vec_csr_gather_set(double *x, const double *src, const int64_t *dof, const int64_t *off,
                              const int64_t *master, const double *w, int64_t n, hipStream_t s);
hipError_t vec_copy_gather_set(double *x, const double *v, const uint8_t *dmask, int64_t n, const int64_t *dof,
                               const int64_t *off, const int64_t *master, const double *w, int64_t nl, hipStream_t s);
hipError_t vec_csr_condense(double *y, const int64_t *tm, const int64_t *toff, const int64_t *tdof, const double *tw,
                            int64_t n, hipStream_t s);
hipError_t vec_csr_spmv(double *y, const double *x, const int64_t *off, const int32_t *col, const double *w, int64_t n,
                        bool add, hipStream_t s, int lanes = 1);  // y (+)= A x, CSR; lanes (1, 2, 4, 8, 16) per row
hipError_t vec_gather_scale_set(double *y, const double *d, const double *v, const int64_t *idx, int64_t m,
                                hipStream_t s, const double *rb = nullptr);  // y[idx] = d[idx]*v[idx] (rb: rb[idx] - d v)
// assembled-ILU helpers: x[idx] = a; val[ent] = y[row] (probe extraction; add: val[ent] += y[row]);
// a_ii <- r a_ii + sign(a_ii) t
hipError_t vec_set_const_indexed(double *x, const int32_t *idx, int64_t m, double a, hipStream_t s);
hipError_t csr_probe_extract(double *val, const int64_t *ent, const int32_t *row, int64_t m, const double *y,
                             hipStream_t s, bool add = false);
// dense column-major A (n x n, A[j * n + i] = A_ij, DoF numbering) from the ILU's probed CSR (rows / columns
// in its renumbered order, perm: DoF -> row); inv (n ints, scratch) receives row -> DoF. A is not zeroed here
hipError_t csr_to_dense(double *A, const int64_t *rowp, const int32_t *col, const double *val, const int32_t *perm,
                        const int32_t *inv, int64_t n, hipStream_t s);
hipError_t vec_permute(double *out, const double *in, const int32_t *idx, int64_t n, int dir, hipStream_t s);
// batched probing of the per-cell operator (nb probe vectors at stride bs / ys, element vectors at evs;
// pid[e] = probe of entry e, p0 = the batch's first probe)
hipError_t probe_set_batched(double *V, int64_t n, const int32_t *dofs, const int32_t *pid, int p0, int64_t m,
                             hipStream_t s);
hipError_t probe_extract_batched(double *val, const int64_t *ent, const int32_t *row, const int32_t *pid, int p0,
                                 int64_t m, const double *Y, int64_t n, hipStream_t s);
hipError_t vec_csr_gather_set_b(double *x, const int64_t *dof, const int64_t *off, const int64_t *master,
                                const double *w, int64_t n, int nb, int64_t bs, hipStream_t s);
hipError_t vec_csr_condense_b(double *y, const int64_t *tm, const int64_t *toff, const int64_t *tdof, const double *tw,
                              int64_t n, int nb, int64_t bs, hipStream_t s);
hipError_t vec_gather_scale_set_b(double *y, const double *d, const double *v, const int64_t *idx, int64_t m, int nb,
                                  int64_t bs, hipStream_t s);
hipError_t gather_element_vectors_b(double *y, const double *ev, const int64_t *voff, const int64_t *vslot, int64_t nv,
                                    const int64_t *poff, const int64_t *pslot, int64_t np, int dim, int nb, int64_t ys,
                                    int64_t evs, const uint8_t *act, int64_t el, int cb, int nblk, hipStream_t s);
// multicolor ILU triangular solves (gls_ilu_kernels.hip): y = L^-1 b, x = U^-1 y on node groups of <=
// kMaxGroupRows rows, colors in order (forward) / reverse order (backward)
constexpr int kMaxGroupRows = 4;
// multicolor ILU numeric factorization in place (same structures; rows of <= kIluMaxRow entries)
constexpr int kIluMaxRow = 640;
// the compact factorization (four workgroups per CU instead of three): rows of <= kIluCompactRow entries (Q2-Q1 3D
// cells of vertex valence <= 8: <= 402). Either needs fewer than 2^35 entries in all.
constexpr int kIluCompactRow = 448;
hipError_t ilu_mc_factor(const int32_t *grow, const int32_t *color_groups, int n_colors, const int64_t *rowp,
                         const int32_t *col, double *val, const int64_t *lsp, const int64_t *didx, double boost_tol,
                         double boost_val, const int64_t *moff, const uint16_t *map, bool compact, double *rdiag,
                         hipStream_t s);  // rdiag (n): 1 / U_ii, written row by row (read for the later colors' pivots)
// the factorization's row-position map (map == nullptr in ilu_mc_factor: column searches instead)
hipError_t ilu_mc_factor_map(int64_t n, const int64_t *rowp, const int32_t *col, const int64_t *lsp,
                             const int64_t *didx, const int64_t *moff, uint16_t *map, hipStream_t s);
// per node group (int64): r0, nr, rowp[r0], rowp[r0 + nr], rowp[r0 + 1..3] (INT64_MAX past nr), 0, lsp[4],
// usp[4], didx[4], rowp[r0 + 1..4] (the solves' group descriptor)
constexpr int kGroupDesc = 24;
hipError_t ilu_mc_solve(const int64_t *gdesc, const int32_t *color_groups, int n_colors, const int32_t *col,
                        const double *val, const double *b, double *y, double *x, const uint8_t *waves_lower,
                        const uint8_t *waves_upper, hipStream_t s);
hipError_t vec_pack_dofs(const double *x, const int32_t *dofs, int64_t m, double *buf, hipStream_t s);
hipError_t vec_unpack_dofs(double *x, const int32_t *dofs, int64_t m, const double *buf, hipStream_t s);
hipError_t vec_add_dofs_ordered(double *x, const int32_t *u, const int32_t *off, const int32_t *slot, int64_t n,
                                const double *buf, hipStream_t s);
hipError_t vec_add_nodes_ordered(double *x, const int32_t *u, const int32_t *off, const int32_t *slot, int64_t n,
                                 int64_t voff, const double *buf, hipStream_t s);  // 4 values per node slot
hipError_t csr_diag_perturb(double *val, const int64_t *didx, int64_t n, double athresh, double rthresh, hipStream_t s);
hipError_t vec_set_const_indexed64(double *x, const int64_t *idx, int64_t m, double a, hipStream_t s);
// x[u[i]] += sum of buf[slot[j]] over j in [off[i], off[i+1]) in order (u: 64-bit positions, the ILU's remote entries)
hipError_t vec_add_pos_ordered(double *x, const int64_t *u, const int32_t *off, const int32_t *slot, int64_t n,
                               const double *buf, hipStream_t s);
hipError_t vec_set_indexed(double *y, const int64_t *idx, const double *vals, int64_t m, hipStream_t s);  // y[idx]=vals (vals null -> 0)
int multidot_work_size();

// ---- Kelly error indicator (gls_kelly.hip): 1D tables of the selected space at the face rule
struct KellyTables {
  int nq;                             // face quadrature points per direction
  double w[kMaxQ1D];                  // Gauss weights on [0, 1]
  double V[kMaxQ1D][kMaxNodes1D];     // basis values at the face points
  double De[2][kMaxNodes1D];          // basis derivatives at xi = 0 and xi = 1
  double xq[kMaxQ1D];                 // Gauss points on [0, 1]
  double xn[kMaxNodes1D];             // support points (Gauss-Lobatto) of the basis
};
// face-list form for meshes with hanging faces: fint[e] = int over the piece of face e of
// sum_c [d_n u_c]^2, the piece being rect_a / rect_b in the reference coordinates of cell fa[e]
// (its face xi_d = 1) and fb[e] (its face xi_d = 0), d = fdir[e]; QGauss(T.nq)^(dim-1) on the piece
hipError_t launch_kelly_faces(int dim, int m, const int32_t *cell_nodes, const double *geo, const double *sol,
                              int64_t n_faces, const int32_t *fa, const int32_t *fb, const int32_t *fdir,
                              const double *rect_a, const double *rect_b, int ncomp, int64_t base, int stride,
                              const KellyTables &T, double *fint, hipStream_t s);
// mapped meshes: per piece e and face point q, xi / g [e][q][side][dim] (g = J^-1 n), jxw [e][q]
hipError_t launch_kelly_mapped(int dim, int m, const int32_t *cell_nodes, const double *sol, int64_t n_pieces, int nqf,
                               const int32_t *ca, const int32_t *cb, const double *xi, const double *g,
                               const double *jxw, int ncomp, int64_t base, int stride, const KellyTables &T,
                               double *fint, hipStream_t s);
// eta[cell] = sqrt(sum over faces with nbr >= 0 of diam/24 * int_F sum_c [d_n u_c]^2); component c of
// node n at sol[base + n * stride + c], c < ncomp; cell_nodes [n_cells][(m+1)^dim]; nbr [n_cells][2 dim]
hipError_t launch_kelly(int dim, int m, const int32_t *cell_nodes, const int32_t *nbr, const double *geo,
                        const double *sol, int n_cells, int ncomp, int64_t base, int stride, const KellyTables &T,
                        double *eta, hipStream_t s);

// ---- geometric multigrid (gls_mg_kernels.hip): nested Qk node lattices (boxes), k <= 2
hipError_t mg_inject(const double *fine, double *coarse, const int nf[3], const int nc[3], hipStream_t s);
// one-pass 3D transfer with per-axis tap tables [n_out][5] (index, weight) and tap counts [n_out]
hipError_t mg_transfer3d(const double *in, double *out, const int nin[3], const int nout[3],
                         const int32_t *const taps[3], const double *const w[3], const int32_t *const cnt[3],
                         hipStream_t s);
// two-pass transfer (LDS-tiled xy pass + z pass); work holds 4 * (xy of the smaller lattice) * (z of the
// larger) doubles. tile_fits: host check that a per-axis tap table (axis 0/1) fits the kernel's tiles.
hipError_t mg_transfer_2pass(const double *in, double *out, const int nin[3], const int nout[3], int restrict_,
                             const int32_t *const taps[3], const double *const w[3], const int32_t *const cnt[3],
                             double *work, hipStream_t s, int add = 0);  // add (prolongation): out += P in
int mg_transfer_tile_fits(int restrict_, int axis, int n_out, const int32_t *taps, const int32_t *cnt);
hipError_t mg_box_gather(const double *loc, double *box, const int32_t *map, int64_t nbox, int64_t nvl,
                         int64_t n_owned, hipStream_t s);  // n_owned < 0: all nodes
hipError_t mg_box_scatter(const double *box, double *loc, const int32_t *map, int64_t nbox, int64_t nvl,
                          hipStream_t s);
// coarsest-level direct solve: invert the probed matrix (Y column-major) into aug = [I | A^-1]
hipError_t mg_dense_invert(const double *Y, double *aug, int n, int *status, hipStream_t s);  // status: dropped columns
hipError_t mg_unit_step(double *e, int64_t j, hipStream_t s);  // e[j-1] = 0, e[j] = 1
// probed columns: constrained rows of column j become D_c(j) delta_ij (gls_jacobian_apply's rule)
hipError_t mg_probe_fix(double *Y, int64_t n, int64_t j0, int nprobe, const int64_t *con, int64_t ncon, const double *d,
                        hipStream_t s);
hipError_t mg_dense_apply(const double *aug, int n, const double *b, double *x, hipStream_t s);
// column-major n x n: row / column `pin` -> identity; zero one row (the LU path's gauge pin)
hipError_t mg_pin_dof(double *A, int64_t n, int64_t pin, hipStream_t s);
hipError_t mg_zero_row(double *A, int64_t n, int64_t row, hipStream_t s);
// x <- (LU)^-1 x for a dense FP32 LU factor without pivoting (column-major, lda = n; gls_mg_kernels.hip)
hipError_t dense_lu_solve_f32(const float *LU, int n, float *x, hipStream_t s, int bl = -1, int bu = -1);  // bl / bu: bandwidths (-1 dense)
hipError_t mg_jacobi_update(double *x, const double *b, const double *y, const double *d, double omega, int64_t n,
                            int zero_start, hipStream_t s);

}  // namespace gls
