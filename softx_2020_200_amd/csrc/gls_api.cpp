// gls_api.cpp — C-ABI implementation: context lifecycle, operator dispatch, GMRES, Newton,
// hyper_cube mesh and time-integration coefficients. Host C++17 over HIP.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <map>
#include <array>
#include <memory>
#include <string>
#include <vector>
#include <set>
#include <thread>

#include <rocblas/rocblas.h>
#include <rocsolver/rocsolver.h>
#include <rocsparse/rocsparse.h>
#include <rccl/rccl.h>

#include "../../include/gls_native.h"
#include "gls_common.hpp"
#include "gls_launch.hpp"
#include "gls_sparse.hpp"

namespace {

thread_local std::string g_err;

int set_err(int code, const char *fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

#define HIP_TRY(expr)                                                                          \
  do {                                                                                         \
    hipError_t e_ = (expr);                                                                    \
    if (e_ != hipSuccess) return set_err(GLS_EHIP, "%s: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__, __LINE__); \
  } while (0)

#define GLS_TRY(expr)          \
  do {                         \
    int r_ = (expr);           \
    if (r_ < 0) return r_;     \
  } while (0)

template <class T>
struct DevBuf {
  T *p = nullptr;
  size_t n = 0;
  DevBuf() = default;
  DevBuf(const DevBuf &) = delete;
  DevBuf &operator=(const DevBuf &) = delete;
  DevBuf(DevBuf &&o) noexcept : p(o.p), n(o.n) { o.p = nullptr; o.n = 0; }
  DevBuf &operator=(DevBuf &&o) noexcept {
    if (this != &o) { release(); p = o.p; n = o.n; o.p = nullptr; o.n = 0; }
    return *this;
  }
  ~DevBuf() { release(); }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
  }
  int alloc(size_t count) {
    release();
    if (count == 0) return GLS_OK;
    if (hipMalloc(&p, count * sizeof(T)) != hipSuccess) {
      p = nullptr;
      return set_err(GLS_ENOMEM, "hipMalloc of %zu bytes failed", count * sizeof(T));
    }
    n = count;
    return GLS_OK;
  }
  int upload(const T *h, size_t count) {
    GLS_TRY(alloc(count));
    if (count && hipMemcpy(p, h, count * sizeof(T), hipMemcpyHostToDevice) != hipSuccess)
      return set_err(GLS_EHIP, "upload failed");
    return GLS_OK;
  }
};

// ---------------- time coefficients (host) ----------------
// Variable-step BDF via divided differences of the backward time levels
// (restates source/core/bdf.cc:23-75: alpha = sum_j prod_{i<j}(t0-ti) * delta_j).
void bdf_delta(int p, int n, int j, const double *times, double *out) {
  if (j == 0) {
    for (int i = 0; i <= p; ++i) out[i] = 0.;
    out[n] = 1.;
    return;
  }
  double a[8], b[8];
  bdf_delta(p, n, j - 1, times, a);
  bdf_delta(p, n + 1, j - 1, times, b);
  const double inv = 1.0 / (times[n] - times[n + j]);
  for (int i = 0; i <= p; ++i) out[i] = (a[i] - b[i]) * inv;
}

bool is_sdirk(int s) { return s >= GLS_SDIRK2 && s <= GLS_SDIRK3_3; }

}  // namespace

int gls_internal_set_err(int code, const char *msg) { return set_err(code, "%s", msg); }
int gls_io_set_error(int code, const char *fmt, ...) {  // gls_io.cpp
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  return set_err(code, "%s", buf);
}

extern "C" {

const char *gls_last_error(void) { return g_err.c_str(); }
const char *gls_version(void) { return "softx_2020_200_amd 0.1 (gfx950)"; }

int gls_bdf_coefficients(int order, const double *dt, int n_dt, double *alpha) {
  if (order < 1 || order > 5 || !dt || !alpha || n_dt < order) return set_err(GLS_EINVAL, "bdf order/dt");
  double times[8];
  for (int i = 0; i <= order; ++i) {
    times[i] = 0.;
    for (int j = 0; j < i; ++j) times[i] -= dt[j];
  }
  for (int i = 0; i <= order; ++i) alpha[i] = 0.;
  double d[8];
  for (int j = 1; j <= order; ++j) {
    double factor = 1.;
    for (int i = 1; i < j; ++i) factor *= times[0] - times[i];
    bdf_delta(order, 0, j, times, d);
    for (int i = 0; i <= order; ++i) alpha[i] += factor * d[i];
  }
  return GLS_OK;
}

// SDIRK2 (alpha = 1 - 1/sqrt(2)) and the 3-stage L-stable SDIRK3 tables of source/core/sdirk.cc:11-44,
// expressed as stage residual coefficients [stage][outcome, step n, intermediate stages...].
int gls_sdirk_coefficients(int order, double dt, double *c) {
  if (!c || dt == 0.) return set_err(GLS_EINVAL, "sdirk args");
  const double sdt = 1. / dt;
  if (order == 2) {
    const double a = (2. - std::sqrt(2.)) / 2.;
    const double v[6] = {1. / a * sdt, -1. / a * sdt, 0., 1. / a * sdt, -(2 * a - 1) / a / a * sdt,
                         -(1 - a) / a / a * sdt};
    std::memcpy(c, v, sizeof(v));
    return GLS_OK;
  }
  if (order == 3) {
    const double g = 2.29428036027904;
    const double v[12] = {g, -g, 0., 0., g, -0.809559354637498, -1.48472100564154, 0.,
                          g, 2.87009860433106, -8.55612780155264, 3.39174883694255};
    for (int i = 0; i < 12; ++i) c[i] = v[i] * sdt;
    return GLS_OK;
  }
  return set_err(GLS_EINVAL, "sdirk order %d", order);
}

}  // extern "C"

// ============================================================================================
// FE tables
// ============================================================================================
namespace {

void legendre_pd(int n, double x, double &P, double &dP) {
  double p0 = 1., p1 = x;
  if (n == 0) { P = 1.; dP = 0.; return; }
  for (int m = 2; m <= n; ++m) {
    const double p2 = ((2. * m - 1.) * x * p1 - (m - 1.) * p0) / m;
    p0 = p1;
    p1 = p2;
  }
  P = p1;
  dP = n * (x * p1 - p0) / (x * x - 1.);
}

// QGauss(n) on [0,1]: Newton on the Legendre roots, ascending.
void gauss_points(int n, double *x, double *w) {
  for (int i = 0; i < n; ++i) {
    double z = std::cos(M_PI * (i + 0.75) / (n + 0.5)), P, dP;
    for (int it = 0; it < 100; ++it) {
      legendre_pd(n, z, P, dP);
      const double dz = P / dP;
      z -= dz;
      if (std::fabs(dz) < 1e-17) break;
    }
    legendre_pd(n, z, P, dP);
    x[n - 1 - i] = 0.5 * (1. + z);
    w[n - 1 - i] = 1. / ((1. - z * z) * dP * dP);
  }
}

// FE_Q support points (Gauss–Lobatto) on [0,1]
void lobatto_points(int k, double *x) {
  x[0] = 0.;
  x[k] = 1.;
  for (int i = 1; i < k; ++i) {
    double z = -std::cos(M_PI * i / k);
    for (int it = 0; it < 100; ++it) {
      double P, dP;
      legendre_pd(k, z, P, dP);
      const double d2P = (2. * z * dP - k * (k + 1.) * P) / (1. - z * z);
      const double dz = dP / d2P;
      z -= dz;
      if (std::fabs(dz) < 1e-17) break;
    }
    x[i] = 0.5 * (1. + z);
  }
  if (k == 2) x[1] = 0.5;
}

// Lagrange basis i on nodes xn (degree k): value, first and second derivative at s,
// via the barycentric-style product expansions.
void lagrange_1d(int k, const double *xn, int i, double s, double &v, double &d, double &dd) {
  v = 1.;
  d = 0.;
  dd = 0.;
  for (int j = 0; j <= k; ++j)
    if (j != i) v *= (s - xn[j]) / (xn[i] - xn[j]);
  for (int m = 0; m <= k; ++m) {
    if (m == i) continue;
    double t = 1. / (xn[i] - xn[m]);
    for (int j = 0; j <= k; ++j)
      if (j != i && j != m) t *= (s - xn[j]) / (xn[i] - xn[j]);
    d += t;
    for (int l = 0; l <= k; ++l) {
      if (l == i || l == m) continue;
      double t2 = 1. / ((xn[i] - xn[m]) * (xn[i] - xn[l]));
      for (int j = 0; j <= k; ++j)
        if (j != i && j != m && j != l) t2 *= (s - xn[j]) / (xn[i] - xn[j]);
      dd += t2;
    }
  }
}

gls::Tables1D make_tables(int k, int kp, int nq1d) {
  gls::Tables1D T;
  std::memset(&T, 0, sizeof(T));
  double xq[gls::kMaxQ1D], wq[gls::kMaxQ1D], xv[gls::kMaxNodes1D], xp[gls::kMaxNodes1D];
  gauss_points(nq1d, xq, wq);
  lobatto_points(k, xv);
  lobatto_points(kp, xp);
  for (int q = 0; q < nq1d; ++q) {
    T.w[q] = wq[q];
    T.xi[q] = xq[q];
    for (int a = 0; a <= k; ++a) lagrange_1d(k, xv, a, xq[q], T.V[q][a], T.D[q][a], T.S[q][a]);
    for (int a = 0; a <= kp; ++a) {
      double dd;
      lagrange_1d(kp, xp, a, xq[q], T.Vp[q][a], T.Dp[q][a], dd);
    }
  }
  return T;
}

}  // namespace

// ============================================================================================
// context
// ============================================================================================
struct gls_ctx {
  int dim = 0, k = 0, kp = 0, nq1d = 0, n_cells = 0, n_vnodes = 0, n_pnodes = 0, nq = 0;
  int64_t n_dofs = 0;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  gls::Tables1D tables;
  DevBuf<int32_t> cell_vnodes, cell_pnodes;
  DevBuf<int32_t> face_nbr;  // [n_cells][2 dim] face neighbours (Kelly), built on first use
  DevBuf<double> geo, x0, force_q;
  DevBuf<double> gq;               // mapped cells: per-q geometry [n_cells][nq][kGeo] (nullptr: boxes)
  std::vector<double> host_x0, host_h, host_support;  // host geometry for gls_quadrature_points
  int map_degree = 0;
  DevBuf<uint8_t> vmask;
  DevBuf<int64_t> con_dofs;  // zero_constraints DoF list
  DevBuf<int64_t> dir_dofs;  // nonzero_constraints (Dirichlet) list
  DevBuf<double> dir_vals;
  double viscosity = 1.0;
  int srf = 0;
  double omega[3] = {0, 0, 0};
  // time state
  int scheme = GLS_STEADY;
  double alpha[4] = {0, 0, 0, 0}, alpha_jac = 0., sdt2 = 0.;
  int n_hist = 0;
  // evaluation state (borrowed device pointers)
  const double *u = nullptr, *u1 = nullptr, *u2 = nullptr, *u3 = nullptr;
  DevBuf<double> diag;  // diagonal at the current state (also D_c for constrained rows)
  bool diag_valid = false;
  DevBuf<double> qdata;   // brick J.v linearization at the quadrature points (MODE_LIN output)
  bool qd_valid = false;  // invalidated with the diagonal by every state / parameter change
  // per-cell kernels: linearization cache (u, grad u, tau, R_s per quadrature point) written by the diagonal
  // pass and read by the J.v (OpParams::cq); valid with qd_valid's rules
  DevBuf<double> cq;
  bool cq_valid = false;
  DevBuf<float> qdata32;  // FP32 copy of qdata: the multigrid smoother's J.v (mixed precision)
  bool qd32_valid = false;  // stale whenever qdata is recomputed
  bool qd32_partial = false;  // the FP32 copy holds only u and tau (written for the Oseen smoother operator)
  // per-cell path: element vectors and each node's slots in them (deterministic scatter)
  DevBuf<double> ev;
  DevBuf<double> bev;  // batched ILU probing: element vectors of a batch of probe vectors
  DevBuf<uint8_t> bact;  // ... and which (probe, cell batch) blocks computed them
  DevBuf<int64_t> ev_voff, ev_vslot, ev_poff, ev_pslot;
  bool smooth_f32 = false;  // this level's V-cycle J.v runs in FP32 (gls_mg_params.mixed_precision)
  bool smooth_oseen = false;  // ... with the Oseen (Picard) operator (gls_mg_params.smoother_operator = 1)
  bool use_qdata = true;  // GLS_JV_RECOMPUTE=1 -> J.v recomputes the state per call (MODE_JV)
  // solver workspace
  DevBuf<double> work, scal, coef;  // multidot partials, device dot results, GMRES coefficients
  DevBuf<double> scal2;  // GMRES: the projection pass's dots (scal holds the coefficients it reads)
  double *hpin = nullptr;  // pinned host copy of the Gram-Schmidt dots (async D2H, one wait per pass pair)
  size_t hpin_n = 0;
  DevBuf<double> krylov;      // (restart+1) x n_dofs
  DevBuf<double> zbasis;      // restart x n_dofs: M^-1 v_j when the preconditioner is the V-cycle
  DevBuf<double> bicg;        // 7 x n_dofs BiCGStab work vectors (when the GMRES basis is smaller)
  int krylov_m = 0;
  DevBuf<double> tmp1, tmp2, tmp3, tmp4, tmp5;
  bool use_brick = false;  // sum-factorized brick kernels (3D Qk-Qk, Morton 2x2x2 bricks)
  // brick-boundary node sums without atomics: each brick stores its partial sums of its NBND
  // surface nodes into a slab; k_slab_sum adds a node's slots in a fixed order (CSR node -> slots)
  bool use_slab = false;
  DevBuf<double> slab;
  DevBuf<double> slab2;  // the fused residual + linearization pass: the residual's brick-surface slab
  DevBuf<int32_t> sum_nodes, sum_off, sum_slots;
  int cube_nb1 = 0;  // > 0: the mesh is the structured hyper_cube with cube_nb1 bricks per direction
                     // (k_slab_sum_cube computes the slab slots from the lattice; GLS_SLAB_CSR=1: off)
  // colored brick launches (opt-in GLS_BRICK_COLORS=1): bricks greedily colored in Morton order so
  // that no two bricks of a color share a node (the 2x2x2 parity classes on a brick lattice: 8
  // colors); surface-node sums carried across colors in acc, no slab and no k_slab_sum. Measured
  // slower at Q2 128^3 (profiles/r02_brick_colors_ab.txt: J.v 3.66 vs 3.00 + 0.55 ms, FP32 3.18 vs
  // 2.44 + 0.45 ms): a color's bricks are not neighbours, so the surface nodes neighbouring bricks
  // share are fetched again from HBM by the later colors instead of hitting L2.
  bool use_colors = false;
  int n_colors = 0;
  int color_off[17] = {0};
  DevBuf<int32_t> color_bricks;
  DevBuf<uint16_t> ncolor;
  DevBuf<double> acc;  // running sums for the fused Jacobi sweep (which stores x, not A x)
  // distributed (rank-local mesh): owned nodes [0, n_owned), ghosts after; exchange via callbacks
  struct Dist {
    bool on = false;
    // dofs: DoF-level exchange of a general mesh (gls_dist_attach_dofs: one double per DoF, owned
    // velocity nodes [0, n_owned) and owned pressure nodes [0, n_owned_p) first); else node-level
    // exchange of a Morton brick mesh (4 doubles per node)
    bool dofs = false;
    int width = 4;  // doubles per exchange entry
    int64_t n_owned = 0, n_owned_p = 0, n_send = 0, n_recv = 0;
    DevBuf<int32_t> add_u, add_off, add_slot;  // export-add (node or DoF exchange) in a fixed order
    DevBuf<int32_t> send_nodes, recv_nodes;
    double *send_buf = nullptr, *recv_buf = nullptr, *red_buf = nullptr;
    gls_exchange_fn xchg = nullptr;
    gls_allreduce_fn allreduce = nullptr;
    void *user = nullptr;
    // in-library RCCL transport (gls_dist_attach_rccl): grouped ncclSend / ncclRecv and ncclAllReduce
    // enqueued on the context stream -- no host callback, no host synchronisation per exchange
    ncclComm_t comm = nullptr;
    std::vector<int> nbrs;
    std::vector<int64_t> soff, roff;
    std::vector<int32_t> h_send, h_recv;  // host copies of the DoF exchange lists (gls_dist_attach_dofs)
    std::vector<int64_t> h_soff, h_roff;
    DevBuf<double> own_send, own_recv, own_red;
    // overlap of the J.v ghost import with the interior bricks (RCCL transport): exchange stream
    hipStream_t xstream = nullptr;
    hipEvent_t ev_ready = nullptr, ev_done = nullptr;
  } dist;
  // brick split for the overlapped J.v: bricks touching a ghost or exported node first
  // (split[0 .. split_bnd)), then the interior bricks (split[split_bnd .. split_bnd + split_int))
  DevBuf<int32_t> split;
  int split_bnd = 0, split_int = 0;
  // assembled ILU(0) preconditioner (gls_ilu_attach; the reference's setup_ILU,
  // gls_navier_stokes.cc:1161-1176): the Jacobian is assembled into CSR by probing the matrix-free
  // operator with distance-2-colored unit vectors, perturbed on the diagonal like Ifpack (athresh,
  // rthresh) and factored in place by rocSPARSE; M^-1 v = U^-1 L^-1 v (two sparse triangular solves)
  struct ILU {
    bool on = false, valid = false;
    // attached by the multigrid for its coarse matrix's probing pattern only (mg_probe_setup): never factored or
    // applied as a preconditioner / smoother of this context
    bool probe_only = false;
    double athresh = 0., rthresh = 1.;
    double boost_tol = 0., boost_val = 0.;  // rocsparse keeps these POINTERS and reads them in csrilu0
    int n_probes = 0, fill = 0;
    int64_t block_dofs = 0;  // subdomain size of the block-Jacobi ILU (gls_ilu_set_options); 0: one block
    int ordering = GLS_ILU_ORDER_CM, n_blocks = 1, n_order_colors = 0;
    // multicolor order with a pattern whose same-color entries stay inside a node (fill 0): the
    // color-by-color solves of gls_ilu_kernels.hip replace rocSPARSE csrsv
    bool mc_solve = false;
    bool mc_factor = false;  // multicolor order: color-by-color numeric factorization (no rocSPARSE csrilu0)
    bool mc_compact = false;  // ... by the compact-LDS kernel (rows <= kIluCompactRow)
    DevBuf<double> rdiag;     // ... its 1 / U_ii per row
    std::vector<uint8_t> mc_wl, mc_wu;  // per color: wavefronts per node group in the lower / upper solve
    DevBuf<int64_t> mc_desc;   // per node group: the solves' descriptor (gls::kGroupDesc int64)
    DevBuf<int64_t> mc_moff;   // factorization position map: per row, its first entry
    DevBuf<uint16_t> mc_map;   // per (row, pivot, upper entry of the pivot row): position in the row
    std::vector<int32_t> mc_cg;          // per color: first node group (host, n_colors + 1)
    DevBuf<int32_t> mc_grow;             // node group -> first row
    DevBuf<int64_t> mc_lsp, mc_usp;      // per row: L / U split entries
    DevBuf<int64_t> ghost_diag;          // across ranks: diagonal entries of the ghost (identity) rows
    // across ranks, complete owned rows: the neighbours' cell contributions to the owned x owned block
    // arrive per probe round through the export exchange (n_rounds = the largest probe count of any
    // rank); round p adds send_buf slots into CSR entries ru[rr[p] .. rr[p+1]) in a fixed order
    bool complete = false;
    int n_rounds = 0;
    std::vector<int64_t> rr;
    DevBuf<int64_t> ru;
    DevBuf<int32_t> ruoff, rslot;
    std::vector<int64_t> pdoff, peoff;   // per probe: offsets into pdofs and (pent, prow)
    DevBuf<int32_t> pdofs, prow;         // probe unit DoFs; the rows of the CSR entries filled by the probe
    DevBuf<int64_t> pent;                // those entries (positions: 64-bit, the fine levels pass 2^31 entries)
    DevBuf<int32_t> pdpid, pepid;        // probe of each unit DoF / each extracted entry (batched probing)
    DevBuf<double> bV, bC, bY;           // batched probing: probe vectors, C V (hanging lines), results [batch][n_dofs]
    // batched probing's activity: which (probe, cell batch) pairs have a nonzero C e_p on their cells depends on
    // the pattern and the hanging lines only, so the first probing records it (the kernel's flags, wact) and the
    // later ones launch just the active pairs (wlist, per chunk from woff; chunk size wB, batches wnblk)
    DevBuf<uint8_t> wact;
    DevBuf<int32_t> wlist;
    std::vector<int64_t> woff;
    int wB = 0;
    int64_t wnblk = 0;
    // CSR pattern (Cuthill-McKee or multicolor order), diagonal entry per row: 64-bit positions (a 13 M-DoF Q2-Q1
    // level has ~2.9e9 entries); rowp32: the 32-bit row pointers rocSPARSE takes, when the pattern fits them
    DevBuf<int64_t> rowp, didx;
    DevBuf<int32_t> col, rowp32;
    DevBuf<int32_t> perm;                // DoF -> its row in the factored (renumbered) matrix
    DevBuf<double> val, vbuf, ybuf, tbuf;
    DevBuf<char> work;
    rocsparse_handle h = nullptr;
    rocsparse_mat_descr dA = nullptr, dL = nullptr, dU = nullptr;
    rocsparse_mat_info info = nullptr;
    int64_t nnz = 0, nnz_a = 0;  // entries of the ILU(fill) pattern / of the system matrix
    void release() {
      if (info) rocsparse_destroy_mat_info(info);
      if (dA) rocsparse_destroy_mat_descr(dA);
      if (dL) rocsparse_destroy_mat_descr(dL);
      if (dU) rocsparse_destroy_mat_descr(dU);
      if (h) rocsparse_destroy_handle(h);
      info = nullptr;
      dA = dL = dU = nullptr;
      h = nullptr;
    }
    ~ILU() { release(); }
  } ilu;
  // hanging-node constraints (gls_set_hanging): lines dof <- sum w * master
  struct Hang {
    bool on = false;
    DevBuf<int64_t> dof, off, master, ooff, omaster;  // all lines; operator lines (Dirichlet masters dropped)
    DevBuf<double> w, ow;
    DevBuf<int64_t> tm, toff, tdof;                     // operator lines transposed: master -> (hanging dof, w)
    DevBuf<double> tw;
    DevBuf<uint8_t> hmask;                             // hanging velocity components per node
    DevBuf<uint8_t> dmask;                             // 1 on the hanging DoFs (C v in one pass)
    DevBuf<double> vbuf;                               // C v for J.v
    std::vector<int64_t> h_dof, h_off, h_master;       // host copy of the lines (ILU sparsity)
  } hang;
  // adapted forests (hanging contexts, 3D Q2-Q2 boxes): the complete sibling groups of leaves run the
  // pencil kernel (cached linearization, element-vector output), the other cells the per-cell kernel
  struct Oct {
    bool on = false;
    int nb = 0;
    DevBuf<int32_t> cell0, list;  // first cell of each brick; 0..nb-1 (the launch's brick list)
    DevBuf<int32_t> rest;         // the cells outside the bricks (the per-cell kernel's list)
    int n_rest = 0;
    bool f32_next = false;        // the next J.v: the bricks in FP32 from qdata32 (the V-cycle's smoother)
  } oct;
  // embedding in the global hyper_cube node lattice (gls_set_lattice): box of local nodes
  struct Lattice {
    bool set = false;
    int n1d = 0, box0[3] = {0, 0, 0}, bdim[3] = {0, 0, 0};
    DevBuf<int32_t> map;  // box node (x fastest) -> local node
  } lat;
  // geometric multigrid preconditioner (levels[0] == this context)
  struct MG {
    bool on = false;
    bool boxed = false;    // distributed levels: transfers go through box gather / scatter
    std::vector<gls_ctx *> lev;
    std::vector<std::array<int, 3>> dims;  // box lattice nodes per direction per level
    int k = 2, pre = 2, post = 2, csweeps = 30;
    std::vector<int> lpre, lpost;  // per-level sweep counts (default pre / post)
    double omega = 0.6, comega = 0.6;
    std::vector<std::unique_ptr<DevBuf<double>>> bufs;  // per level l>=1: u,u1,u2,u3,b,x,y ; level 0: y
    // per level pair (l, l+1) and axis: 1D tap tables [n_out][5] of prolongation / restriction
    struct Taps {
      DevBuf<int32_t> pi[3], ri[3], pc[3], rc[3];
      DevBuf<double> pw[3], rw[3];
      bool two_pass = false;  // the xy tiles of mg_transfer_2pass fit these tables
    };
    std::vector<std::unique_ptr<Taps>> taps;
    // general hierarchies (gls_mg_attach_transfers): per level pair the prolongation P (fine rows), the
    // restriction R = P^T (coarse rows) as CSR, and the state injection (coarse DoF <- fine DoF)
    bool csr = false;
    bool ilu_smooth = false;  // gls_mg_params.smoother = 1: ILU(0) sweeps on the levels above the coarsest
    struct Csr {
      DevBuf<int64_t> poff, roff;
      DevBuf<int32_t> pcol, rcol, inj;
      DevBuf<double> pw, rw;
      int64_t nf = 0, nc = 0;
      int plane = 1, rlane = 1;  // SpMV lanes per row (from the mean row length)
    };
    std::vector<std::unique_ptr<Csr>> xfer;
    std::vector<gls_ctx *> ilu_levels;  // levels whose ILU(0) smoother this attach created (smoother = 1)
    DevBuf<double> xwork;  // two-pass transfer intermediate (coarse xy x fine z, 4 fields)
    // coarsest level: direct solve with the probed, regularised, inverted Jacobian
    bool direct = false, direct_ok = false;
    // per-cell coarsest level: its matrix for the direct solve assembled by the ILU's colored batched probes
    // (a structure-only ILU(0) on that level, never factored) instead of one J.v per column
    gls_ctx *probe_ilu = nullptr;
    DevBuf<int32_t> pinv;
    // direct solve by LU (rocSOLVER getrf + getri -> explicit inverse, applied by rocBLAS gemv) with
    // the first pressure DoF pinned (enclosed-flow gauge); falls back to the one-workgroup
    // Gauss-Jordan (mg_dense_invert) for small levels or when the LU reports a zero pivot
    bool lu = false;
    // large coarsest levels (kDirectSmall < n <= kDirectMax, e.g. a Q1-Q1 p-level of a 4.7 k-cell base mesh):
    // the pinned FP64 matrix rounded to FP32, pivoted sgetrf + sgetri, applied by sgemv (a preconditioner's
    // coarse solve: FP32 rounding of A^-1 is far below the V-cycle's own error; half the bytes and the FP32
    // matrix-core rate for the O(n^3) setup)
    bool lu32 = false;
    bool lu32_npvt = false;  // the FP32 factor is unpivoted (applied by dense_lu_solve_f32), else an explicit inverse
    bool lu32_refine = false;  // ... applied with one step of iterative refinement against the FP64 matrix
    // banded coarse matrix: the probed CSR's Cuthill-McKee order kept (the dense array holds A in that order), its
    // lower / upper bandwidths; the factorization works by column blocks as wide as the band (no fill outside it
    // without pivoting) and the solves skip the blocks outside it. configs[4]'s 25 k-DoF Q1-Q1 p-level: ~1.9 k
    bool lu_cm = false;
    int64_t lu_bl = -1, lu_bu = -1, lu_pin_cm = -1;
    DevBuf<int32_t> lu_ident;  // identity permutation (csr_to_dense in the CSR's own order)
    DevBuf<double> lu_tmp;     // the coarse right-hand side / correction in that order
    DevBuf<float> probe32, b32, x32;
    DevBuf<double> chk32;    // the FP32 factor's check: A x - b for b = 1 (FP64)
    int64_t npvt_ipiv_n = -1;  // ipiv holds the identity permutation of this size (unpivoted LU)
    struct Blas {  // owning rocBLAS handle (movable, destroyed with the MG state)
      rocblas_handle h = nullptr;
      Blas() = default;
      Blas(const Blas &) = delete;
      Blas &operator=(const Blas &) = delete;
      Blas(Blas &&o) noexcept : h(o.h) { o.h = nullptr; }
      Blas &operator=(Blas &&o) noexcept {
        if (this != &o) {
          if (h) rocblas_destroy_handle(h);
          h = o.h;
          o.h = nullptr;
        }
        return *this;
      }
      ~Blas() {
        if (h) rocblas_destroy_handle(h);
      }
      operator rocblas_handle() const { return h; }
    } blas;
    DevBuf<int> ipiv, info;
    DevBuf<double> probe, aug, unit;
    DevBuf<double> probe_bak;  // the probed coarse matrix kept for the pivoted retry of an unpivoted LU
    DevBuf<double> chk;        // coarse_inverse_check's y = A^-1 e and z = A y
    DevBuf<int> status;
    // the FP32 unpivoted factorization and its check run on a stream of their own, overlapping the finer levels'
    // ILU setup and first smoothing on the context stream; the first coarse solve waits for them
    // (coarse_lu32_finish). Declared after the buffers it uses, so it is destroyed (synchronized) first.
    // rocSOLVER's getrf returns to the host only when the factorization is done (82-89 ms of host time at
    // n = 25000, box r06v), so the calls are made from a worker thread: the host thread queues the finer levels'
    // setup meanwhile
    struct Side {
      hipStream_t s = nullptr;
      hipEvent_t e0 = nullptr, e1 = nullptr;
      std::thread worker;
      int rc = 0;  // the worker's result: 0, or the failing call's number
      Side() = default;
      Side(const Side &) = delete;
      Side &operator=(const Side &) = delete;
      Side(Side &&o) noexcept : s(o.s), e0(o.e0), e1(o.e1), worker(std::move(o.worker)), rc(o.rc) {
        o.s = nullptr, o.e0 = o.e1 = nullptr;
      }
      Side &operator=(Side &&o) noexcept {
        if (this != &o) {
          reset();
          s = o.s, e0 = o.e0, e1 = o.e1, worker = std::move(o.worker), rc = o.rc;
          o.s = nullptr, o.e0 = o.e1 = nullptr;
        }
        return *this;
      }
      void join() {
        if (worker.joinable()) worker.join();
      }
      hipError_t ensure() {
        if (s) return hipSuccess;
        hipError_t e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&e0, hipEventDisableTiming);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&e1, hipEventDisableTiming);
        return e;
      }
      void reset() {
        join();
        if (s) {
          (void)hipStreamSynchronize(s);
          (void)hipStreamDestroy(s);
        }
        if (e0) (void)hipEventDestroy(e0);
        if (e1) (void)hipEventDestroy(e1);
        s = nullptr, e0 = e1 = nullptr;
      }
      ~Side() { reset(); }
    } side;
    bool lu_pending = false;  // side-stream factorization in flight, not yet checked
    int64_t lu_n = 0, lu_pin = 0;
    DevBuf<double> lu_rel;  // |A x - 1| of the check (device pointer mode)
    // coarsest-level Jacobi sweeps (single rank, fused brick path) replayed as one HIP graph: the
    // ~2×csweeps tiny launches per V-cycle are captured once per state (mg_prepare) and launched
    // as a single graph by every V-cycle of that Newton step
    struct Graph {
      hipGraphExec_t h = nullptr;
      Graph() = default;
      Graph(const Graph &) = delete;
      Graph &operator=(const Graph &) = delete;
      Graph(Graph &&o) noexcept : h(o.h) { o.h = nullptr; }
      Graph &operator=(Graph &&o) noexcept {
        if (this != &o) {
          reset();
          h = o.h;
          o.h = nullptr;
        }
        return *this;
      }
      void reset() {
        if (h) (void)hipGraphExecDestroy(h);
        h = nullptr;
      }
      ~Graph() { reset(); }
    } cgraph;
    std::vector<unsigned char> cgraph_key;  // launch parameters the graph was captured with
    bool cgraph_failed = false;  // capture refused once: stay on plain launches
    bool dirty = true;
    // multi-GPU (gls_mg_set_coarse_replica): the coarsest DISTRIBUTED level's correction is computed
    // by a replica -- a single-rank context of that level's whole mesh with its own hierarchy below
    // it -- identically on every rank, from the all-reduced (gathered) right-hand side
    gls_ctx *replica = nullptr;
    // general hierarchies across ranks (gls_mg_attach_replica): the distributed fine level smooths its own
    // rows, every coarser level is a replica on every rank (rep2, with its own hierarchy); restriction over the
    // rank's OWNED fine rows into the replica numbering + a sum all-reduce, prolongation onto all local rows
    bool rep_csr = false;
    gls_ctx *rep2 = nullptr;
    DevBuf<int64_t> r2p_off, r2r_off;  // P (local fine rows x replica DoFs), R = P_owned^T (replica rows)
    DevBuf<int32_t> r2p_col, r2r_col;
    DevBuf<double> r2p_w, r2r_w;
    int r2p_lane = 1, r2r_lane = 1;
    DevBuf<int32_t> r2inj_c, r2inj_f;  // replica DoF <- owned local fine DoF (state injection pairs)
    DevBuf<int32_t> rep_own_loc, rep_own_glob;  // owned local rows of the coarsest level -> replica rows
    DevBuf<int32_t> rep_map;                    // every local row -> replica row
    DevBuf<double> rep_b, rep_x, rep_tmp, rep_u[4];
  } mg;
  double time_steps[4] = {1, 1, 1, 1};
  // frozen Jacobian (skip_newton: the matrix and its preconditioner are reused across Newton
  // iterations, skip_newton_non_linear_solver.h:66-70, 126-130): snapshot of the state and time
  // coefficients the Jacobian operators (J.v, diagonal, linearization, multigrid levels) are taken
  // at, while gls_set_state / gls_set_time move only the residual's state
  struct JacFreeze {
    bool on = false;
    DevBuf<double> u, h[3];
    bool has[3] = {false, false, false};
    double alpha[4] = {0, 0, 0, 0}, alpha_jac = 0., sdt2 = 0., ts[4] = {1, 1, 1, 1};
    int n_hist = 0, scheme = GLS_STEADY;
  } jf;
  int skip_consecutive = 0;  // SkipNewtonNonLinearSolver::consecutive_iters (persists across solves)
  bool probe_local = false;  // ILU probe across ranks: J.v on the rank's cells only (no ghost exchange)
  // TimerOutput sections of the reference's Newton/GMRES path (gls_section_timing): wall seconds and
  // calls, stream-synchronised at the section boundaries while enabled
  bool sec_on = false;
  double sec_t[GLS_N_SECTIONS] = {};
  int sec_n[GLS_N_SECTIONS] = {};
  // timing
  bool timing = false;
  struct Ev { int which; hipEvent_t a, b; };
  std::vector<Ev> events;
  // residual, J.v, diagonal, J.v linearization, FP32 smoother J.v, brick-surface slab sums
  double t_ms[6] = {0, 0, 0, 0, 0, 0};
  int64_t t_n[6] = {0, 0, 0, 0, 0, 0};

  ~gls_ctx() {
    if (hpin) (void)hipHostFree(hpin);
    for (auto &e : events) { (void)hipEventDestroy(e.a); (void)hipEventDestroy(e.b); }
    if (dist.ev_ready) (void)hipEventDestroy(dist.ev_ready);
    if (dist.ev_done) (void)hipEventDestroy(dist.ev_done);
    if (dist.xstream) (void)hipStreamDestroy(dist.xstream);
    if (own_stream && stream) (void)hipStreamDestroy(stream);
  }
};

namespace {

// The brick kernels need: 3D, equal order k==kp in {1,2}, QGauss(k+1), pressure on the velocity
// nodes, and every 8 consecutive cells forming a conforming 2x2x2 brick (Morton order) whose
// interior nodes belong to no other brick (they are written with plain stores).
bool detect_bricks(const gls_mesh_desc *d, int nq1d) {
  if (getenv("GLS_DISABLE_BRICK")) return false;
  if (d->dim != 3 || d->k != d->kp || (d->k != 1 && d->k != 2) || nq1d != d->k + 1) return false;
  if (d->cell_pnodes || d->n_cells % 8 != 0 || d->n_cells == 0) return false;
  const int K = d->k, K1 = K + 1, N3 = K1 * K1 * K1, BN = 2 * K + 1;
  const int nb = d->n_cells / 8;
  std::vector<int32_t> owner((size_t)d->n_vnodes, -1);
  std::vector<int32_t> bnode((size_t)BN * BN * BN);
  for (int b = 0; b < nb; ++b) {
    std::fill(bnode.begin(), bnode.end(), -1);
    for (int cc = 0; cc < 8; ++cc) {
      const int cx = cc & 1, cy = (cc >> 1) & 1, cz = cc >> 2;
      const int32_t *cv = d->cell_vnodes + ((size_t)b * 8 + cc) * N3;
      for (int a = 0; a < N3; ++a) {
        const int ax = a % K1, ay = (a / K1) % K1, az = a / (K1 * K1);
        const int n = (K * cx + ax) + BN * ((K * cy + ay) + BN * (K * cz + az));
        if (bnode[n] == -1) bnode[n] = cv[a];
        else if (bnode[n] != cv[a]) return false;  // not a conforming brick
      }
    }
    for (int Z = 1; Z < BN - 1; ++Z)
      for (int Y = 1; Y < BN - 1; ++Y)
        for (int X = 1; X < BN - 1; ++X) {
          const int32_t node = bnode[X + BN * (Y + BN * Z)];
          if (owner[node] != -1) return false;
          owner[node] = b;
        }
  }
  for (int cix = 0; cix < d->n_cells; ++cix)
    for (int a = 0; a < N3; ++a) {
      const int32_t o = owner[d->cell_vnodes[(size_t)cix * N3 + a]];
      if (o != -1 && o != cix / 8) return false;
    }
  return true;
}

// node -> slab slots of the bricks whose surface holds it (CSR sorted by node, slots ascending)
int build_slab_map(gls_ctx *c, const gls_mesh_desc *d) {
  const int K = d->k, K1 = K + 1, N3 = K1 * K1 * K1, BN = 2 * K + 1;
  const int nbnd = gls::brick_boundary_nodes(K);
  const int64_t nb = d->n_cells / 8;
  if (nb * nbnd >= INT32_MAX) return GLS_OK;  // keep atomics beyond int32 slot ids
  std::vector<int32_t> cnt((size_t)d->n_vnodes + 1, 0), slot_node((size_t)(nb * nbnd));
  for (int64_t b = 0; b < nb; ++b) {
    int j = 0;
    for (int Z = 0; Z < BN; ++Z)
      for (int Y = 0; Y < BN; ++Y)
        for (int X = 0; X < BN; ++X) {
          if (X > 0 && X < BN - 1 && Y > 0 && Y < BN - 1 && Z > 0 && Z < BN - 1) continue;
          const int cx = std::min(X / K, 1), cy = std::min(Y / K, 1), cz = std::min(Z / K, 1);
          const int a = (X - K * cx) + K1 * ((Y - K * cy) + K1 * (Z - K * cz));
          const int32_t node = d->cell_vnodes[((size_t)b * 8 + cx + 2 * cy + 4 * cz) * N3 + a];
          slot_node[(size_t)(b * nbnd + j)] = node;
          ++cnt[(size_t)node + 1];
          ++j;
        }
    if (j != nbnd) return set_err(GLS_EINVAL, "brick boundary count %d != %d", j, nbnd);
  }
  std::vector<int32_t> nodes, off{0};
  std::vector<int32_t> start((size_t)d->n_vnodes + 1, 0);
  for (int64_t n = 0; n < d->n_vnodes; ++n) {
    start[(size_t)n + 1] = start[(size_t)n] + cnt[(size_t)n + 1];
    if (cnt[(size_t)n + 1] > 0) {
      nodes.push_back((int32_t)n);
      off.push_back(start[(size_t)n + 1]);
    }
  }
  std::vector<int32_t> slots((size_t)(nb * nbnd)), fill(start.begin(), start.end() - 1);
  for (int64_t sl = 0; sl < nb * nbnd; ++sl) slots[(size_t)fill[(size_t)slot_node[(size_t)sl]]++] = (int32_t)sl;
  const std::vector<int32_t> slots_by_node = slots;  // node n's slots at [start[n], start[n+1])
  // sum order: nodes by their first (lowest) slot, i.e. in slab order of their lowest brick, so
  // that consecutive threads of k_slab_sum read consecutive slab entries (node order would leave
  // the x-face nodes of every brick row 4 lattice points apart: 2.3x read amplification, PMC)
  {
    const size_t m = nodes.size();
    std::vector<int32_t> perm(m);
    for (size_t i = 0; i < m; ++i) perm[i] = (int32_t)i;
    std::sort(perm.begin(), perm.end(), [&](int32_t a, int32_t b) { return slots[(size_t)off[a]] < slots[(size_t)off[b]]; });
    std::vector<int32_t> n2(m), off2{0}, s2;
    s2.reserve(slots.size());
    for (size_t i = 0; i < m; ++i) {
      const int32_t a = perm[i];
      n2[i] = nodes[(size_t)a];
      for (int32_t j = off[(size_t)a]; j < off[(size_t)a + 1]; ++j) s2.push_back(slots[(size_t)j]);
      off2.push_back((int32_t)s2.size());
    }
    nodes.swap(n2);
    off.swap(off2);
    slots.swap(s2);
  }
  GLS_TRY(c->sum_nodes.upload(nodes.data(), nodes.size()));
  GLS_TRY(c->sum_off.upload(off.data(), off.size()));
  GLS_TRY(c->sum_slots.upload(slots.data(), slots.size()));
  c->use_slab = true;
  // structured hyper_cube (gls_mesh_hyper_cube: lexicographic node lattice, cells in Morton order, no
  // periodic wrap): verified cell by cell, then the slab sums run without the index arrays
  c->cube_nb1 = 0;
  if (!std::getenv("GLS_SLAB_CSR")) {
    int64_t n = (int64_t)std::llround(std::cbrt((double)d->n_cells));
    const int64_t NX = K * n + 1;
    bool ok = n >= 2 && n % 2 == 0 && n * n * n == d->n_cells && NX * NX * NX == d->n_vnodes && n <= 2048;
    for (int64_t cl = 0; ok && cl < d->n_cells; ++cl) {
      const int64_t b = cl / 8, ci = cl % 8;
      int64_t bx = 0, by = 0, bz = 0;
      for (int bit = 0; bit < 21; ++bit) {
        bx |= ((b >> (3 * bit)) & 1) << bit;
        by |= ((b >> (3 * bit + 1)) & 1) << bit;
        bz |= ((b >> (3 * bit + 2)) & 1) << bit;
      }
      if (bx >= n / 2 || by >= n / 2 || bz >= n / 2) { ok = false; break; }
      const int64_t x0 = K * (2 * bx + (ci & 1)), y0 = K * (2 * by + ((ci >> 1) & 1)), z0 = K * (2 * bz + (ci >> 2));
      for (int a = 0; a < N3 && ok; ++a) {
        const int ax = a % K1, ay = (a / K1) % K1, az = a / (K1 * K1);
        ok = d->cell_vnodes[(size_t)cl * N3 + a] == (int32_t)((x0 + ax) + NX * ((y0 + ay) + NX * (z0 + az)));
      }
    }
    if (ok) c->cube_nb1 = (int)(n / 2);
  }
  // brick coloring: greedy in brick (Morton) order over the bricks sharing a surface node
  if (!gls::brick_colors_supported(K)) return GLS_OK;  // only in a -DGLS_BRICK_COLORS_BUILD library (A/B)
  std::vector<int> color((size_t)nb, -1);
  int ncol = 0;
  for (int64_t b = 0; b < nb; ++b) {
    uint32_t used = 0;
    for (int j = 0; j < nbnd; ++j) {
      const int32_t node = slot_node[(size_t)(b * nbnd + j)];
      for (int32_t t = start[(size_t)node]; t < start[(size_t)node + 1]; ++t) {
        const int64_t ob = slots_by_node[(size_t)t] / nbnd;
        if (ob != b && color[(size_t)ob] >= 0) used |= 1u << color[(size_t)ob];
      }
    }
    int col = 0;
    while (col < 32 && ((used >> col) & 1u)) ++col;
    if (col >= 16) return GLS_OK;  // more than 16 colors: keep the slab path
    color[(size_t)b] = col;
    ncol = std::max(ncol, col + 1);
  }
  std::vector<uint16_t> ncm((size_t)d->n_vnodes, 0);
  for (int64_t sl = 0; sl < nb * nbnd; ++sl) ncm[(size_t)slot_node[(size_t)sl]] |= (uint16_t)(1u << color[(size_t)(sl / nbnd)]);
  std::vector<int32_t> order;
  order.reserve((size_t)nb);
  c->color_off[0] = 0;
  for (int col = 0; col < ncol; ++col) {
    for (int64_t b = 0; b < nb; ++b)
      if (color[(size_t)b] == col) order.push_back((int32_t)b);
    c->color_off[col + 1] = (int)order.size();
  }
  GLS_TRY(c->color_bricks.upload(order.data(), order.size()));
  GLS_TRY(c->ncolor.upload(ncm.data(), ncm.size()));
  c->n_colors = ncol;
  c->use_colors = true;
  return GLS_OK;
}

// colored brick launch: surface-node sums carried in acc (y, or scratch for the fused Jacobi sweep)
void set_colors(gls_ctx *c, gls::OpParams &P, double *acc) {
  P.bricks = c->color_bricks.p;
  P.ncolor = c->ncolor.p;
  P.acc = acc;
  P.n_colors = c->n_colors;
  for (int i = 0; i <= c->n_colors; ++i) P.color_off[i] = c->color_off[i];
  P.slab = nullptr;
  P.slabf = nullptr;
}

// brick launch output: slab (allocated on first use) or nullptr (atomics into a zeroed y)
double *brick_slab(gls_ctx *c) {
  if (!c->use_slab) return nullptr;
  const size_t n = (size_t)(c->n_cells / 8) * gls::brick_boundary_nodes(c->k) * 4;
  if (c->slab.n != n && c->slab.alloc(n) != GLS_OK) return nullptr;
  return c->slab.p;
}

// MappingQ(md) on one cell at the QGauss(nq1d) points: x_q, JxW, J^-1, G = J^-1 J^-T and the
// Hessian correction c_k = sum_ab G_ab d2x_k/dxi_a dxi_b (kGeo layout, gls_common.hpp); support
// points S[(md+1)^dim][dim] on the equidistant lattice (Gauss-Lobatto for md <= 2)
void mapped_geometry(int dim, int md, int nq1d, const double *S, double *out) {
  double xq[gls::kMaxQ1D], wq[gls::kMaxQ1D];
  gauss_points(nq1d, xq, wq);
  const int m1 = md + 1, ns = gls::ipow(m1, dim), nq = gls::ipow(nq1d, dim);
  double xn[4];
  for (int i = 0; i <= md; ++i) xn[i] = (double)i / md;
  double L[gls::kMaxQ1D][4], dL[gls::kMaxQ1D][4], ddL[gls::kMaxQ1D][4];
  for (int q = 0; q < nq1d; ++q)
    for (int a = 0; a <= md; ++a) lagrange_1d(md, xn, a, xq[q], L[q][a], dL[q][a], ddL[q][a]);
  for (int q = 0; q < nq; ++q) {
    const int qi[3] = {q % nq1d, (q / nq1d) % nq1d, dim == 3 ? q / (nq1d * nq1d) : 0};
    double x[3] = {0, 0, 0}, J[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
    double H[3][3][3] = {};
    for (int b = 0; b < ns; ++b) {
      const int ib[3] = {b % m1, (b / m1) % m1, dim == 3 ? b / (m1 * m1) : 0};
      double v[3], dv[3], ddv[3];
      for (int d = 0; d < 3; ++d) {
        v[d] = d < dim ? L[qi[d]][ib[d]] : 1.0;
        dv[d] = d < dim ? dL[qi[d]][ib[d]] : 0.0;
        ddv[d] = d < dim ? ddL[qi[d]][ib[d]] : 0.0;
      }
      const double N = v[0] * v[1] * v[2];
      double g[3], h[3][3];
      for (int a = 0; a < dim; ++a) {
        g[a] = 1.0;
        for (int d = 0; d < dim; ++d) g[a] *= d == a ? dv[d] : v[d];
        for (int a2 = 0; a2 < dim; ++a2) {
          h[a][a2] = 1.0;
          for (int d = 0; d < dim; ++d) h[a][a2] *= (d == a && d == a2) ? ddv[d] : ((d == a || d == a2) ? dv[d] : v[d]);
        }
      }
      for (int i = 0; i < dim; ++i) {
        const double Sb = S[b * dim + i];
        x[i] += N * Sb;
        for (int a = 0; a < dim; ++a) {
          J[i][a] += Sb * g[a];
          for (int a2 = 0; a2 < dim; ++a2) H[i][a][a2] += Sb * h[a][a2];
        }
      }
    }
    double det, JI[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
    if (dim == 2) {
      det = J[0][0] * J[1][1] - J[0][1] * J[1][0];
      JI[0][0] = J[1][1] / det;
      JI[0][1] = -J[0][1] / det;
      JI[1][0] = -J[1][0] / det;
      JI[1][1] = J[0][0] / det;
    } else {
      det = J[0][0] * (J[1][1] * J[2][2] - J[1][2] * J[2][1]) - J[0][1] * (J[1][0] * J[2][2] - J[1][2] * J[2][0]) +
            J[0][2] * (J[1][0] * J[2][1] - J[1][1] * J[2][0]);
      for (int a = 0; a < 3; ++a)
        for (int i = 0; i < 3; ++i) {  // inverse = adjugate / det: JI[a][i] = cof(J)[i][a] / det
          const int r0 = (i + 1) % 3, r1 = (i + 2) % 3, c0 = (a + 1) % 3, c1 = (a + 2) % 3;
          JI[a][i] = (J[r0][c0] * J[r1][c1] - J[r0][c1] * J[r1][c0]) / det;
        }
    }
    double G[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
    for (int a = 0; a < dim; ++a)
      for (int b = 0; b < dim; ++b)
        for (int i = 0; i < dim; ++i) G[a][b] += JI[a][i] * JI[b][i];
    double *o = out + (size_t)q * gls::kGeo;
    for (int i = 0; i < gls::kGeo; ++i) o[i] = 0.0;
    double w = 1.0;
    for (int d = 0; d < dim; ++d) w *= wq[qi[d]];
    for (int i = 0; i < dim; ++i) o[gls::kGeoX + i] = x[i];
    o[gls::kGeoJxW] = w * det;
    for (int a = 0; a < dim; ++a)
      for (int i = 0; i < dim; ++i) o[gls::kGeoJI + 3 * a + i] = JI[a][i];
    o[gls::kGeoG + 0] = G[0][0];
    o[gls::kGeoG + 1] = G[1][1];
    o[gls::kGeoG + 2] = G[2][2];
    o[gls::kGeoG + 3] = G[0][1];
    o[gls::kGeoG + 4] = G[0][2];
    o[gls::kGeoG + 5] = G[1][2];
    for (int k = 0; k < dim; ++k) {
      double cs = 0;
      for (int a = 0; a < dim; ++a)
        for (int b = 0; b < dim; ++b) cs += G[a][b] * H[k][a][b];
      o[gls::kGeoC + k] = cs;
    }
  }
}

// cell->measure() of a mapped cell from its corner support points (exact bilinear / trilinear
// volume: 2-point Gauss of the multilinear det J)
double corner_measure(int dim, int md, const double *S) {
  const int m1 = md + 1;
  double X[8][3] = {};
  for (int v = 0; v < (1 << dim); ++v) {
    const int b = (v & 1) * md + m1 * (((v >> 1) & 1) * md + (dim == 3 ? m1 * (((v >> 2) & 1) * md) : 0));
    for (int i = 0; i < dim; ++i) X[v][i] = S[b * dim + i];
  }
  const double g = 0.5 / std::sqrt(3.0), xs[2] = {0.5 - g, 0.5 + g};
  double vol = 0;
  for (int q = 0; q < (1 << dim); ++q) {
    const double xi[3] = {xs[q & 1], xs[(q >> 1) & 1], xs[(q >> 2) & 1]};
    double J[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
    for (int v = 0; v < (1 << dim); ++v)
      for (int a = 0; a < dim; ++a) {
        double gr = ((v >> a) & 1) ? 1.0 : -1.0;
        for (int b = 0; b < dim; ++b)
          if (b != a) gr *= ((v >> b) & 1) ? xi[b] : 1 - xi[b];
        for (int i = 0; i < dim; ++i) J[i][a] += gr * X[v][i];
      }
    vol += (dim == 2 ? J[0][0] * J[1][1] - J[0][1] * J[1][0]
                     : J[0][0] * (J[1][1] * J[2][2] - J[1][2] * J[2][1]) - J[0][1] * (J[1][0] * J[2][2] - J[1][2] * J[2][0]) +
                           J[0][2] * (J[1][0] * J[2][1] - J[1][1] * J[2][0])) /
           (1 << dim);
  }
  return vol;
}

int check_ctx(gls_ctx *c) {
  if (!c) return set_err(GLS_EINVAL, "null context");
  return GLS_OK;
}

// jac: parameters of the Jacobian operators (the frozen snapshot when gls_freeze_jacobian is on)
gls::OpParams make_params(gls_ctx *c, bool jac = false) {
  gls::OpParams P;
  std::memset(&P, 0, sizeof(P));
  P.n_cells = c->n_cells;
  P.n_vnodes = c->n_vnodes;
  P.n_pnodes = c->n_pnodes;
  P.n_hist = c->n_hist;
  P.cell_vnodes = c->cell_vnodes.p;
  P.cell_pnodes = c->cell_pnodes.p;
  P.geo = c->geo.p;
  P.x0 = c->x0.p;
  P.gq = c->gq.p;
  P.force_q = c->force_q.p;
  P.vmask = c->vmask.p;
  P.u = c->u;
  P.h1 = c->u1 ? c->u1 : c->u;
  P.h2 = c->u2 ? c->u2 : c->u;
  P.h3 = c->u3 ? c->u3 : c->u;
  P.nu = c->viscosity;
  for (int i = 0; i < 4; ++i) P.alpha[i] = c->alpha[i];
  P.alpha_jac = c->alpha_jac;
  P.sdt2 = c->sdt2;
  P.srf = c->srf;
  for (int i = 0; i < 3; ++i) P.omega[i] = c->omega[i];
  if (jac && c->jf.on) {
    const auto &j = c->jf;
    P.u = j.u.p;
    P.h1 = j.has[0] ? j.h[0].p : j.u.p;
    P.h2 = j.has[1] ? j.h[1].p : j.u.p;
    P.h3 = j.has[2] ? j.h[2].p : j.u.p;
    P.n_hist = j.n_hist;
    for (int i = 0; i < 4; ++i) P.alpha[i] = j.alpha[i];
    P.alpha_jac = j.alpha_jac;
    P.sdt2 = j.sdt2;
  }
  return P;
}

struct TimedLaunch {
  gls_ctx *c;
  int which;
  hipEvent_t a = nullptr, b = nullptr;
  TimedLaunch(gls_ctx *c_, int w) : c(c_), which(w) {
    if (c->timing) {
      (void)hipEventCreate(&a);
      (void)hipEventCreate(&b);
      (void)hipEventRecord(a, c->stream);
    }
  }
  ~TimedLaunch() {
    if (c->timing) {
      (void)hipEventRecord(b, c->stream);
      c->events.push_back({which, a, b});
    }
  }
};

// ---- distributed hooks (no-ops on a single rank)
int dist_import(gls_ctx *c, double *x) {
  if (!c->dist.on) return GLS_OK;
  if (c->dist.dofs) {
    HIP_TRY(gls::vec_pack_dofs(x, c->dist.send_nodes.p, c->dist.n_send, c->dist.send_buf, c->stream));
    if (c->dist.xchg(c->dist.user, 0) != 0) return set_err(GLS_ECOMM, "ghost import exchange failed");
    HIP_TRY(gls::vec_unpack_dofs(x, c->dist.recv_nodes.p, c->dist.n_recv, c->dist.recv_buf, c->stream));
    return GLS_OK;
  }
  const int64_t voff = 3 * (int64_t)c->n_vnodes;
  HIP_TRY(gls::vec_pack_nodes(x, c->dist.send_nodes.p, c->dist.n_send, voff, c->dist.send_buf, c->stream));
  if (c->dist.xchg(c->dist.user, 0) != 0) return set_err(GLS_ECOMM, "ghost import exchange failed");
  HIP_TRY(gls::vec_unpack_nodes(x, c->dist.recv_nodes.p, c->dist.n_recv, voff, c->dist.recv_buf, 0, c->stream));
  return GLS_OK;
}
// export-add order: every owned entry's incoming exchange slots in ascending slot (= neighbour) order,
// so the sums over several neighbours are deterministic
int upload_export_order(gls_ctx::Dist &D, const int32_t *send, int64_t ns) {
  std::vector<std::pair<int32_t, int32_t>> ds;
  ds.reserve((size_t)ns);
  for (int64_t j = 0; j < ns; ++j) ds.push_back({send[j], (int32_t)j});
  std::stable_sort(ds.begin(), ds.end(), [](const std::pair<int32_t, int32_t> &a, const std::pair<int32_t, int32_t> &b) {
    return a.first < b.first;
  });
  std::vector<int32_t> au, aoff{0}, aslot;
  for (size_t t = 0; t < ds.size(); ++t) {
    if (t == 0 || ds[t].first != ds[t - 1].first) {
      if (t) aoff.push_back((int32_t)aslot.size());
      au.push_back(ds[t].first);
    }
    aslot.push_back(ds[t].second);
  }
  if (!au.empty()) aoff.push_back((int32_t)aslot.size());
  GLS_TRY(D.add_u.upload(au.data(), au.size()));
  GLS_TRY(D.add_off.upload(aoff.data(), au.empty() ? 0 : aoff.size()));
  return D.add_slot.upload(aslot.data(), aslot.size());
}
int dist_export_add(gls_ctx *c, double *y) {
  if (!c->dist.on) return GLS_OK;
  if (c->dist.dofs) {
    HIP_TRY(gls::vec_pack_dofs(y, c->dist.recv_nodes.p, c->dist.n_recv, c->dist.recv_buf, c->stream));
    if (c->dist.xchg(c->dist.user, 1) != 0) return set_err(GLS_ECOMM, "ghost export exchange failed");
    HIP_TRY(gls::vec_add_dofs_ordered(y, c->dist.add_u.p, c->dist.add_off.p, c->dist.add_slot.p, (int64_t)c->dist.add_u.n,
                                      c->dist.send_buf, c->stream));
    return GLS_OK;
  }
  const int64_t voff = 3 * (int64_t)c->n_vnodes;
  HIP_TRY(gls::vec_pack_nodes(y, c->dist.recv_nodes.p, c->dist.n_recv, voff, c->dist.recv_buf, c->stream));
  if (c->dist.xchg(c->dist.user, 1) != 0) return set_err(GLS_ECOMM, "ghost export exchange failed");
  HIP_TRY(gls::vec_add_nodes_ordered(y, c->dist.add_u.p, c->dist.add_off.p, c->dist.add_slot.p, (int64_t)c->dist.add_u.n,
                                     voff, c->dist.send_buf, c->stream));
  return GLS_OK;
}
// out[k] = sum over OWNED DoFs of A[k] . w, reduced over ranks (host result)
int dist_multidot(gls_ctx *c, const double *A, int64_t lda, int nk, const double *w, double *host_out) {
  const int64_t n1 = c->dist.on ? (int64_t)c->dim * c->dist.n_owned : c->n_dofs;
  const int64_t off2 = c->dist.on ? (int64_t)c->dim * c->n_vnodes : 0;
  const int64_t n2 = c->dist.on ? c->dist.n_owned_p : 0;
  HIP_TRY(gls::vec_multidot2(A, lda, nk, w, n1, off2, n2, c->scal.p, c->work.p, c->stream));
  if (c->dist.on) {
    HIP_TRY(hipMemcpyAsync(c->dist.red_buf, c->scal.p, sizeof(double) * nk, hipMemcpyDeviceToDevice, c->stream));
    if (c->dist.allreduce(c->dist.user, c->dist.red_buf, nk) != 0) return set_err(GLS_ECOMM, "allreduce failed");
    HIP_TRY(hipMemcpyAsync(host_out, c->dist.red_buf, sizeof(double) * nk, hipMemcpyDeviceToHost, c->stream));
  } else {
    HIP_TRY(hipMemcpyAsync(host_out, c->scal.p, sizeof(double) * nk, hipMemcpyDeviceToHost, c->stream));
  }
  HIP_TRY(hipStreamSynchronize(c->stream));
  return GLS_OK;
}

// a mixed-precision smoothing level gets the FP32 copy of its linearization from the same MODE_LIN
// launch (workgroup brick kernel): no separate FP64 -> FP32 conversion pass over the linearization
int lin_f32_target(gls_ctx *c, gls::OpParams &P) {
  P.qdf = nullptr;
  if (!c->smooth_f32 || !gls::brick_fused_jacobi_supported(c->k)) return GLS_OK;
  if (c->qdata32.n != c->qdata.n) GLS_TRY(c->qdata32.alloc(c->qdata.n));
  P.qdf = c->qdata32.p;
  P.oseen = c->smooth_oseen ? 1 : 0;  // the Oseen smoother reads u and tau only: the other FP32 rows are not written
  return GLS_OK;
}

// J.v linearization (u, grad u, tau, R_s at every quadrature point), once per state
int ensure_qdata(gls_ctx *c) {
  if (c->qd_valid) return GLS_OK;
  const size_t n = gls::brick_qdata_size(c->k, c->n_cells);
  if (c->qdata.n != n) GLS_TRY(c->qdata.alloc(n));
  gls::OpParams P = make_params(c, true);
  P.qd = c->qdata.p;
  GLS_TRY(lin_f32_target(c, P));
  {
    TimedLaunch t(c, 3);
    HIP_TRY(gls::launch_brick_kernel(c->k, gls::MODE_LIN, P, c->tables, c->stream));
  }
  c->qd_valid = true;
  c->qd32_valid = P.qdf != nullptr;
  c->qd32_partial = P.qdf != nullptr && P.oseen;
  return GLS_OK;
}

// the slab node sums with an FP32 slab and / or the fused damped-Jacobi sweep / residual form
hipError_t slab_sum_ex(gls_ctx *g, const double *slab, const float *slabf, double *y, const uint8_t *vmask,
                       const double *jb, const double *jd, double omega, const double *rb, double *x0 = nullptr) {
  if (g->cube_nb1 > 0)
    return gls::brick_slab_sum_cube(g->k, g->cube_nb1, slab, slabf, g->n_vnodes, y, vmask, jb, jd, omega, g->stream, rb,
                                    x0);
  if (x0) return hipErrorInvalidValue;
  return gls::brick_slab_sum_ex(slab, slabf, g->sum_nodes.p, g->sum_off.p, g->sum_slots.p, (int64_t)g->sum_nodes.n,
                                g->n_vnodes, y, vmask, jb, jd, omega, g->stream, rb);
}
hipError_t slab_sum(gls_ctx *c, double *y) {
  if (c->cube_nb1 > 0)
    return gls::brick_slab_sum_cube(c->k, c->cube_nb1, c->slab.p, nullptr, c->n_vnodes, y, nullptr, nullptr, nullptr, 0.0,
                                    c->stream);
  return gls::brick_slab_sum(c->slab.p, c->sum_nodes.p, c->sum_off.p, c->sum_slots.p, (int64_t)c->sum_nodes.n,
                             c->n_vnodes, y, c->stream);
}

int rccl_exchange_on(gls_ctx *c, int phase, hipStream_t stream);  // RCCL transport (below)

// the brick split: a brick is a boundary brick when one of its cells holds a flagged node (ghost or
// exported); boundary bricks first, then interior ones, each in ascending (Morton) order
int build_brick_split(gls_ctx *c, const std::vector<char> &flag) {
  const int nvc = gls::ipow(c->k + 1, 3), nb = c->n_cells / 8;
  std::vector<int32_t> cv((size_t)c->n_cells * nvc);
  HIP_TRY(hipMemcpy(cv.data(), c->cell_vnodes.p, cv.size() * sizeof(int32_t), hipMemcpyDeviceToHost));
  std::vector<int32_t> bnd, inn;
  for (int b = 0; b < nb; ++b) {
    bool on = false;
    for (size_t e = (size_t)b * 8 * nvc; e < (size_t)(b + 1) * 8 * nvc && !on; ++e) on = flag[(size_t)cv[e]] != 0;
    (on ? bnd : inn).push_back(b);
  }
  c->split_bnd = (int)bnd.size();
  c->split_int = (int)inn.size();
  bnd.insert(bnd.end(), inn.begin(), inn.end());
  return c->split.upload(bnd.data(), std::max<size_t>(bnd.size(), 1));
}

// J.v launched as two brick subsets (boundary, then interior) with the ghost import between them:
// the RCCL transport imports on the exchange stream while the interior bricks run
// GLS_SPLIT_TEST=m on a single-GPU context splits at "bricks b % m == 0"
// with no exchange, for the bitwise test of the split launch; GLS_SPLIT_DIST=1 runs the same split
// launch with the callback transport (import first, then interior and boundary bricks), so the
// boundary / interior classification of a real partition is tested without an RCCL communicator
bool split_jv_enabled(gls_ctx *c) {
  if (!c->use_brick || !c->use_qdata || c->use_colors || c->hang.on || !gls::brick_subset_supported(c->k)) return false;
  if (c->dist.on)
    return c->split.p && (c->dist.comm != nullptr || std::getenv("GLS_SPLIT_DIST"));
  const char *t = std::getenv("GLS_SPLIT_TEST");
  if (!t || std::atoi(t) < 1) return false;
  if (!c->split.p) {
    const int m = std::atoi(t), nb = c->n_cells / 8;
    std::vector<int32_t> bnd, inn;
    for (int b = 0; b < nb; ++b) (b % m == 0 ? bnd : inn).push_back(b);
    c->split_bnd = (int)bnd.size();
    c->split_int = (int)inn.size();
    bnd.insert(bnd.end(), inn.begin(), inn.end());
    if (c->split.upload(bnd.data(), std::max<size_t>(bnd.size(), 1)) != GLS_OK) return false;
  }
  return true;
}

// slots of every node in the per-cell element vectors [n_cells][NV*dim + NP], ascending (cell, local
// node) order: the fixed summation order of gather_element_vectors
int ensure_element_maps(gls_ctx *c) {
  if (c->ev.p || c->n_cells == 0) return GLS_OK;
  const int dim = c->dim, nv = gls::ipow(c->k + 1, dim), np = gls::ipow(c->kp + 1, dim), el = nv * dim + np;
  std::vector<int32_t> cv((size_t)c->n_cells * nv), cp;
  HIP_TRY(hipMemcpy(cv.data(), c->cell_vnodes.p, cv.size() * sizeof(int32_t), hipMemcpyDeviceToHost));
  if (c->cell_pnodes.p) {
    cp.resize((size_t)c->n_cells * np);
    HIP_TRY(hipMemcpy(cp.data(), c->cell_pnodes.p, cp.size() * sizeof(int32_t), hipMemcpyDeviceToHost));
  }
  const std::vector<int32_t> &pn = c->cell_pnodes.p ? cp : cv;
  std::vector<int64_t> voff((size_t)c->n_vnodes + 1, 0), poff((size_t)c->n_pnodes + 1, 0);
  for (int64_t e = 0; e < (int64_t)c->n_cells * nv; ++e) ++voff[(size_t)cv[(size_t)e] + 1];
  for (int64_t e = 0; e < (int64_t)c->n_cells * np; ++e) ++poff[(size_t)pn[(size_t)e] + 1];
  for (size_t i = 1; i < voff.size(); ++i) voff[i] += voff[i - 1];
  for (size_t i = 1; i < poff.size(); ++i) poff[i] += poff[i - 1];
  std::vector<int64_t> vslot((size_t)voff.back()), pslot((size_t)poff.back());
  std::vector<int64_t> vf(voff.begin(), voff.end() - 1), pf(poff.begin(), poff.end() - 1);
  for (int64_t cell = 0; cell < c->n_cells; ++cell) {
    for (int a = 0; a < nv; ++a) vslot[(size_t)vf[(size_t)cv[(size_t)(cell * nv + a)]]++] = cell * el + (int64_t)a * dim;
    for (int a = 0; a < np; ++a) pslot[(size_t)pf[(size_t)pn[(size_t)(cell * np + a)]]++] = cell * el + (int64_t)nv * dim + a;
  }
  GLS_TRY(c->ev_voff.upload(voff.data(), voff.size()));
  GLS_TRY(c->ev_vslot.upload(vslot.data(), std::max<size_t>(vslot.size(), 1)));
  GLS_TRY(c->ev_poff.upload(poff.data(), poff.size()));
  GLS_TRY(c->ev_pslot.upload(pslot.data(), std::max<size_t>(pslot.size(), 1)));
  return c->ev.alloc((size_t)c->n_cells * el);
}

int ensure_diag(gls_ctx *c);
// the per-cell linearization cache: on for contexts that run the per-cell kernels
bool cell_cache_on(const gls_ctx *c) {
  return !c->use_brick && c->n_cells > 0;
}
size_t cell_cache_size(const gls_ctx *c) {
  const int dim = c->dim;
  return (size_t)c->n_cells * (size_t)gls::ipow(c->nq1d, dim) * (size_t)(dim + dim * dim + 1 + dim);
}

// adapted forest bricks: the pencil linearization (no output) at the current state
int oct_lin(gls_ctx *c) {
  gls::OpParams L = make_params(c, true);
  L.qd = c->qdata.p;
  L.subset = c->oct.list.p;
  L.subset_n = c->oct.nb;
  L.brick_cell0 = c->oct.cell0.p;
  HIP_TRY(gls::launch_pencil_ev(gls::MODE_LIN, L, c->tables, c->stream));
  c->qd_valid = true;
  c->qd32_valid = false;
  return GLS_OK;
}
int run_cell(gls_ctx *c, int mode, const double *v, double *y) {
  if (!c->u) return set_err(GLS_EINVAL, "gls_set_state was not called");
  if (c->n_hist > 0 && !c->u1) return set_err(GLS_EINVAL, "scheme needs solution_m1");
  if (c->n_hist > 1 && !c->u2) return set_err(GLS_EINVAL, "scheme needs solution_m2");
  if (c->n_hist > 2 && !c->u3) return set_err(GLS_EINVAL, "scheme needs solution_m3");
  // per-cell J.v from the diagonal pass's linearization cache
  const bool cq_on = cell_cache_on(c) && (mode == gls::MODE_JV || mode == gls::MODE_DIAG);
  if (cq_on) {
    const size_t need = cell_cache_size(c);
    if (c->cq.n != need) {
      GLS_TRY(c->cq.alloc(need));
      c->cq_valid = false;
    }
    if (mode == gls::MODE_JV && !c->cq_valid) {  // the diagonal pass at this state writes it
      c->diag_valid = false;
      GLS_TRY(ensure_diag(c));
    }
  }
  const bool split_jv = mode == gls::MODE_JV && split_jv_enabled(c);
  if (mode == gls::MODE_JV && !split_jv && !c->probe_local) GLS_TRY(dist_import(c, const_cast<double *>(v)));  // ghost values of v
  gls::OpParams P = make_params(c, mode != gls::MODE_RESIDUAL);
  if (mode == gls::MODE_JV && c->use_brick && c->use_qdata) {
    GLS_TRY(ensure_qdata(c));
    P.qd = c->qdata.p;
    mode = gls::MODE_JVQ;
  }
  bool lin_diag = false;  // brick path: the diagonal comes out of the linearization pass
  if (mode == gls::MODE_DIAG && c->use_brick && c->use_qdata) {
    const size_t nq = gls::brick_qdata_size(c->k, c->n_cells);
    if (c->qdata.n != nq) GLS_TRY(c->qdata.alloc(nq));
    P.qd = c->qdata.p;
    GLS_TRY(lin_f32_target(c, P));
    mode = gls::MODE_LIN;
    lin_diag = true;
  }
  if (mode == gls::MODE_JV && c->hang.on) {  // C v: hanging entries interpolated from their masters
    if (c->hang.vbuf.n != (size_t)c->n_dofs) GLS_TRY(c->hang.vbuf.alloc((size_t)c->n_dofs));
    if (c->hang.dmask.n == (size_t)c->n_dofs) {  // one pass: copy the free DoFs, interpolate the hanging ones
      HIP_TRY(gls::vec_copy_gather_set(c->hang.vbuf.p, v, c->hang.dmask.p, c->n_dofs, c->hang.dof.p, c->hang.ooff.p,
                                       c->hang.omaster.p, c->hang.ow.p, (int64_t)c->hang.dof.n, c->stream));
    } else {
      HIP_TRY(gls::vec_copy(c->hang.vbuf.p, v, c->n_dofs, c->stream));
      HIP_TRY(gls::vec_csr_gather_set(c->hang.vbuf.p, c->hang.vbuf.p, c->hang.dof.p, c->hang.ooff.p, c->hang.omaster.p,
                                      c->hang.ow.p, (int64_t)c->hang.dof.n, c->stream));
    }
    v = c->hang.vbuf.p;
  }
  P.v = v;
  P.y = y;
  P.hmask = c->hang.on ? c->hang.hmask.p : nullptr;
  const bool brick = c->use_brick && mode != gls::MODE_DIAG;
  const bool col = brick && c->use_colors;
  if (col) set_colors(c, P, y);  // every node is written exactly once: no zeroing, no slab sum
  else P.slab = brick ? brick_slab(c) : nullptr;
  if (!brick) {  // per-cell kernels: element vectors, then ordered per-node sums (no atomics)
    GLS_TRY(ensure_element_maps(c));
    P.ev = c->ev.p;
    if (cq_on) {
      P.cq = c->cq.p;
      P.cq_mode = mode == gls::MODE_DIAG ? 1 : 2;
    }
  }
  // adapted forest: the sibling-group bricks by the pencil kernel (J.v from the cached linearization; the
  // diagonal pass computes that cache), the other cells by the per-cell kernel (its cell list)
  const bool oct = c->oct.on && (mode == gls::MODE_JV || mode == gls::MODE_DIAG) && !brick;
  if (oct) {
    const size_t nq = gls::brick_qdata_size(c->k, 8 * c->oct.nb);
    if (c->qdata.n != nq) {
      GLS_TRY(c->qdata.alloc(nq));
      c->qd_valid = false;
      c->cq_valid = false;
    }
    if (mode == gls::MODE_JV && !c->qd_valid) GLS_TRY(oct_lin(c));  // linearization only, current state
    if (mode == gls::MODE_JV && c->oct.f32_next && !c->qd32_valid) {
      if (c->qdata32.n != c->qdata.n) GLS_TRY(c->qdata32.alloc(c->qdata.n));
      HIP_TRY(gls::vec_to_f32(c->qdata.p, c->qdata32.p, (int64_t)c->qdata.n, c->stream));
      c->qd32_valid = true;
    }
    P.cell_list = c->oct.rest.p;  // the per-cell kernel runs the cells outside the bricks only
    P.cell_list_n = c->oct.n_rest;
  }
  if (!col && !P.slab && !P.ev) HIP_TRY(hipMemsetAsync(y, 0, sizeof(double) * c->n_dofs, c->stream));
  {
    TimedLaunch t(c, mode == gls::MODE_JVQ ? (int)gls::MODE_JV : (lin_diag ? (int)gls::MODE_DIAG : mode));
    if (brick && split_jv && mode == gls::MODE_JVQ) {
      auto &D = c->dist;
      double *vv = const_cast<double *>(v);
      const int64_t voff = 3 * (int64_t)c->n_vnodes;
      if (D.on && !D.comm) {  // callback transport (GLS_SPLIT_DIST): the import completes first
        GLS_TRY(dist_import(c, vv));
      } else if (D.on) {  // ghost import of v on the exchange stream, ordered after v's producer
        HIP_TRY(hipEventRecord(D.ev_ready, c->stream));
        HIP_TRY(hipStreamWaitEvent(D.xstream, D.ev_ready, 0));
        HIP_TRY(gls::vec_pack_nodes(vv, D.send_nodes.p, D.n_send, voff, D.send_buf, D.xstream));
        if (rccl_exchange_on(c, 0, D.xstream) != 0) return set_err(GLS_ECOMM, "ghost import exchange failed");
        HIP_TRY(gls::vec_unpack_nodes(vv, D.recv_nodes.p, D.n_recv, voff, D.recv_buf, 0, D.xstream));
        HIP_TRY(hipEventRecord(D.ev_done, D.xstream));
      }
      gls::OpParams Q = P;  // interior bricks read no ghost value
      Q.subset = c->split.p + c->split_bnd;
      Q.subset_n = c->split_int;
      if (Q.subset_n > 0) HIP_TRY(gls::launch_brick_kernel(c->k, mode, Q, c->tables, c->stream));
      if (D.on && D.comm) HIP_TRY(hipStreamWaitEvent(c->stream, D.ev_done, 0));
      Q.subset = c->split.p;
      Q.subset_n = c->split_bnd;
      if (Q.subset_n > 0) HIP_TRY(gls::launch_brick_kernel(c->k, mode, Q, c->tables, c->stream));
    } else if (brick) {
      HIP_TRY(gls::launch_brick_kernel(c->k, mode, P, c->tables, c->stream));
    } else {
      // (the bricks' pencil launch forked onto a side stream, concurrent with this one and joined before the
      // gather, measured 1.0-1.4 ms per Newton step SLOWER on the 1.28 M-DoF octree line: the cross-stream event
      // pair costs more than the overlap of two ~20 us launches gains; profiles/r05_ab_octree_overlap.txt)
      HIP_TRY(gls::launch_cell_kernel(c->dim, c->k, c->kp, c->nq1d, mode, P, c->tables, c->stream));
      if (oct) {  // the bricks' cells: element vectors from the pencil kernel
        gls::OpParams Q = P;
        Q.cell_list = nullptr;
        Q.cell_list_n = 0;
        Q.y = nullptr;  // element vectors only
        Q.qd = c->qdata.p;
        Q.subset = c->oct.list.p;
        Q.subset_n = c->oct.nb;
        Q.brick_cell0 = c->oct.cell0.p;
        const bool f32 = mode == gls::MODE_JV && c->oct.f32_next;
        if (f32) Q.qdf = c->qdata32.p;
        HIP_TRY(gls::launch_pencil_ev(mode == gls::MODE_JV ? gls::MODE_JVQ : gls::MODE_LIN, Q, c->tables, c->stream, f32));
        if (mode == gls::MODE_DIAG) {
          c->qd_valid = true;
          c->qd32_valid = false;
        }
      }
    }
  }
  if (P.ev)
    HIP_TRY(gls::gather_element_vectors(y, c->ev.p, c->ev_voff.p, c->ev_vslot.p, c->n_vnodes, c->ev_poff.p,
                                        c->ev_pslot.p, c->n_pnodes, c->dim, c->stream));
  if (brick && !col && P.slab) {
    TimedLaunch t(c, 5);
    HIP_TRY(slab_sum(c, y));
  }
  // C^T y: the local cells' hanging rows onto their masters (masters across the partition are local
  // ghosts), then the ghost contributions to their owners (compress(add)); condensing the partial
  // rows before the export equals condensing the summed rows after it. (Folding this pass into the
  // element-vector gather measured slower on the 1.28 M-DoF octree line both ways: each master re-summing
  // its hanging rows' slots through their node maps +6.6 ms per Newton step, flattened (slot, weight) lists
  // per master DoF +1.6 ms -- the gather is bound by its dependent load chain, which either form lengthens;
  // profiles/r05_ab_cell_cache_fold.txt, r05_ab_condense_fold2.txt.)
  if (c->hang.on && (mode == gls::MODE_RESIDUAL || mode == gls::MODE_JV))
    HIP_TRY(gls::vec_csr_condense(y, c->hang.tm.p, c->hang.toff.p, c->hang.tdof.p, c->hang.tw.p,
                                  (int64_t)c->hang.tm.n, c->stream));
  if (!c->probe_local) GLS_TRY(dist_export_add(c, y));
  if (P.cq_mode == 1) c->cq_valid = true;
  if (lin_diag) {  // the same launch stored the J.v linearization
    c->qd_valid = true;
    c->qd32_valid = P.qdf != nullptr;
    c->qd32_partial = P.qdf != nullptr && P.oseen;
  }
  return GLS_OK;
}

int ensure_diag(gls_ctx *c) {
  if (c->diag_valid) return GLS_OK;
  GLS_TRY(run_cell(c, gls::MODE_DIAG, nullptr, c->diag.p));
  if (c->dist.on) {  // ghost rows are not owned here: keep the Jacobi division finite
    const int64_t d = c->dim, nl = c->n_vnodes, no = c->dist.n_owned, npl = c->n_dofs - d * nl, nop = c->dist.n_owned_p;
    HIP_TRY(gls::vec_fill(c->diag.p + d * no, d * (nl - no), 1.0, c->stream));
    HIP_TRY(gls::vec_fill(c->diag.p + d * nl + nop, npl - nop, 1.0, c->stream));
  }
  c->diag_valid = true;
  return GLS_OK;
}

int device_dot(gls_ctx *c, const double *a, const double *b, double *host_out) {
  return dist_multidot(c, a, 0, 1, b, host_out);
}

// Stream-ordered variants for GMRES (no host wait): the dots land in `out` (device), are reduced over
// ranks, and are copied to the pinned host buffer `hp` (read after the caller's next wait). The return
// value is the device address of the reduced dots, which the next projection reads as its
// coefficients directly (no host round trip, no H2D copy).
const double *reduce_dots_async(gls_ctx *c, const double *out, int nd, double *hp, int *err) {
  const double *res = out;
  *err = GLS_OK;
  if (c->dist.on) {
    if (hipMemcpyAsync(c->dist.red_buf, out, sizeof(double) * nd, hipMemcpyDeviceToDevice, c->stream) != hipSuccess) {
      *err = set_err(GLS_EHIP, "reduce_dots_async: D2D copy");
      return nullptr;
    }
    if (c->dist.allreduce(c->dist.user, c->dist.red_buf, nd) != 0) {
      *err = set_err(GLS_ECOMM, "allreduce failed");
      return nullptr;
    }
    res = c->dist.red_buf;
  }
  if (hipMemcpyAsync(hp, res, sizeof(double) * nd, hipMemcpyDeviceToHost, c->stream) != hipSuccess) {
    *err = set_err(GLS_EHIP, "reduce_dots_async: D2H copy");
    return nullptr;
  }
  return res;
}
int multidot_async(gls_ctx *c, const double *A, int64_t lda, int nk, const double *w, double *out, double *hp,
                   const double **dev_res) {
  const int64_t n1 = c->dist.on ? (int64_t)c->dim * c->dist.n_owned : c->n_dofs;
  const int64_t off2 = c->dist.on ? (int64_t)c->dim * c->n_vnodes : 0;
  const int64_t n2 = c->dist.on ? c->dist.n_owned_p : 0;
  HIP_TRY(gls::vec_multidot2(A, lda, nk, w, n1, off2, n2, out, c->work.p, c->stream));
  int err;
  *dev_res = reduce_dots_async(c, out, nk, hp, &err);
  return err;
}
int multiaxpy_dots_async(gls_ctx *c, double *w, const double *V, int64_t lda, int nk, const double *h, bool dots,
                         double *out, double *hp, const double **dev_res, double scale = 1.0) {
  const int64_t n1 = c->dist.on ? (int64_t)c->dim * c->dist.n_owned : c->n_dofs;
  const int64_t off2 = c->dist.on ? (int64_t)c->dim * c->n_vnodes : 0;
  const int64_t n2 = c->dist.on ? c->dist.n_owned_p : 0;
  HIP_TRY(gls::vec_multiaxpy_dots(w, V, lda, nk, h, 1.0, c->n_dofs, n1, off2, n2, dots, scale, out, c->work.p,
                                  c->stream));
  int err;
  *dev_res = reduce_dots_async(c, out, dots ? nk + 1 : 1, hp, &err);
  return err;
}

}  // namespace

extern "C" {

int gls_create(const gls_mesh_desc *d, gls_ctx **out) {
  if (!d || !out) return set_err(GLS_EINVAL, "null argument");
  *out = nullptr;
  const int nq1d = d->nq1d > 0 ? d->nq1d : d->k + 1;
  if (d->dim != 2 && d->dim != 3) return set_err(GLS_EINVAL, "dim must be 2 or 3");
  if (!gls::cell_kernel_supported(d->dim, d->k, d->kp, nq1d))
    return set_err(GLS_EINVAL, "unsupported element Q%d-Q%d (dim %d, QGauss %d)", d->k, d->kp, d->dim, nq1d);
  const bool mapped = d->map_degree > 0;
  if (d->n_cells < 0 || d->n_vnodes <= 0 || d->n_pnodes <= 0 || !d->cell_vnodes || (!mapped && !d->cell_h))
    return set_err(GLS_EINVAL, "incomplete mesh description");
  if (mapped && (d->map_degree > 2 || !d->cell_support))
    return set_err(GLS_EINVAL, "mapped cells: map_degree 1 or 2 with cell_support");
  if (d->kp != d->k && !d->cell_pnodes) return set_err(GLS_EINVAL, "cell_pnodes required when kp != k");
  if (d->srf && !d->cell_x0 && !mapped) return set_err(GLS_EINVAL, "srf requires cell_x0");
  std::unique_ptr<gls_ctx> c(new gls_ctx);
  c->dim = d->dim;
  c->k = d->k;
  c->kp = d->kp;
  c->nq1d = nq1d;
  c->n_cells = d->n_cells;
  c->n_vnodes = d->n_vnodes;
  c->n_pnodes = d->n_pnodes;
  c->nq = gls::ipow(nq1d, d->dim);
  c->n_dofs = (int64_t)d->dim * d->n_vnodes + d->n_pnodes;
  c->viscosity = d->viscosity;
  c->srf = d->srf;
  for (int i = 0; i < 3; ++i) c->omega[i] = d->omega[i];
  c->tables = make_tables(d->k, d->kp, nq1d);
  const int nv = gls::ipow(d->k + 1, d->dim), np = gls::ipow(d->kp + 1, d->dim);
  // validate indices
  for (int64_t i = 0; i < (int64_t)d->n_cells * nv; ++i)
    if (d->cell_vnodes[i] < 0 || d->cell_vnodes[i] >= d->n_vnodes) return set_err(GLS_EINVAL, "cell_vnodes out of range");
  if (d->cell_pnodes)
    for (int64_t i = 0; i < (int64_t)d->n_cells * np; ++i)
      if (d->cell_pnodes[i] < 0 || d->cell_pnodes[i] >= d->n_pnodes) return set_err(GLS_EINVAL, "cell_pnodes out of range");
  if (!d->cell_pnodes && d->n_pnodes != d->n_vnodes) return set_err(GLS_EINVAL, "n_pnodes != n_vnodes without cell_pnodes");

  GLS_TRY(c->cell_vnodes.upload(d->cell_vnodes, (size_t)d->n_cells * nv));
  c->use_brick = !mapped && detect_bricks(d, nq1d);
  if (c->use_brick) GLS_TRY(build_slab_map(c.get(), d));
  if (const char *e = std::getenv("GLS_JV_RECOMPUTE")) c->use_qdata = std::atoi(e) == 0;
  if (d->cell_pnodes) GLS_TRY(c->cell_pnodes.upload(d->cell_pnodes, (size_t)d->n_cells * np));
  std::vector<double> geo((size_t)d->n_cells * 4);
  const int nsup = mapped ? gls::ipow(d->map_degree + 1, d->dim) : 0;
  for (int cix = 0; cix < d->n_cells; ++cix) {
    double meas = 1.;
    if (mapped) {
      meas = corner_measure(d->dim, d->map_degree, d->cell_support + (size_t)cix * nsup * d->dim);
      if (!(meas > 0)) return set_err(GLS_EINVAL, "cell %d: non-positive measure (inverted cell)", cix);
      geo[cix * 4 + 0] = geo[cix * 4 + 1] = geo[cix * 4 + 2] = 1.0;
    } else {
      for (int e = 0; e < d->dim; ++e) {
        geo[cix * 4 + e] = d->cell_h[(size_t)cix * d->dim + e];
        meas *= geo[cix * 4 + e];
      }
      if (d->dim == 2) geo[cix * 4 + 2] = 1.0;
    }
    // element size for tau (gls_navier_stokes.cc:340-345)
    geo[cix * 4 + 3] = d->dim == 2 ? std::sqrt(4. * meas / M_PI) / d->k : std::pow(6 * meas / M_PI, 1. / 3.) / d->k;
  }
  GLS_TRY(c->geo.upload(geo.data(), geo.size()));
  if (mapped) {  // FEValues geometry per quadrature point (MappingQ(map_degree))
    c->map_degree = d->map_degree;
    c->host_support.assign(d->cell_support, d->cell_support + (size_t)d->n_cells * nsup * d->dim);
    std::vector<double> gq((size_t)d->n_cells * c->nq * gls::kGeo);
    for (int cix = 0; cix < d->n_cells; ++cix) {
      mapped_geometry(d->dim, d->map_degree, nq1d, d->cell_support + (size_t)cix * nsup * d->dim,
                      gq.data() + (size_t)cix * c->nq * gls::kGeo);
      for (int q = 0; q < c->nq; ++q)
        if (!(gq[((size_t)cix * c->nq + q) * gls::kGeo + gls::kGeoJxW] > 0))
          return set_err(GLS_EINVAL, "cell %d: non-positive Jacobian at quadrature point %d", cix, q);
    }
    GLS_TRY(c->gq.upload(gq.data(), gq.size()));
  } else {
    c->host_h.assign(d->cell_h, d->cell_h + (size_t)d->n_cells * d->dim);
    if (d->cell_x0) c->host_x0.assign(d->cell_x0, d->cell_x0 + (size_t)d->n_cells * d->dim);
  }
  if (d->cell_x0) {
    std::vector<double> x0((size_t)d->n_cells * 3, 0.);
    for (int cix = 0; cix < d->n_cells; ++cix)
      for (int e = 0; e < d->dim; ++e) x0[cix * 3 + e] = d->cell_x0[(size_t)cix * d->dim + e];
    GLS_TRY(c->x0.upload(x0.data(), x0.size()));
  }
  if (d->force_q) GLS_TRY(c->force_q.upload(d->force_q, (size_t)d->n_cells * c->nq * d->dim));
  std::vector<int64_t> con;
  if (d->vnode_mask) {
    GLS_TRY(c->vmask.upload(d->vnode_mask, (size_t)d->n_vnodes));
    for (int64_t n = 0; n < d->n_vnodes; ++n)
      for (int e = 0; e < d->dim; ++e)
        if ((d->vnode_mask[n] >> e) & 1) con.push_back(n * d->dim + e);
  }
  GLS_TRY(c->con_dofs.upload(con.data(), con.size()));
  GLS_TRY(c->diag.alloc(c->n_dofs));
  GLS_TRY(c->work.alloc(gls::multidot_work_size()));
  GLS_TRY(c->scal.alloc(64));
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess)
    return set_err(GLS_EHIP, "stream create failed");
  c->own_stream = true;
  HIP_TRY(hipDeviceSynchronize());
  *out = c.release();
  return GLS_OK;
}

int gls_destroy(gls_ctx *c) {
  if (!c) return GLS_OK;
  (void)hipStreamSynchronize(c->stream);
  delete c;
  return GLS_OK;
}

int gls_set_stream(gls_ctx *c, void *s) {
  GLS_TRY(check_ctx(c));
  if (c->own_stream && c->stream) {
    (void)hipStreamSynchronize(c->stream);
    (void)hipStreamDestroy(c->stream);
  }
  c->own_stream = false;
  c->stream = (hipStream_t)s;
  // multigrid levels run on the fine level's stream (the V-cycle interleaves their kernels)
  if (c->mg.on) {
    for (size_t l = 1; l < c->mg.lev.size(); ++l) GLS_TRY(gls_set_stream(c->mg.lev[l], s));
    // the replica's V-cycle is ordered with replica_gather / vec_pack_dofs on this stream
    if (c->mg.replica) GLS_TRY(gls_set_stream(c->mg.replica, s));
    if (c->mg.rep2) GLS_TRY(gls_set_stream(c->mg.rep2, s));
  }
  return GLS_OK;
}

int gls_uses_brick_kernels(const gls_ctx *c) { return c && c->use_brick ? 1 : 0; }

int gls_quadrature_points(const gls_ctx *c, double *xq) {
  if (!c || !xq) return set_err(GLS_EINVAL, "null argument");
  const int dim = c->dim, nq = c->nq;
  if (c->map_degree > 0) {
    const int nsup = gls::ipow(c->map_degree + 1, dim);
    std::vector<double> g((size_t)nq * gls::kGeo);
    for (int cix = 0; cix < c->n_cells; ++cix) {
      mapped_geometry(dim, c->map_degree, c->nq1d, c->host_support.data() + (size_t)cix * nsup * dim, g.data());
      for (int q = 0; q < nq; ++q)
        for (int e = 0; e < dim; ++e) xq[((size_t)cix * nq + q) * dim + e] = g[(size_t)q * gls::kGeo + gls::kGeoX + e];
    }
    return GLS_OK;
  }
  if (c->host_x0.empty()) return set_err(GLS_EINVAL, "gls_quadrature_points: the mesh was created without cell_x0");
  for (int cix = 0; cix < c->n_cells; ++cix)
    for (int q = 0; q < nq; ++q) {
      const int qi[3] = {q % c->nq1d, (q / c->nq1d) % c->nq1d, q / (c->nq1d * c->nq1d)};
      for (int e = 0; e < dim; ++e)
        xq[((size_t)cix * nq + q) * dim + e] =
            c->host_x0[(size_t)cix * dim + e] + c->host_h[(size_t)cix * dim + e] * c->tables.xi[qi[e]];
    }
  return GLS_OK;
}

int gls_n_dofs(const gls_ctx *c, int64_t *n) {
  if (!c || !n) return set_err(GLS_EINVAL, "null argument");
  *n = c->n_dofs;
  return GLS_OK;
}

int gls_set_force(gls_ctx *c, const double *f) {
  GLS_TRY(check_ctx(c));
  HIP_TRY(hipStreamSynchronize(c->stream));
  if (!f) {
    c->force_q.release();
  } else {
    GLS_TRY(c->force_q.upload(f, (size_t)c->n_cells * c->nq * c->dim));
  }
  c->diag_valid = false;
  c->ilu.valid = false;
  c->qd_valid = false;
  c->cq_valid = false;
  return GLS_OK;
}

int gls_set_viscosity(gls_ctx *c, double nu) {
  GLS_TRY(check_ctx(c));
  c->viscosity = nu;
  c->diag_valid = false;
  c->ilu.valid = false;
  c->qd_valid = false;
  c->cq_valid = false;
  return GLS_OK;
}

// assembleGLS preamble: gls_navier_stokes.cc:295-329 and the scheme branches :477-516, :530-533
int gls_set_time(gls_ctx *c, int scheme, const double ts[4]) {
  GLS_TRY(check_ctx(c));
  if (scheme < GLS_STEADY || scheme > GLS_SDIRK3_3) return set_err(GLS_EINVAL, "scheme %d", scheme);
  if (scheme != GLS_STEADY && (!ts || ts[0] == 0.)) return set_err(GLS_EINVAL, "time steps required");
  c->scheme = scheme;
  if (ts)
    for (int i = 0; i < 4; ++i) c->time_steps[i] = ts[i];
  if (!c->jf.on) c->mg.dirty = true;
  for (double &a : c->alpha) a = 0.;
  c->alpha_jac = 0.;
  c->sdt2 = 0.;
  c->n_hist = 0;
  if (scheme != GLS_STEADY) {
    const double sdt = 1. / ts[0];
    c->sdt2 = sdt * sdt;
  }
  if (scheme == GLS_BDF1 || scheme == GLS_BDF2 || scheme == GLS_BDF3) {
    const int order = scheme - GLS_BDF1 + 1;
    double a[6];
    GLS_TRY(gls_bdf_coefficients(order, ts, 4, a));
    for (int i = 0; i <= order; ++i) c->alpha[i] = a[i];
    c->alpha_jac = a[0];
    c->n_hist = order;
  } else if (is_sdirk(scheme)) {
    const bool three = scheme == GLS_SDIRK3 || scheme == GLS_SDIRK3_1 || scheme == GLS_SDIRK3_2 || scheme == GLS_SDIRK3_3;
    const int order = three ? 3 : 2;
    double t[12];
    GLS_TRY(gls_sdirk_coefficients(order, ts[0], t));
    int stage = 0;  // sdirk2 / sdirk3 (no stage) contribute no time term, like the reference
    if (scheme == GLS_SDIRK2_1 || scheme == GLS_SDIRK3_1) stage = 1;
    if (scheme == GLS_SDIRK2_2 || scheme == GLS_SDIRK3_2) stage = 2;
    if (scheme == GLS_SDIRK3_3) stage = 3;
    c->alpha_jac = t[0];
    if (stage > 0) {
      for (int i = 0; i <= stage; ++i) c->alpha[i] = t[(stage - 1) * (order + 1) + i];
      c->n_hist = stage;
    }
  }
  if (!c->jf.on) {  // a frozen Jacobian keeps its own time coefficients
    c->diag_valid = false;
    c->ilu.valid = false;
    c->qd_valid = false;
    c->cq_valid = false;
  }
  return GLS_OK;
}

int gls_set_state(gls_ctx *c, const double *u, const double *u1, const double *u2, const double *u3) {
  GLS_TRY(check_ctx(c));
  if (!u) return set_err(GLS_EINVAL, "u is null");
  c->u = u;
  c->u1 = u1;
  c->u2 = u2;
  c->u3 = u3;
  if (!c->jf.on) {  // a frozen Jacobian stays at its snapshot (gls_freeze_jacobian)
    c->diag_valid = false;
    c->ilu.valid = false;
    c->qd_valid = false;
    c->cq_valid = false;
    c->mg.dirty = true;
  }
  // distributed: refresh the ghost values of the evaluation point (history vectors are imported
  // by the caller once per time step with gls_dist_import)
  return dist_import(c, const_cast<double *>(u));
}

// Jacobian snapshot for skip_newton (skip_newton_non_linear_solver.h:66-70, 126-130): freeze = 1
// copies the current state vectors and time coefficients; the Jacobian operators (J.v, diagonal,
// linearization, multigrid levels) stay at that snapshot while later gls_set_state / gls_set_time
// calls move only the residual. freeze = 0 releases it (everything is re-derived lazily).
int gls_freeze_jacobian(gls_ctx *c, int freeze) {
  GLS_TRY(check_ctx(c));
  auto &j = c->jf;
  if (!freeze) {
    if (j.on) {
      j.on = false;
      c->diag_valid = false;
      c->ilu.valid = false;
      c->qd_valid = false;
      c->cq_valid = false;
      c->mg.dirty = true;
    }
    return GLS_OK;
  }
  if (!c->u) return set_err(GLS_EINVAL, "gls_freeze_jacobian: gls_set_state was not called");
  if (j.on) return GLS_OK;  // already frozen at its snapshot
  const size_t n = (size_t)c->n_dofs;
  if (j.u.n != n) GLS_TRY(j.u.alloc(n));
  HIP_TRY(hipMemcpyAsync(j.u.p, c->u, sizeof(double) * n, hipMemcpyDeviceToDevice, c->stream));
  const double *hs[3] = {c->u1, c->u2, c->u3};
  for (int h = 0; h < 3; ++h) {
    j.has[h] = hs[h] != nullptr && h < c->n_hist;
    if (!j.has[h]) continue;
    if (j.h[h].n != n) GLS_TRY(j.h[h].alloc(n));
    HIP_TRY(hipMemcpyAsync(j.h[h].p, hs[h], sizeof(double) * n, hipMemcpyDeviceToDevice, c->stream));
  }
  for (int i = 0; i < 4; ++i) {
    j.alpha[i] = c->alpha[i];
    j.ts[i] = c->time_steps[i];
  }
  j.alpha_jac = c->alpha_jac;
  j.sdt2 = c->sdt2;
  j.n_hist = c->n_hist;
  j.scheme = c->scheme;
  j.on = true;  // diag / linearization / multigrid computed so far belong to this very state
  return GLS_OK;
}

int gls_dist_import(gls_ctx *c, double *x) {
  GLS_TRY(check_ctx(c));
  return dist_import(c, x);
}

int gls_dist_attach(gls_ctx *c, int64_t n_owned_nodes, int n_nbrs, const int64_t *send_offsets,
                    const int32_t *send_nodes, const int64_t *recv_offsets, const int32_t *recv_nodes, double *send_buf,
                    double *recv_buf, double *red_buf, gls_exchange_fn xchg, gls_allreduce_fn allreduce, void *user) {
  GLS_TRY(check_ctx(c));
  if (c->dim != 3 || c->k != c->kp || c->cell_pnodes.p) return set_err(GLS_EINVAL, "distributed path: 3D Qk-Qk only");
  if (n_owned_nodes < 0 || n_owned_nodes > c->n_vnodes || n_nbrs < 0 || !xchg || !allreduce || !red_buf)
    return set_err(GLS_EINVAL, "gls_dist_attach: bad arguments");
  const int64_t ns = n_nbrs ? send_offsets[n_nbrs] : 0, nr = n_nbrs ? recv_offsets[n_nbrs] : 0;
  for (int64_t i = 0; i < ns; ++i)
    if (send_nodes[i] < 0 || send_nodes[i] >= n_owned_nodes) return set_err(GLS_EINVAL, "send node not owned");
  for (int64_t i = 0; i < nr; ++i)
    if (recv_nodes[i] < n_owned_nodes || recv_nodes[i] >= c->n_vnodes) return set_err(GLS_EINVAL, "recv node not a ghost");
  if ((ns && !send_buf) || (nr && !recv_buf)) return set_err(GLS_EINVAL, "exchange buffers missing");
  GLS_TRY(upload_export_order(c->dist, send_nodes, ns));
  GLS_TRY(c->dist.send_nodes.upload(send_nodes, (size_t)ns));
  GLS_TRY(c->dist.recv_nodes.upload(recv_nodes, (size_t)nr));
  c->dist.n_owned = n_owned_nodes;
  c->dist.n_owned_p = n_owned_nodes;
  c->dist.dofs = false;
  c->dist.width = 4;
  c->dist.n_send = ns;
  c->dist.n_recv = nr;
  c->dist.send_buf = send_buf;
  c->dist.recv_buf = recv_buf;
  c->dist.red_buf = red_buf;
  c->dist.xchg = xchg;
  c->dist.allreduce = allreduce;
  c->dist.user = user;
  c->dist.on = true;
  c->diag_valid = false;
  c->ilu.valid = false;
  c->qd_valid = false;
  c->cq_valid = false;
  if (c->use_brick && gls::brick_subset_supported(c->k)) {  // boundary / interior bricks (overlapped J.v)
    std::vector<char> flag((size_t)c->n_vnodes, 0);
    for (int64_t i = 0; i < ns; ++i) flag[(size_t)send_nodes[i]] = 1;
    for (int64_t i = 0; i < nr; ++i) flag[(size_t)recv_nodes[i]] = 1;
    GLS_TRY(build_brick_split(c, flag));
  }
  return GLS_OK;
}

int gls_dist_attach_dofs(gls_ctx *c, int64_t n_owned_vnodes, int64_t n_owned_pnodes, int n_nbrs,
                         const int64_t *send_offsets, const int32_t *send_dofs, const int64_t *recv_offsets,
                         const int32_t *recv_dofs, double *send_buf, double *recv_buf, double *red_buf,
                         gls_exchange_fn xchg, gls_allreduce_fn allreduce, void *user) {
  GLS_TRY(check_ctx(c));
  const int64_t nvd = (int64_t)c->dim * c->n_vnodes, npn = c->n_dofs - nvd;
  if (n_owned_vnodes < 0 || n_owned_vnodes > c->n_vnodes || n_owned_pnodes < 0 || n_owned_pnodes > npn || n_nbrs < 0 ||
      !xchg || !allreduce || !red_buf)
    return set_err(GLS_EINVAL, "gls_dist_attach_dofs: bad arguments");
  if (c->mg.on) return set_err(GLS_EINVAL, "gls_dist_attach_dofs: no multigrid");
  const int64_t ns = n_nbrs ? send_offsets[n_nbrs] : 0, nr = n_nbrs ? recv_offsets[n_nbrs] : 0;
  auto owned = [&](int64_t d) { return d < nvd ? d / c->dim < n_owned_vnodes : d - nvd < n_owned_pnodes; };
  for (int64_t i = 0; i < ns; ++i)
    if (send_dofs[i] < 0 || send_dofs[i] >= c->n_dofs || !owned(send_dofs[i])) return set_err(GLS_EINVAL, "send DoF not owned");
  for (int64_t i = 0; i < nr; ++i)
    if (recv_dofs[i] < 0 || recv_dofs[i] >= c->n_dofs || owned(recv_dofs[i])) return set_err(GLS_EINVAL, "recv DoF not a ghost");
  if ((ns && !send_buf) || (nr && !recv_buf)) return set_err(GLS_EINVAL, "exchange buffers missing");
  auto &D = c->dist;
  GLS_TRY(upload_export_order(D, send_dofs, ns));
  GLS_TRY(D.send_nodes.upload(send_dofs, (size_t)ns));
  GLS_TRY(D.recv_nodes.upload(recv_dofs, (size_t)nr));
  D.h_send.assign(send_dofs, send_dofs + ns);
  D.h_recv.assign(recv_dofs, recv_dofs + nr);
  D.h_soff.assign(1, 0);
  D.h_roff.assign(1, 0);
  if (n_nbrs > 0) {
    D.h_soff.assign(send_offsets, send_offsets + n_nbrs + 1);
    D.h_roff.assign(recv_offsets, recv_offsets + n_nbrs + 1);
  }
  D.dofs = true;
  D.width = 1;
  D.n_owned = n_owned_vnodes;
  D.n_owned_p = n_owned_pnodes;
  D.n_send = ns;
  D.n_recv = nr;
  D.send_buf = send_buf;
  D.recv_buf = recv_buf;
  D.red_buf = red_buf;
  D.xchg = xchg;
  D.allreduce = allreduce;
  D.user = user;
  D.on = true;
  c->diag_valid = false;
  c->ilu.valid = false;
  c->qd_valid = false;
  c->cq_valid = false;
  return GLS_OK;
}

int gls_residual(gls_ctx *c, double *rhs) {
  GLS_TRY(check_ctx(c));
  if (!rhs) return set_err(GLS_EINVAL, "rhs is null");
  GLS_TRY(run_cell(c, gls::MODE_RESIDUAL, nullptr, rhs));
  HIP_TRY(gls::vec_set_indexed(rhs, c->con_dofs.p, nullptr, (int64_t)c->con_dofs.n, c->stream));
  return GLS_OK;
}

// assemble_matrix_and_rhs (gls_navier_stokes.cc:917-1000: assembleGLS<true>, the matrix and the rhs in
// one cell loop): on
// the Q2 brick path one pencil launch (MODE_RESLIN) computes the residual, the J.v linearization and
// the Jacobian diagonal at the current state (the residual's and the diagonal's node sums are bitwise
// those of the separate launches); elsewhere -- and with a frozen Jacobian, hanging nodes, colored or
// distributed launches, GLS_NO_RESLIN=1 -- the residual and the diagonal separately
int gls_residual_and_diagonal(gls_ctx *c, double *rhs, double *d) {
  GLS_TRY(check_ctx(c));
  if (!rhs) return set_err(GLS_EINVAL, "rhs is null");
  if (!c->u) return set_err(GLS_EINVAL, "gls_set_state was not called");
  if (c->n_hist > 0 && !c->u1) return set_err(GLS_EINVAL, "scheme needs solution_m1");
  if (c->n_hist > 1 && !c->u2) return set_err(GLS_EINVAL, "scheme needs solution_m2");
  if (c->n_hist > 2 && !c->u3) return set_err(GLS_EINVAL, "scheme needs solution_m3");
  const bool fuse = !c->diag_valid && c->use_brick && c->use_qdata && c->use_slab && !c->use_colors && !c->hang.on &&
                    !c->dist.on && !c->jf.on && c->k == 2 && c->cube_nb1 > 0 && gls::pencil_enabled() &&
                    std::getenv("GLS_NO_RESLIN") == nullptr;
  if (fuse) {
    const size_t nq = gls::brick_qdata_size(c->k, c->n_cells);
    if (c->qdata.n != nq) GLS_TRY(c->qdata.alloc(nq));
    double *slab = brick_slab(c);
    if (!slab) return set_err(GLS_ENOMEM, "slab allocation failed");
    if (c->slab2.n != c->slab.n) GLS_TRY(c->slab2.alloc(c->slab.n));
    gls::OpParams P = make_params(c, true);
    P.qd = c->qdata.p;
    GLS_TRY(lin_f32_target(c, P));
    P.y = c->diag.p;
    P.slab = slab;
    P.res_y = rhs;
    P.res_slab = c->slab2.p;
    {
      TimedLaunch t(c, gls::MODE_DIAG);
      HIP_TRY(gls::launch_pencil_reslin(P, c->tables, c->stream));
    }
    {
      TimedLaunch t(c, 5);
      HIP_TRY(slab_sum_ex(c, c->slab2.p, nullptr, rhs, nullptr, nullptr, nullptr, 0.0, nullptr));
    }
    {
      TimedLaunch t(c, 5);
      HIP_TRY(slab_sum(c, c->diag.p));
    }
    HIP_TRY(gls::vec_set_indexed(rhs, c->con_dofs.p, nullptr, (int64_t)c->con_dofs.n, c->stream));
    c->qd_valid = true;
    c->qd32_valid = P.qdf != nullptr;
  c->qd32_partial = P.qdf != nullptr && P.oseen;
    c->diag_valid = true;
  } else {
    GLS_TRY(gls_residual(c, rhs));
    GLS_TRY(ensure_diag(c));
  }
  if (d && d != c->diag.p) HIP_TRY(gls::vec_copy(d, c->diag.p, c->n_dofs, c->stream));
  return GLS_OK;
}

int gls_jacobian_diagonal(gls_ctx *c, double *d) {
  GLS_TRY(check_ctx(c));
  GLS_TRY(ensure_diag(c));
  if (d && d != c->diag.p) HIP_TRY(gls::vec_copy(d, c->diag.p, c->n_dofs, c->stream));
  return GLS_OK;
}

int gls_jacobian_apply(gls_ctx *c, const double *v, double *y) {
  GLS_TRY(check_ctx(c));
  if (!v || !y || v == y) return set_err(GLS_EINVAL, "v/y null or aliased");
  if (c->con_dofs.n || c->dist.on) GLS_TRY(ensure_diag(c));  // (collective across ranks: on every rank)
  GLS_TRY(run_cell(c, gls::MODE_JV, v, y));
  HIP_TRY(gls::vec_gather_scale_set(y, c->diag.p, v, c->con_dofs.p, (int64_t)c->con_dofs.n, c->stream));
  return GLS_OK;
}

namespace {
// the V-cycle's operator on level g: J.v in FP32 arithmetic from the FP32 linearization when the
// level smooths in mixed precision (brick path), else the FP64 gls_jacobian_apply. Same
// constraint handling (constrained rows D_c v) and ghost exchange as gls_jacobian_apply.
// full = false: u and tau suffice (the Oseen smoother operator); else every row of the FP32 copy
int ensure_qdata32(gls_ctx *g, bool full = true) {
  GLS_TRY(ensure_qdata(g));
  if (!g->qd32_valid || (full && g->qd32_partial)) {
    if (g->qdata32.n != g->qdata.n) GLS_TRY(g->qdata32.alloc(g->qdata.n));
    HIP_TRY(gls::vec_to_f32(g->qdata.p, g->qdata32.p, (int64_t)g->qdata.n, g->stream));
    g->qd32_valid = true;
    g->qd32_partial = false;
  }
  return GLS_OK;
}
// FP32 kernels write their brick-surface partial sums in FP32 (half the slab traffic; summed in FP64)
bool slab_f32() { return std::getenv("GLS_SLAB_F64") == nullptr; }
// rb != nullptr: y = rb - A v (the V-cycle's residual), fused into the kernels' stores on one rank.
// first_omega > 0 (only where first_sweep_fusable): v is not read but formed as the first damped-Jacobi
// sweep from 0, v = 0 + first_omega rb / D (mg_jacobi_update's arithmetic), in the J.v's gather and
// stored to v by the J.v (brick-interior nodes) and the slab sum (surface nodes). Opt-in
// (GLS_MG_FIRST_FUSE=1): bitwise the separate update, but measured slower at Q2 128^3 (99.5 vs 96.0 ms per
// Newton step, profiles/r04_ab_env_switches.txt: the gather's two extra FP64 loads and FP64 divisions per
// node cost the J.v more than the update pass it saves)
bool first_sweep_fusable(gls_ctx *g) {
  const char *e = std::getenv("GLS_MG_FIRST_FUSE");
  return e && std::atoi(e) != 0 && g->smooth_f32 && g->use_brick && g->use_qdata && !g->use_colors && !g->dist.on &&
         !g->hang.on && g->k == 2 && g->cube_nb1 > 0 && g->use_slab && gls::pencil_enabled() &&
         std::getenv("GLS_MG_NO_FUSE") == nullptr;
}
int jacobian_apply_f32(gls_ctx *g, const double *v, double *y, const double *rb = nullptr, double first_omega = 0.0,
                       bool oseen = false) {
  if (!g->u) return set_err(GLS_EINVAL, "gls_set_state was not called");
  GLS_TRY(ensure_diag(g));
  GLS_TRY(ensure_qdata32(g, !oseen));
  GLS_TRY(dist_import(g, const_cast<double *>(v)));
  gls::OpParams P = make_params(g, true);
  P.qdf = g->qdata32.p;
  P.oseen = oseen ? 1 : 0;
  P.v = v;
  P.y = y;
  const bool col = g->use_colors;
  P.slab = col ? nullptr : brick_slab(g);
  const bool fuse_rb = rb && (P.slab || col) && !g->dist.on && gls::brick_fused_jacobi_supported(g->k) &&
                       std::getenv("GLS_MG_NO_FUSE") == nullptr;
  P.rb = fuse_rb ? rb : nullptr;
  P.slabf = P.slab && slab_f32() && gls::brick_fused_jacobi_supported(g->k) ? reinterpret_cast<float *>(P.slab)
                                                                             : nullptr;
  if (first_omega > 0.0) {
    if (!fuse_rb || !first_sweep_fusable(g)) return set_err(GLS_EINVAL, "fused first sweep not applicable");
    P.jx0 = const_cast<double *>(v);
    P.jd = g->diag.p;
    P.jomega = first_omega;
  }
  if (col) set_colors(g, P, y);
  if (!col && !P.slab) HIP_TRY(hipMemsetAsync(y, 0, sizeof(double) * g->n_dofs, g->stream));
  {
    TimedLaunch t(g, 4);
    HIP_TRY(gls::launch_brick_jv_f32(g->k, P, g->tables, g->stream));
  }
  if (P.slab) {
    TimedLaunch t(g, 5);
    HIP_TRY(slab_sum_ex(g, P.slab, P.slabf, y, nullptr, nullptr, P.jx0 ? g->diag.p : nullptr, P.jomega, P.rb, P.jx0));
  }
  GLS_TRY(dist_export_add(g, y));
  HIP_TRY(gls::vec_gather_scale_set(y, g->diag.p, v, g->con_dofs.p, (int64_t)g->con_dofs.n, g->stream, P.rb));
  if (rb && !fuse_rb) HIP_TRY(gls::vec_axpby(y, 1.0, rb, -1.0, g->n_dofs, g->stream));
  return GLS_OK;
}
// y = A v with the level's smoothing operator; rb != nullptr: y = rb - A v
int smoother_apply(gls_ctx *g, const double *v, double *y, const double *rb = nullptr) {
  if (g->smooth_f32 && g->use_brick && g->use_qdata) return jacobian_apply_f32(g, v, y, rb, 0.0, g->smooth_oseen);
  g->oct.f32_next = g->smooth_f32 && g->oct.on;  // adapted forest: its bricks in FP32, the other cells FP64
  const int rc = gls_jacobian_apply(g, v, y);
  g->oct.f32_next = false;
  GLS_TRY(rc);
  if (rb) HIP_TRY(gls::vec_axpby(y, 1.0, rb, -1.0, g->n_dofs, g->stream));
  return GLS_OK;
}
// one damped-Jacobi sweep x <- x + omega D^-1 (b - A x) with the smoother's operator A (constrained
// rows D_c x). Single rank on the brick path: fused into the J.v (brick-interior nodes) and the slab
// sum (brick-surface nodes), so A x is never stored; otherwise smoother_apply + mg_jacobi_update.
}  // namespace
static int ensure_ilu(gls_ctx *c);
static int ilu_probe(gls_ctx *c);
static int apply_ilu(gls_ctx *c, const double *v, double *z);
namespace {
// one ILU(0) smoothing sweep x <- x + M^-1 (b - A x) (M = the level's ILU(0), undamped; z: scratch)
int ilu_sweep(gls_ctx *g, double *x, const double *b, double *y, double *z) {
  GLS_TRY(ensure_ilu(g));
  GLS_TRY(gls_jacobian_apply(g, x, y));
  HIP_TRY(gls::vec_axpby(y, 1.0, b, -1.0, g->n_dofs, g->stream));  // y = b - A x
  GLS_TRY(apply_ilu(g, y, z));
  HIP_TRY(gls::vec_axpy(x, 1.0, z, g->n_dofs, g->stream));
  return GLS_OK;
}
int smoother_sweep(gls_ctx *g, double *x, const double *b, double *y, double omega, double *z = nullptr) {
  if (z && g->ilu.on && !g->ilu.probe_only) return ilu_sweep(g, x, b, y, z);
  const bool nofuse = std::getenv("GLS_MG_NO_FUSE") != nullptr;
  const bool brick = g->use_brick && g->use_qdata && (g->use_colors || brick_slab(g)) && !g->dist.on &&
                     !g->hang.on && gls::brick_fused_jacobi_supported(g->k);
  if (nofuse || !brick) {
    GLS_TRY(smoother_apply(g, x, y));
    HIP_TRY(gls::mg_jacobi_update(x, b, y, g->diag.p, omega, g->n_dofs, 0, g->stream));
    return GLS_OK;
  }
  if (!g->u) return set_err(GLS_EINVAL, "gls_set_state was not called");
  GLS_TRY(ensure_diag(g));
  const bool f32 = g->smooth_f32;
  GLS_TRY(f32 ? ensure_qdata32(g, !g->smooth_oseen) : ensure_qdata(g));
  gls::OpParams P = make_params(g, true);
  P.v = x;
  P.y = x;
  P.jx = x;
  P.jb = b;
  P.jd = g->diag.p;
  P.jomega = omega;
  if (g->use_colors) {  // surface-node running sums in a scratch vector (x is updated in place)
    if (g->acc.n != (size_t)g->n_dofs) GLS_TRY(g->acc.alloc((size_t)g->n_dofs));
    set_colors(g, P, g->acc.p);
  } else {
    P.slab = brick_slab(g);
  }
  if (f32) {
    P.qdf = g->qdata32.p;
    P.oseen = g->smooth_oseen ? 1 : 0;
    P.slabf = P.slab && slab_f32() ? reinterpret_cast<float *>(P.slab) : nullptr;
    TimedLaunch t(g, 4);
    HIP_TRY(gls::launch_brick_jv_f32(g->k, P, g->tables, g->stream));
  } else {
    P.qd = g->qdata.p;
    TimedLaunch t(g, 1);
    HIP_TRY(gls::launch_brick_kernel(g->k, gls::MODE_JVQ, P, g->tables, g->stream));
  }
  if (g->use_colors) return GLS_OK;
  TimedLaunch t(g, 5);
  HIP_TRY(slab_sum_ex(g, P.slab, P.slabf, x, g->vmask.p, b, g->diag.p, omega, nullptr));
  return GLS_OK;
}
}  // namespace

// y = A_s v with the operator the attached V-cycle smooths this level with (FP32 / Oseen per gls_mg_params)
int gls_mg_smoother_apply(gls_ctx *c, const double *v, double *y) {
  GLS_TRY(check_ctx(c));
  if (!v || !y || v == y) return set_err(GLS_EINVAL, "v/y null or aliased");
  return smoother_apply(c, v, y);
}

int gls_jacobian_apply_f32(gls_ctx *c, const double *v, double *y) {
  GLS_TRY(check_ctx(c));
  if (!v || !y || v == y) return set_err(GLS_EINVAL, "v/y null or aliased");
  if (!(c->use_brick && c->use_qdata)) return set_err(GLS_EINVAL, "FP32 J.v needs the 3D Qk-Qk brick path");
  return jacobian_apply_f32(c, v, y);
}

int gls_set_dirichlet(gls_ctx *c, int64_t n, const int64_t *dofs, const double *vals) {
  GLS_TRY(check_ctx(c));
  if (n < 0 || (n > 0 && (!dofs || !vals))) return set_err(GLS_EINVAL, "dirichlet arrays");
  for (int64_t i = 0; i < n; ++i)
    if (dofs[i] < 0 || dofs[i] >= c->n_dofs) return set_err(GLS_EINVAL, "dirichlet dof out of range");
  HIP_TRY(hipStreamSynchronize(c->stream));
  GLS_TRY(c->dir_dofs.upload(dofs, (size_t)n));
  GLS_TRY(c->dir_vals.upload(vals, (size_t)n));
  return GLS_OK;
}

int gls_apply_dirichlet(gls_ctx *c, double *x) {
  GLS_TRY(check_ctx(c));
  HIP_TRY(gls::vec_set_indexed(x, c->dir_dofs.p, c->dir_vals.p, (int64_t)c->dir_dofs.n, c->stream));
  // across ranks the masters of the lines below may be ghosts: their owners' values first (on every
  // rank, whether or not it holds lines: the exchange is collective)
  if (c->dist.on && c->dist.dofs) GLS_TRY(dist_import(c, x));
  if (c->hang.on)  // hanging values from their masters (all masters: Dirichlet values included)
    HIP_TRY(gls::vec_csr_gather_set(x, x, c->hang.dof.p, c->hang.off.p, c->hang.master.p, c->hang.w.p,
                                    (int64_t)c->hang.dof.n, c->stream));
  if (!c->jf.on && (x == c->u || x == c->u1 || x == c->u2 || x == c->u3)) {  // the captured state changed
    c->diag_valid = false;
    c->ilu.valid = false;
    c->qd_valid = false;
    c->cq_valid = false;
    c->mg.dirty = true;
  }
  return GLS_OK;
}

}  // extern "C"
// sibling groups of an adapted forest's leaves that form 2x2x2 bricks: 8 consecutive cells (the forest's
// depth-first order keeps a complete family together, children x fastest) of equal extents whose node
// maps agree on the 5^3 brick lattice (a node shared by two cells sits at the same brick position in
// both). GLS_OCT_BRICKS=0: per-cell kernels only.
static int detect_oct_bricks(gls_ctx *c) {
  auto &O = c->oct;
  O = gls_ctx::Oct();
  const char *e = std::getenv("GLS_OCT_BRICKS");
  if ((e && std::atoi(e) == 0) || c->dim != 3 || c->k != 2 || c->kp != 2 || c->map_degree > 0 || c->dist.on ||
      c->cell_pnodes.p || c->host_h.empty() || !gls::pencil_enabled() || c->n_cells < 8)
    return GLS_OK;
  const int64_t nc = c->n_cells;
  std::vector<int32_t> cv((size_t)nc * 27);
  HIP_TRY(hipMemcpy(cv.data(), c->cell_vnodes.p, cv.size() * sizeof(int32_t), hipMemcpyDeviceToHost));
  std::vector<int32_t> cell0;
  std::vector<char> in((size_t)nc, 0);
  int32_t lat[125];
  for (int64_t i = 0; i + 8 <= nc;) {
    bool ok = true;
    for (int ci = 1; ci < 8 && ok; ++ci)
      for (int d = 0; d < 3; ++d) ok = ok && c->host_h[(size_t)(i + ci) * 3 + d] == c->host_h[(size_t)i * 3 + d];
    for (int t = 0; t < 125 && ok; ++t) lat[t] = -1;
    for (int ci = 0; ci < 8 && ok; ++ci) {
      const int cx = ci & 1, cy = (ci >> 1) & 1, cz = ci >> 2;
      for (int a = 0; a < 27 && ok; ++a) {
        const int X = 2 * cx + a % 3, Y = 2 * cy + (a / 3) % 3, Z = 2 * cz + a / 9;
        int32_t &slot = lat[X + 5 * (Y + 5 * Z)];
        const int32_t nd = cv[(size_t)(i + ci) * 27 + a];
        if (slot < 0) slot = nd;
        else ok = slot == nd;
      }
    }
    if (ok) {  // 125 distinct nodes
      std::vector<int32_t> u(lat, lat + 125);
      std::sort(u.begin(), u.end());
      ok = std::adjacent_find(u.begin(), u.end()) == u.end();
    }
    if (ok) {
      cell0.push_back((int32_t)i);
      for (int ci = 0; ci < 8; ++ci) in[(size_t)(i + ci)] = 1;
      i += 8;
    } else {
      ++i;
    }
  }
  if (cell0.empty()) return GLS_OK;
  std::vector<int32_t> rest;
  for (int64_t q = 0; q < nc; ++q)
    if (!in[(size_t)q]) rest.push_back((int32_t)q);
  std::vector<int32_t> list(cell0.size());
  for (size_t b = 0; b < list.size(); ++b) list[b] = (int32_t)b;
  GLS_TRY(O.cell0.upload(cell0.data(), cell0.size()));
  GLS_TRY(O.list.upload(list.data(), list.size()));
  O.n_rest = (int)rest.size();
  if (rest.empty()) rest.push_back(0);  // (no per-cell launch when n_rest == 0)
  GLS_TRY(O.rest.upload(rest.data(), rest.size()));
  O.nb = (int)cell0.size();
  O.on = true;
  return GLS_OK;
}
extern "C" {
int gls_forest_bricks(const gls_ctx *c) { return c && c->oct.on ? c->oct.nb : 0; }

int gls_set_hanging(gls_ctx *c, int64_t n, const int64_t *dofs, const int64_t *off, const int64_t *masters,
                    const double *w) {
  GLS_TRY(check_ctx(c));
  if (n < 0 || (n > 0 && (!dofs || !off || !masters || !w))) return set_err(GLS_EINVAL, "gls_set_hanging: arrays");
  if (c->mg.on) return set_err(GLS_EINVAL, "hanging constraints: no multigrid");
  if (c->dist.on && !c->dist.dofs) return set_err(GLS_EINVAL, "hanging constraints across ranks: gls_dist_attach_dofs");
  HIP_TRY(hipStreamSynchronize(c->stream));
  const int dim = c->dim;
  const int64_t N = c->n_dofs, nvd = (int64_t)dim * c->n_vnodes;
  std::vector<uint8_t> vm((size_t)c->n_vnodes, 0);
  if (c->vmask.p) HIP_TRY(hipMemcpy(vm.data(), c->vmask.p, (size_t)c->n_vnodes, hipMemcpyDeviceToHost));
  auto dirichlet = [&](int64_t d) { return d < nvd && ((vm[(size_t)(d / dim)] >> (d % dim)) & 1); };
  std::vector<char> is_h((size_t)N, 0);
  if (n > 0 && off[0] != 0) return set_err(GLS_EINVAL, "gls_set_hanging: offsets[0] != 0");
  for (int64_t i = 0; i < n; ++i) {
    const int64_t d = dofs[i];
    if (d < 0 || d >= N || off[i + 1] < off[i]) return set_err(GLS_EINVAL, "gls_set_hanging: line %lld", (long long)i);
    if (dirichlet(d)) return set_err(GLS_EINVAL, "hanging DoF %lld carries a Dirichlet mask bit", (long long)d);
    if (is_h[(size_t)d]) return set_err(GLS_EINVAL, "hanging DoF %lld listed twice", (long long)d);
    is_h[(size_t)d] = 1;
  }
  const int64_t nm = n ? off[n] : 0;
  for (int64_t j = 0; j < nm; ++j)
    if (masters[j] < 0 || masters[j] >= N || is_h[(size_t)masters[j]])
      return set_err(GLS_EINVAL, "gls_set_hanging: master %lld out of range or hanging itself", (long long)masters[j]);
  // operator lines (closed zero_constraints: Dirichlet masters drop out) and their transpose
  std::vector<int64_t> ooff{0}, omas, cnt((size_t)N + 1, 0);
  std::vector<double> ow;
  for (int64_t i = 0; i < n; ++i) {
    for (int64_t j = off[i]; j < off[i + 1]; ++j)
      if (!dirichlet(masters[j])) {
        omas.push_back(masters[j]);
        ow.push_back(w[j]);
        ++cnt[(size_t)masters[j] + 1];
      }
    ooff.push_back((int64_t)omas.size());
  }
  std::vector<int64_t> tm, toff{0};
  std::vector<int64_t> start((size_t)N + 1, 0);
  for (int64_t m = 0; m < N; ++m) {
    start[(size_t)m + 1] = start[(size_t)m] + cnt[(size_t)m + 1];
    if (cnt[(size_t)m + 1]) {
      tm.push_back(m);
      toff.push_back(start[(size_t)m + 1]);
    }
  }
  std::vector<int64_t> tdof(omas.size()), fill(start.begin(), start.end() - 1);
  std::vector<double> tw(omas.size());
  for (int64_t i = 0; i < n; ++i)  // lines in order: each master sums its hanging rows in a fixed order
    for (int64_t j = ooff[(size_t)i]; j < ooff[(size_t)i + 1]; ++j) {
      const int64_t slot = fill[(size_t)omas[(size_t)j]]++;
      tdof[(size_t)slot] = dofs[i];
      tw[(size_t)slot] = ow[(size_t)j];
    }
  c->hang.h_dof.assign(dofs, dofs + n);
  c->hang.h_off.assign(off, off + n + 1);
  c->hang.h_master.assign(masters, masters + nm);
  if (n == 0) c->hang.h_off.assign(1, 0);
  std::vector<uint8_t> hm((size_t)c->n_vnodes, 0), dm((size_t)N, 0);
  std::vector<int64_t> con;  // zero_constraints: Dirichlet + hanging
  for (int64_t d = 0; d < N; ++d) {
    if (is_h[(size_t)d] && d < nvd) hm[(size_t)(d / dim)] |= (uint8_t)(1u << (d % dim));
    dm[(size_t)d] = is_h[(size_t)d] ? 1 : 0;
    if (is_h[(size_t)d] || dirichlet(d)) con.push_back(d);
  }
  auto &h = c->hang;
  GLS_TRY(h.dof.upload(dofs, (size_t)n));
  GLS_TRY(h.off.upload(off, (size_t)(n ? n + 1 : 0)));
  GLS_TRY(h.master.upload(masters, (size_t)nm));
  GLS_TRY(h.w.upload(w, (size_t)nm));
  GLS_TRY(h.ooff.upload(ooff.data(), n ? ooff.size() : 0));
  GLS_TRY(h.omaster.upload(omas.data(), omas.size()));
  GLS_TRY(h.ow.upload(ow.data(), ow.size()));
  GLS_TRY(h.tm.upload(tm.data(), tm.size()));
  GLS_TRY(h.toff.upload(toff.data(), tm.empty() ? 0 : toff.size()));
  GLS_TRY(h.tdof.upload(tdof.data(), tdof.size()));
  GLS_TRY(h.tw.upload(tw.data(), tw.size()));
  GLS_TRY(h.hmask.upload(hm.data(), hm.size()));
  GLS_TRY(h.dmask.upload(dm.data(), dm.size()));
  GLS_TRY(c->con_dofs.upload(con.data(), con.size()));
  h.on = n > 0;
  c->use_brick = false;  // mixed cell sizes: the general per-cell kernels
  c->use_slab = false;
  c->use_colors = false;
  c->diag_valid = false;
  c->ilu.valid = false;
  c->qd_valid = false;
  c->cq_valid = false;
  return detect_oct_bricks(c);
}

// --------------------------------------------------------------------------------------------
// Geometric multigrid V-cycle (right preconditioner). Levels are nested hyper_cube meshes; the
// coarse operators are the same GLS Jacobian re-discretised on the coarse mesh at the injected
// state (Galerkin-free, matrix-free), smoothed by damped Jacobi on their own diagonals.
// --------------------------------------------------------------------------------------------
namespace {
enum { MB_U = 0, MB_U1, MB_U2, MB_U3, MB_B, MB_X, MB_Y, MB_BOX, MB_N };
constexpr int64_t kDirectSmall = 8192, kDirectMax = 40000;  // coarsest-level dense LU: FP64 / FP32 ranges
double *mgbuf(gls_ctx *c, int l, int which) { return c->mg.bufs[(size_t)l * MB_N + which]->p; }
int64_t mg_nbox(const gls_ctx *c, int l) {
  const auto &d = c->mg.dims[(size_t)l];
  return (int64_t)d[0] * d[1] * d[2];
}
// level-l local vector -> box lattice layout (identity on a single GPU: returns loc itself)
const double *mg_to_box(gls_ctx *c, int l, const double *loc, bool owned_only) {
  if (!c->mg.boxed) return loc;
  gls_ctx *g = c->mg.lev[(size_t)l];
  double *box = mgbuf(c, l, MB_BOX);
  if (gls::mg_box_gather(loc, box, g->lat.map.p, mg_nbox(c, l), g->n_vnodes, owned_only ? g->dist.n_owned : -1,
                         c->stream) != hipSuccess)
    return nullptr;
  return box;
}
// where a transfer writing level-l data must put it (the box buffer, or loc itself)
double *mg_box_target(gls_ctx *c, int l, double *loc) { return c->mg.boxed ? mgbuf(c, l, MB_BOX) : loc; }
int mg_from_box(gls_ctx *c, int l, double *loc) {
  if (!c->mg.boxed) return GLS_OK;
  gls_ctx *g = c->mg.lev[(size_t)l];
  HIP_TRY(gls::mg_box_scatter(mgbuf(c, l, MB_BOX), loc, g->lat.map.p, mg_nbox(c, l), g->n_vnodes, c->stream));
  return GLS_OK;
}

// injected coarse state (every second lattice node); history likewise
int mg_inject_level(gls_ctx *c, int l, const double *fine, double *coarse) {
  if (c->mg.csr) {  // general hierarchy: the fine value at each coarse DoF's position (hanging values follow)
    const auto &X = *c->mg.xfer[(size_t)l - 1];
    HIP_TRY(gls::vec_pack_dofs(fine, X.inj.p, X.nc, coarse, c->stream));
    gls_ctx *g = c->mg.lev[(size_t)l];
    if (g->hang.on)
      HIP_TRY(gls::vec_csr_gather_set(coarse, coarse, g->hang.dof.p, g->hang.off.p, g->hang.master.p, g->hang.w.p,
                                      (int64_t)g->hang.dof.n, c->stream));
    return GLS_OK;
  }
  const double *fb = mg_to_box(c, l - 1, fine, false);
  if (!fb) return set_err(GLS_EHIP, "mg box gather failed");
  HIP_TRY(gls::mg_inject(fb, mg_box_target(c, l, coarse), c->mg.dims[(size_t)l - 1].data(), c->mg.dims[(size_t)l].data(),
                         c->stream));
  return mg_from_box(c, l, coarse);
}

int replica_gather(gls_ctx *c, const double *loc, double *glob);
int rep2_inject(gls_ctx *c, const double *loc, double *glob);
// The explicit coarse inverse (mg.probe) against the pinned matrix it came from (mg.probe_bak): y = A^-1 e,
// z = A y for e = (1, ..., 1); good = y finite and max|z - e| <= 1e-8 max(1, max|A| max|y|) (a backward-stable
// factorization leaves ~n eps there; an unpivoted LU through a tiny pivot leaves O(1) or non-finite values)
static int coarse_inverse_check(gls_ctx *c, int64_t n, bool *good) {
  auto &mg = c->mg;
  *good = false;
  if (mg.chk.n < (size_t)(2 * n)) GLS_TRY(mg.chk.alloc((size_t)(2 * n)));
  double *y = mg.chk.p, *z = mg.chk.p + n;
  HIP_TRY(gls::vec_fill(mg.unit.p, n, 1.0, c->stream));
  const double one = 1.0, zero = 0.0;
  rocblas_int imax = 0;
  if (rocblas_set_stream(mg.blas, c->stream) != rocblas_status_success ||
      rocblas_dgemv(mg.blas, rocblas_operation_none, (rocblas_int)n, (rocblas_int)n, &one, mg.probe.p, (rocblas_int)n,
                    mg.unit.p, 1, &zero, y, 1) != rocblas_status_success ||
      rocblas_dgemv(mg.blas, rocblas_operation_none, (rocblas_int)n, (rocblas_int)n, &one, mg.probe_bak.p,
                    (rocblas_int)n, y, 1, &zero, z, 1) != rocblas_status_success ||
      rocblas_idamax(mg.blas, (rocblas_int)(n * n), mg.probe_bak.p, 1, &imax) != rocblas_status_success)
    return set_err(GLS_EHIP, "coarse inverse check: rocBLAS failed");
  std::vector<double> h((size_t)(2 * n));
  double amax = 0.0;
  HIP_TRY(hipMemcpyAsync(h.data(), mg.chk.p, sizeof(double) * (size_t)(2 * n), hipMemcpyDeviceToHost, c->stream));
  if (imax > 0)
    HIP_TRY(hipMemcpyAsync(&amax, mg.probe_bak.p + (imax - 1), sizeof(double), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  double ymax = 0.0, err = 0.0;
  for (int64_t i = 0; i < n; ++i) {
    if (!std::isfinite(h[(size_t)i]) || !std::isfinite(h[(size_t)(n + i)])) return GLS_OK;
    ymax = std::max(ymax, std::fabs(h[(size_t)i]));
    err = std::max(err, std::fabs(h[(size_t)(n + i)] - 1.0));
  }
  *good = err <= 1e-8 * std::max(1.0, std::fabs(amax) * ymax);
  if (std::getenv("GLS_MG_VERBOSE"))
    std::printf("mg: coarse inverse check n=%lld max|Ay-e| %.3e max|A| %.3e max|y| %.3e -> %s\n", (long long)n, err,
                std::fabs(amax), ymax, *good ? "ok" : "FAILED");
  return GLS_OK;
}

// the direct coarse solve's matrix by colored probing on a per-cell level (mg.probe_ilu; brick levels and
// distributed or nested contexts: one J.v per column): the ILU structure (CM order, fill 0, one block) is attached once
int mg_probe_setup(gls_ctx *c, gls_ctx *g) {
  auto &mg = c->mg;
  mg.probe_ilu = nullptr;
  if ((g->use_brick && g->use_qdata) || g->dist.on || g->mg.on || g->ilu.on)
    return GLS_OK;
  GLS_TRY(gls_ilu_set_options(g, GLS_ILU_ORDER_CM, 0));
  GLS_TRY(gls_ilu_attach(g, 0, 0.0, 1.0));
  g->ilu.probe_only = true;
  mg.ilu_levels.push_back(g);  // detached with the multigrid
  GLS_TRY(mg.pinv.alloc((size_t)g->n_dofs));
  mg.probe_ilu = g;
  return GLS_OK;
}

// the large coarsest level's FP32 factorization (kDirectSmall < n): rocSOLVER sgetrf_npvt of the pinned matrix (138 ms
// at n = 25000 against sgetrf's 410 + sgetri's ~800) and its check |A x - 1| / |1| on the side stream, ordered after
// the context stream's probing / rounding; nothing here waits on the host
int coarse_lu32_start(gls_ctx *c, int64_t n, int64_t pin) {
  auto &mg = c->mg;
  HIP_TRY(mg.side.ensure());
  hipStream_t s = mg.side.s;
  if (mg.chk32.n != (size_t)(2 * n)) GLS_TRY(mg.chk32.alloc((size_t)(2 * n)));
  if (mg.lu_rel.n != 1) GLS_TRY(mg.lu_rel.alloc(1));
  HIP_TRY(hipEventRecord(mg.side.e0, c->stream));
  HIP_TRY(hipStreamWaitEvent(s, mg.side.e0, 0));
  int dev = 0;
  HIP_TRY(hipGetDevice(&dev));
  mg.side.join();
  mg.side.rc = 0;
  auto *m = &mg;
  const bool verbose = std::getenv("GLS_MG_VERBOSE") != nullptr;
  const int64_t bl = mg.lu_cm ? mg.lu_bl : -1, bu = mg.lu_cm ? mg.lu_bu : -1;
  mg.side.worker = std::thread([m, s, n, pin, dev, verbose, bl, bu]() {
    const double one = 1.0, mone = -1.0;
    int &rc = m->side.rc;
    const auto h0 = std::chrono::steady_clock::now();
    // banded: right-looking by column blocks as wide as the band (rocSOLVER's calls return only when done, so few
    // wide blocks: 256-wide ones took 98 calls and longer than the dense factorization, profiles/
    // r06_ab_banded_coarse_lu.txt): the block's panel down to the lower band, its rows of U to the upper band, the
    // trailing band update; without pivoting nothing outside the band fills
    const int64_t nb = bl < 0 ? n : std::max<int64_t>(512, ((std::max(bl, bu) + 255) / 256) * 256);
    if (hipSetDevice(dev) != hipSuccess) rc = 1;
    else if (rocblas_set_stream(m->blas, s) != rocblas_status_success) rc = 2;
    const float fone = 1.0f, fmone = -1.0f;
    float *A = m->probe32.p;
    for (int64_t k0 = 0; k0 < n && !rc; k0 += nb) {
      const int64_t kb = std::min(nb, n - k0), mr = bl < 0 ? n - k0 : std::min(n - k0, kb + bl);
      const int64_t nc = bl < 0 ? 0 : std::min(n - k0 - kb, bu);
      float *A11 = A + k0 + k0 * n, *A12 = A + k0 + (k0 + kb) * n;
      if (rocsolver_sgetrf_npvt(m->blas, (rocblas_int)mr, (rocblas_int)kb, A11, (rocblas_int)n, m->info.p) !=
          rocblas_status_success)
        rc = 3;
      else if (nc > 0 &&
               rocblas_strsm(m->blas, rocblas_side_left, rocblas_fill_lower, rocblas_operation_none, rocblas_diagonal_unit,
                             (rocblas_int)kb, (rocblas_int)nc, &fone, A11, (rocblas_int)n, A12, (rocblas_int)n) !=
                   rocblas_status_success)
        rc = 3;
      else if (nc > 0 && mr > kb &&
               rocblas_sgemm(m->blas, rocblas_operation_none, rocblas_operation_none, (rocblas_int)(mr - kb),
                             (rocblas_int)nc, (rocblas_int)kb, &fmone, A11 + kb, (rocblas_int)n, A12, (rocblas_int)n,
                             &fone, A12 + kb, (rocblas_int)n) != rocblas_status_success)
        rc = 3;
    }
    if (verbose)
      std::printf("mg: the %s FP32 LU returned to its worker thread after %.2f ms\n", bl < 0 ? "dense" : "banded",
                  std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - h0).count());
    if (!rc &&
        !(gls::vec_fill(m->chk32.p, n, 1.0, s) == hipSuccess && gls::mg_zero_row(m->chk32.p, 1, pin, s) == hipSuccess &&
          gls::vec_to_f32(m->chk32.p, m->x32.p, n, s) == hipSuccess &&
          gls::dense_lu_solve_f32(m->probe32.p, (int)n, m->x32.p, s, (int)bl, (int)bu) == hipSuccess &&
          gls::vec_from_f32(m->x32.p, m->chk32.p + n, n, s) == hipSuccess &&
          rocblas_dgemv(m->blas, rocblas_operation_none, (rocblas_int)n, (rocblas_int)n, &one, m->probe.p,
                        (rocblas_int)n, m->chk32.p + n, 1, &mone, m->chk32.p, 1) == rocblas_status_success &&
          rocblas_set_pointer_mode(m->blas, rocblas_pointer_mode_device) == rocblas_status_success &&
          rocblas_dnrm2(m->blas, (rocblas_int)n, m->chk32.p, 1, m->lu_rel.p) == rocblas_status_success))
      rc = 4;
    (void)rocblas_set_pointer_mode(m->blas, rocblas_pointer_mode_host);
    if (!rc && hipEventRecord(m->side.e1, s) != hipSuccess) rc = 5;
  });
  mg.lu_pending = true;
  mg.lu_n = n;
  mg.lu_pin = pin;
  return GLS_OK;
}
// before the first coarse solve of the state: the side stream's factorization checked; a factorization that pivot growth
// broke (O(1) or non-finite residual) is replaced by the pivoted sgetrf + sgetri inverse on the context stream. A
// coarse-grid correction accurate to 1 % is exact enough for the V-cycle.
int coarse_lu32_finish(gls_ctx *c) {
  auto &mg = c->mg;
  if (!mg.lu_pending) return GLS_OK;
  mg.lu_pending = false;
  mg.side.join();
  (void)rocblas_set_stream(mg.blas, c->stream);
  if (mg.side.rc) {
    mg.direct_ok = mg.lu32 = false;
    mg.dirty = true;
    return set_err(GLS_EHIP, "coarse FP32 LU on the side stream failed (step %d)", mg.side.rc);
  }
  const int64_t n = mg.lu_n;
  int inf = -1;
  double rn = INFINITY;
  HIP_TRY(hipMemcpyAsync(&inf, mg.info.p, sizeof(int), hipMemcpyDeviceToHost, mg.side.s));
  HIP_TRY(hipMemcpyAsync(&rn, mg.lu_rel.p, sizeof(double), hipMemcpyDeviceToHost, mg.side.s));
  HIP_TRY(hipStreamSynchronize(mg.side.s));
  const double rel = inf == 0 ? rn / std::sqrt((double)n) : INFINITY;
  const bool verbose = std::getenv("GLS_MG_VERBOSE") != nullptr;
  // (below 1e-2 the correction is used as it is; up to 0.5 with one refinement step x += LU^-1 (b - A x) against the
  // FP64 matrix (an extra solve and one FP64 matrix pass per coarse solve: residual error ~ rel^2); beyond, or a
  // broken factorization, the pivoted route)
  mg.lu32_refine = inf == 0 && rel >= 1e-2 && rel < 0.5;
  if (verbose)
    std::printf("mg: coarse FP32 unpivoted LU n=%lld info=%d, check |A x - 1| / |1| = %.2e%s\n", (long long)n, inf, rel,
                mg.lu32_refine ? ", applied with one refinement step" : "");
  if (inf == 0 && rel < 0.5) return GLS_OK;
  mg.lu32_npvt = mg.lu32_refine = false;
  HIP_TRY(gls::vec_to_f32(mg.probe.p, mg.probe32.p, n * n, c->stream));  // the pinned matrix again
  if (rocblas_set_stream(mg.blas, c->stream) != rocblas_status_success ||
      rocsolver_sgetrf(mg.blas, (rocblas_int)n, (rocblas_int)n, mg.probe32.p, (rocblas_int)n, mg.ipiv.p, mg.info.p) !=
          rocblas_status_success)
    return set_err(GLS_EHIP, "rocsolver_sgetrf failed");
  HIP_TRY(hipMemcpyAsync(&inf, mg.info.p, sizeof(int), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  if (inf == 0) {
    if (rocsolver_sgetri(mg.blas, (rocblas_int)n, mg.probe32.p, (rocblas_int)n, mg.ipiv.p, mg.info.p) !=
        rocblas_status_success)
      return set_err(GLS_EHIP, "rocsolver_sgetri failed");
    HIP_TRY(hipMemcpyAsync(&inf, mg.info.p, sizeof(int), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
  }
  if (verbose) std::printf("mg: coarse FP32 pivoted LU + inverse n=%lld info=%d\n", (long long)n, inf);
  if (inf != 0) {
    mg.direct_ok = mg.lu32 = false;
    mg.dirty = true;
    return set_err(GLS_EINVAL, "coarse FP32 LU: zero pivot %d", inf);
  }
  return GLS_OK;
}

int mg_prepare(gls_ctx *c) {
  auto &mg = c->mg;
  if (!mg.dirty) return GLS_OK;
  GLS_TRY(coarse_lu32_finish(c));  // (its buffers are re-probed below)
  const bool verbose = std::getenv("GLS_MG_VERBOSE") != nullptr;
  auto tick = [&]() {  // host wall time of the preparation phases (verbose only: synchronizes)
    if (verbose) (void)hipStreamSynchronize(c->stream);
    return std::chrono::steady_clock::now();
  };
  auto ms = [](std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
    return std::chrono::duration<double, std::milli>(b - a).count();
  };
  const auto t0 = tick();
  const int L = (int)mg.lev.size();
  // the levels are re-discretised at the Jacobian's state (the frozen snapshot under skip_newton)
  const bool fz = c->jf.on;
  const double *ju = fz ? c->jf.u.p : c->u;
  const double *jh[3] = {fz ? (c->jf.has[0] ? c->jf.h[0].p : nullptr) : c->u1,
                         fz ? (c->jf.has[1] ? c->jf.h[1].p : nullptr) : c->u2,
                         fz ? (c->jf.has[2] ? c->jf.h[2].p : nullptr) : c->u3};
  const int jscheme = fz ? c->jf.scheme : c->scheme;
  const double *jts = fz ? c->jf.ts : c->time_steps;
  for (int l = 1; l < L; ++l) {
    gls_ctx *g = mg.lev[l];
    const double *fu = l == 1 ? ju : mgbuf(c, l - 1, MB_U);
    const double *fh[3] = {l == 1 ? jh[0] : (jh[0] ? mgbuf(c, l - 1, MB_U1) : nullptr),
                           l == 1 ? jh[1] : (jh[1] ? mgbuf(c, l - 1, MB_U2) : nullptr),
                           l == 1 ? jh[2] : (jh[2] ? mgbuf(c, l - 1, MB_U3) : nullptr)};
    GLS_TRY(mg_inject_level(c, l, fu, mgbuf(c, l, MB_U)));
    GLS_TRY(gls_apply_dirichlet(g, mgbuf(c, l, MB_U)));
    double *gh[3] = {nullptr, nullptr, nullptr};
    for (int h = 0; h < 3; ++h)
      if (fh[h]) {
        gh[h] = mgbuf(c, l, MB_U1 + h);
        GLS_TRY(mg_inject_level(c, l, fh[h], gh[h]));
      }
    g->viscosity = c->viscosity;
    GLS_TRY(gls_set_time(g, jscheme, jts));
    GLS_TRY(gls_set_state(g, mgbuf(c, l, MB_U), gh[0], gh[1], gh[2]));
    GLS_TRY(ensure_diag(g));
  }
  if (mg.rep_csr) {  // the replica hierarchy takes the fine state (injected, summed over ranks) and time data
    gls_ctx *r = mg.rep2;
    const double *st[4] = {ju, jh[0], jh[1], jh[2]};
    for (int i = 0; i < 4; ++i)
      if (st[i]) GLS_TRY(rep2_inject(c, st[i], mg.rep_u[i].p));
    GLS_TRY(gls_apply_dirichlet(r, mg.rep_u[0].p));
    r->viscosity = c->viscosity;
    GLS_TRY(gls_set_time(r, jscheme, jts));
    GLS_TRY(gls_set_state(r, mg.rep_u[0].p, st[1] ? mg.rep_u[1].p : nullptr, st[2] ? mg.rep_u[2].p : nullptr,
                          st[3] ? mg.rep_u[3].p : nullptr));
    if (!mg.direct) {
      mg.dirty = false;
      return GLS_OK;
    }
  }
  if (mg.replica) {  // the replica takes the coarsest distributed level's state (gathered) and time data
    gls_ctx *g = mg.lev[(size_t)L - 1], *r = mg.replica;
    const double *st[4] = {g->u, g->u1, g->u2, g->u3};
    for (int i = 0; i < 4; ++i)
      if (st[i]) GLS_TRY(replica_gather(c, st[i], mg.rep_u[i].p));
    r->viscosity = c->viscosity;
    GLS_TRY(gls_set_time(r, jscheme, jts));
    GLS_TRY(gls_set_state(r, mg.rep_u[0].p, st[1] ? mg.rep_u[1].p : nullptr, st[2] ? mg.rep_u[2].p : nullptr,
                          st[3] ? mg.rep_u[3].p : nullptr));
  }
  mg.direct_ok = false;
  if (mg.direct) {  // probe A = J_coarse column by column, then invert on the device
    // coarsest level: the last one, or the whole-mesh replica below a distributed fine level (rep_csr)
    gls_ctx *g = mg.rep_csr ? mg.rep2 : mg.lev[(size_t)L - 1];
    const int64_t n = g->n_dofs;
    if (g->use_brick && g->use_qdata) {  // all unit vectors in one launch per batch
      GLS_TRY(ensure_diag(g));
      GLS_TRY(ensure_qdata(g));
      gls::OpParams P = make_params(g, true);
      P.qd = g->qdata.p;
      P.y = mg.probe.p;
      HIP_TRY(hipMemsetAsync(mg.probe.p, 0, sizeof(double) * (size_t)(n * n), c->stream));
      const int batch = 4096;
      for (int64_t j0 = 0; j0 < n; j0 += batch) {
        const int nb = (int)std::min<int64_t>(batch, n - j0);
        P.y = mg.probe.p + j0 * n;
        HIP_TRY(gls::launch_brick_probe(g->k, P, g->tables, j0, nb, c->stream));
        HIP_TRY(gls::mg_probe_fix(mg.probe.p + j0 * n, n, j0, nb, g->con_dofs.p, (int64_t)g->con_dofs.n, g->diag.p,
                                  c->stream));
      }
    } else if (mg.probe_ilu == g && g->ilu.on) {  // colored batched probes into the ILU's CSR, then dense
      GLS_TRY(ensure_diag(g));
      GLS_TRY(ilu_probe(g));
      HIP_TRY(hipMemsetAsync(mg.probe.p, 0, sizeof(double) * (size_t)(n * n), c->stream));
      const auto &I = g->ilu;
      mg.lu_cm = n > kDirectSmall;
      if (mg.lu_cm) {  // FP32 range: keep the CSR's Cuthill-McKee order (banded), bandwidths from its pattern once
        if (mg.lu_bl < 0) {
          std::vector<int64_t> rp((size_t)n + 1);
          std::vector<int32_t> cl((size_t)I.nnz), pm((size_t)n), id((size_t)n);
          HIP_TRY(hipMemcpy(rp.data(), I.rowp.p, sizeof(int64_t) * rp.size(), hipMemcpyDeviceToHost));
          HIP_TRY(hipMemcpy(cl.data(), I.col.p, sizeof(int32_t) * cl.size(), hipMemcpyDeviceToHost));
          HIP_TRY(hipMemcpy(pm.data(), I.perm.p, sizeof(int32_t) * pm.size(), hipMemcpyDeviceToHost));
          int64_t bl = 0, bu = 0;
          for (int64_t r = 0; r < n; ++r)
            for (int64_t e = rp[(size_t)r]; e < rp[(size_t)r + 1]; ++e) {
              bl = std::max<int64_t>(bl, r - cl[(size_t)e]);
              bu = std::max<int64_t>(bu, cl[(size_t)e] - r);
            }
          for (int64_t i = 0; i < n; ++i) id[(size_t)i] = (int32_t)i;
          GLS_TRY(mg.lu_ident.upload(id.data(), id.size()));
          GLS_TRY(mg.lu_tmp.alloc((size_t)n));
          mg.lu_bl = bl;
          mg.lu_bu = bu;
          mg.lu_pin_cm = pm[(size_t)((int64_t)g->dim * g->n_vnodes)];  // the first pressure DoF's row
          if (verbose) std::printf("mg: coarse matrix n=%lld in Cuthill-McKee order: bandwidths %lld / %lld\n", (long long)n,
                                   (long long)bl, (long long)bu);
        }
        HIP_TRY(gls::csr_to_dense(mg.probe.p, I.rowp.p, I.col.p, I.val.p, mg.lu_ident.p, mg.pinv.p, n, c->stream));
      } else {
        HIP_TRY(gls::csr_to_dense(mg.probe.p, I.rowp.p, I.col.p, I.val.p, I.perm.p, mg.pinv.p, n, c->stream));
      }
    } else {
      HIP_TRY(gls::vec_fill(mg.unit.p, n, 0.0, c->stream));
      for (int64_t j = 0; j < n; ++j) {
        HIP_TRY(gls::mg_unit_step(mg.unit.p, j, c->stream));
        GLS_TRY(gls_jacobian_apply(g, mg.unit.p, mg.probe.p + j * n));
      }
    }
    const auto t1 = tick();
    mg.lu = false;
    mg.lu32 = false;
    if (n > kDirectSmall) {  // FP32 LU of the pinned matrix: unpivoted (checked), else pivoted + explicit inverse
      const int64_t pin0 = (int64_t)g->dim * g->n_vnodes;  // the first pressure DoF
      if (pin0 >= n) return set_err(GLS_EINVAL, "mg: coarsest level without pressure DoFs");
      if (!(mg.probe_ilu == g && g->ilu.on)) mg.lu_cm = false;
      const int64_t pin = mg.lu_cm ? mg.lu_pin_cm : pin0;  // (its row in the matrix's order)
      HIP_TRY(gls::mg_pin_dof(mg.probe.p, n, pin, c->stream));
      HIP_TRY(gls::vec_to_f32(mg.probe.p, mg.probe32.p, n * n, c->stream));
      GLS_TRY(coarse_lu32_start(c, n, pin));
      if (verbose) std::printf("mg: coarse FP32 unpivoted LU n=%lld queued on the side stream at %.2f ms\n", (long long)n,
                               ms(t0, tick()));
      mg.lu32 = mg.lu32_npvt = mg.direct_ok = true;
      mg.dirty = false;
      return GLS_OK;
    }
    // gj | lu | lu_npvt. Default: LU without pivoting (rocSOLVER's pivoted panel factorization is ~1 ms of
    // a Newton step at n = 500, profiles/r04_ab_env_switches.txt) with a pivoted retry when a pivot vanishes
    const char *cs = std::getenv("GLS_MG_COARSE_SOLVER");
    const bool use_lu = cs ? std::strncmp(cs, "lu", 2) == 0 : true;  // LU: 1.5-3 ms at n = 500 vs the one-workgroup GJ's ~15
    bool npvt = cs ? std::strcmp(cs, "lu_npvt") == 0 : true;
    if (use_lu) {  // LU with the pressure gauge pinned
      const int64_t pin = (int64_t)g->dim * g->n_vnodes;  // the first pressure DoF
      if (pin >= n) return set_err(GLS_EINVAL, "mg: coarsest level without pressure DoFs");
      HIP_TRY(gls::mg_pin_dof(mg.probe.p, n, pin, c->stream));
      if (npvt && !cs) {  // keep the matrix for a pivoted retry
        if (mg.probe_bak.n != (size_t)(n * n)) GLS_TRY(mg.probe_bak.alloc((size_t)(n * n)));
        HIP_TRY(gls::vec_copy(mg.probe_bak.p, mg.probe.p, n * n, c->stream));
      }
      int inf = -1;
      for (int attempt = 0; attempt < 2; ++attempt) {
        if (rocblas_set_stream(mg.blas, c->stream) != rocblas_status_success ||
            (npvt ? rocsolver_dgetrf_npvt(mg.blas, (rocblas_int)n, (rocblas_int)n, mg.probe.p, (rocblas_int)n, mg.info.p)
                  : rocsolver_dgetrf(mg.blas, (rocblas_int)n, (rocblas_int)n, mg.probe.p, (rocblas_int)n, mg.ipiv.p,
                                     mg.info.p)) != rocblas_status_success)
          return set_err(GLS_EHIP, "rocsolver_dgetrf failed");
        if (npvt) {  // identity permutation for getri
          if (mg.npvt_ipiv_n != n) {
            std::vector<int> id((size_t)n);
            for (int64_t i = 0; i < n; ++i) id[(size_t)i] = (int)(i + 1);
            HIP_TRY(hipMemcpyAsync(mg.ipiv.p, id.data(), sizeof(int) * (size_t)n, hipMemcpyHostToDevice, c->stream));
            HIP_TRY(hipStreamSynchronize(c->stream));
            mg.npvt_ipiv_n = n;
          }
        }
        HIP_TRY(hipMemcpyAsync(&inf, mg.info.p, sizeof(int), hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipStreamSynchronize(c->stream));
        if (inf == 0 || !npvt || cs) break;
        if (verbose) std::printf("mg: unpivoted coarse LU hit pivot %d, retrying with pivoting\n", inf);
        HIP_TRY(gls::vec_copy(mg.probe.p, mg.probe_bak.p, n * n, c->stream));  // the pinned matrix again
        npvt = false;
        mg.npvt_ipiv_n = -1;  // getrf overwrites ipiv with its permutation
      }
      const auto t2 = tick();
      if (verbose) std::printf("mg: levels+probe %.2f ms, getrf %.2f ms\n", ms(t0, t1), ms(t1, t2));
      if (inf == 0) {
        if (rocsolver_dgetri(mg.blas, (rocblas_int)n, mg.probe.p, (rocblas_int)n, mg.ipiv.p, mg.info.p) !=
            rocblas_status_success)
          return set_err(GLS_EHIP, "rocsolver_dgetri failed");
        HIP_TRY(hipMemcpyAsync(&inf, mg.info.p, sizeof(int), hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipStreamSynchronize(c->stream));
        // an unpivoted LU of the indefinite velocity-pressure Jacobian passes getrf with a tiny nonzero
        // pivot and can return a wildly wrong (or non-finite) inverse: check A (A^-1 e) = e and redo the
        // factorization with partial pivoting when it fails
        if (inf == 0 && npvt && !cs) {
          bool good = false;
          GLS_TRY(coarse_inverse_check(c, n, &good));
          if (!good) {
            if (verbose) std::printf("mg: unpivoted coarse inverse failed its check, refactoring with pivoting\n");
            HIP_TRY(gls::vec_copy(mg.probe.p, mg.probe_bak.p, n * n, c->stream));
            mg.npvt_ipiv_n = -1;
            npvt = false;
            if (rocsolver_dgetrf(mg.blas, (rocblas_int)n, (rocblas_int)n, mg.probe.p, (rocblas_int)n, mg.ipiv.p,
                                 mg.info.p) != rocblas_status_success)
              return set_err(GLS_EHIP, "rocsolver_dgetrf failed");
            HIP_TRY(hipMemcpyAsync(&inf, mg.info.p, sizeof(int), hipMemcpyDeviceToHost, c->stream));
            HIP_TRY(hipStreamSynchronize(c->stream));
            if (inf == 0) {
              if (rocsolver_dgetri(mg.blas, (rocblas_int)n, mg.probe.p, (rocblas_int)n, mg.ipiv.p, mg.info.p) !=
                  rocblas_status_success)
                return set_err(GLS_EHIP, "rocsolver_dgetri failed");
              HIP_TRY(hipMemcpyAsync(&inf, mg.info.p, sizeof(int), hipMemcpyDeviceToHost, c->stream));
              HIP_TRY(hipStreamSynchronize(c->stream));
            }
          }
        }
        if (inf == 0) HIP_TRY(gls::mg_zero_row(mg.probe.p, n, pin, c->stream));  // pinned unknown: zero correction
      }
      mg.lu = mg.direct_ok = inf == 0;
      if (verbose) std::printf("mg: coarse LU n=%lld info=%d, getri done at %.2f ms\n", (long long)n, inf, ms(t0, tick()));
      if (!mg.lu) {  // re-probe for the Gauss-Jordan fallback below (getrf overwrote the matrix)
        mg.dirty = true;
        return set_err(GLS_EINVAL, "coarse LU: zero pivot %d (set GLS_MG_COARSE_SOLVER=gj)", inf);
      }
    } else {
      HIP_TRY(gls::mg_dense_invert(mg.probe.p, mg.aug.p, (int)n, mg.status.p, c->stream));
      int st = -1;
      HIP_TRY(hipMemcpyAsync(&st, mg.status.p, sizeof(int), hipMemcpyDeviceToHost, c->stream));
      HIP_TRY(hipStreamSynchronize(c->stream));
      // a couple of dependent columns (pressure gauge) are expected; many mean a broken operator
      mg.direct_ok = st >= 0 && st <= 4;
      if (std::getenv("GLS_MG_VERBOSE")) std::printf("mg: coarse direct solve n=%lld dropped=%d ok=%d\n", (long long)n, st, (int)mg.direct_ok);
    }
  }
  mg.dirty = false;
  return GLS_OK;
}

// coarse rhs bc (level l+1) = R y (y on level l): restrict the owned rows, export-add coarse ghost rows
int mg_restrict(gls_ctx *c, int l, const double *y, double *bc) {
  auto &mg = c->mg;
  gls_ctx *h = mg.lev[(size_t)l + 1];
  hipStream_t s = c->stream;
  if (mg.csr) {
    const auto &X = *mg.xfer[(size_t)l];
    HIP_TRY(gls::vec_csr_spmv(bc, y, X.roff.p, X.rcol.p, X.rw.p, X.nc, false, s, X.rlane));
    (void)h;
    return GLS_OK;
  }
  const double *yb = mg_to_box(c, l, y, true);
  if (!yb) return set_err(GLS_EHIP, "mg box gather failed");
  {
    const auto &T = *mg.taps[(size_t)l];
    const int32_t *ti[3] = {T.ri[0].p, T.ri[1].p, T.ri[2].p}, *tc[3] = {T.rc[0].p, T.rc[1].p, T.rc[2].p};
    const double *tw[3] = {T.rw[0].p, T.rw[1].p, T.rw[2].p};
    if (T.two_pass)
      HIP_TRY(gls::mg_transfer_2pass(yb, mg_box_target(c, l + 1, bc), mg.dims[l].data(), mg.dims[l + 1].data(), 1, ti,
                                     tw, tc, mg.xwork.p, s));
    else
      HIP_TRY(gls::mg_transfer3d(yb, mg_box_target(c, l + 1, bc), mg.dims[l].data(), mg.dims[l + 1].data(), ti, tw,
                                 tc, s));
  }
  GLS_TRY(mg_from_box(c, l + 1, bc));
  GLS_TRY(dist_export_add(h, bc));
  return GLS_OK;
}

// y (level l) = P xc (xc on level l+1; its ghost values are imported first); add: y += P xc
// (single rank, two-pass transfer only: the caller checks mg_prolong_add_ok)
bool mg_prolong_add_ok(gls_ctx *c, int l) {
  if (c->mg.csr) return false;  // general hierarchies: P xc, constrained rows zeroed, then added
  return !c->mg.boxed && c->mg.taps[(size_t)l]->two_pass && std::getenv("GLS_MG_NO_FUSE") == nullptr;
}
int mg_prolong(gls_ctx *c, int l, double *xc, double *y, bool add = false) {
  auto &mg = c->mg;
  gls_ctx *h = mg.lev[(size_t)l + 1];
  hipStream_t s = c->stream;
  if (mg.csr) {
    const auto &X = *mg.xfer[(size_t)l];
    HIP_TRY(gls::vec_csr_spmv(y, xc, X.poff.p, X.pcol.p, X.pw.p, X.nf, add, s, X.plane));
    return GLS_OK;
  }
  GLS_TRY(dist_import(h, xc));
  const double *xb = mg_to_box(c, l + 1, xc, false);
  if (!xb) return set_err(GLS_EHIP, "mg box gather failed");
  {
    const auto &T = *mg.taps[(size_t)l];
    const int32_t *ti[3] = {T.pi[0].p, T.pi[1].p, T.pi[2].p}, *tc[3] = {T.pc[0].p, T.pc[1].p, T.pc[2].p};
    const double *tw[3] = {T.pw[0].p, T.pw[1].p, T.pw[2].p};
    if (T.two_pass)
      HIP_TRY(gls::mg_transfer_2pass(xb, mg_box_target(c, l, y), mg.dims[l + 1].data(), mg.dims[l].data(), 0, ti, tw,
                                     tc, mg.xwork.p, s, add ? 1 : 0));
    else if (add)
      return set_err(GLS_EINVAL, "mg_prolong: accumulate needs the two-pass transfer");
    else
      HIP_TRY(gls::mg_transfer3d(xb, mg_box_target(c, l, y), mg.dims[l + 1].data(), mg.dims[l].data(), ti, tw, tc, s));
  }
  GLS_TRY(mg_from_box(c, l, y));
  return GLS_OK;
}

// coarsest level by HIP graph (opt-in, GLS_MG_GRAPH=1: measured at 128^3, 138.0 vs 138.6 ms per
// Newton step -- the coarse sweeps are bound by the kernels' own latency, not by launch overhead,
// profiles/r01_coarse_graph_bench.txt): one rank, fused brick sweeps, the level's own b / x buffers (the
// captured launches bake in their pointers and this state's OpParams; mg_prepare drops the graph)
bool coarse_graph_eligible(gls_ctx *c, gls_ctx *g, const double *b, const double *x) {
  const int l = (int)c->mg.lev.size() - 1;
  return !c->mg.cgraph_failed && !c->mg.boxed && !g->dist.on && !g->hang.on && g->use_brick && g->use_qdata &&
         brick_slab(g) && gls::brick_fused_jacobi_supported(g->k) && g->stream == c->stream &&
         b == mgbuf(c, l, MB_B) && x == mgbuf(c, l, MB_X) && std::getenv("GLS_MG_NO_FUSE") == nullptr &&
         std::getenv("GLS_MG_GRAPH") != nullptr;
}
// everything the captured launches bake in: the level's OpParams (pointers, time coefficients,
// viscosity), the sweep count and damping, and the buffers the sweeps read and write. Buffer
// CONTENTS (state, linearization, diagonal) are read at replay time, so a new Newton state with
// unchanged parameters replays the same graph.
}  // extern "C"
static std::vector<unsigned char> coarse_graph_key(gls_ctx *g, const double *b, const double *x, const double *y,
                                                   int pre, double om) {
  const gls::OpParams P = make_params(g);
  const void *ptrs[7] = {b, x, y, g->diag.p, g->qdata.p, g->qdata32.p, brick_slab(g)};
  const int64_t ints[4] = {pre, g->n_dofs, (int64_t)g->smooth_f32, (int64_t)slab_f32()};
  std::vector<unsigned char> k(sizeof(P) + sizeof(ptrs) + sizeof(ints) + sizeof(om));
  unsigned char *o = k.data();
  std::memcpy(o, &P, sizeof(P));
  std::memcpy(o += sizeof(P), ptrs, sizeof(ptrs));
  std::memcpy(o += sizeof(ptrs), ints, sizeof(ints));
  std::memcpy(o + sizeof(ints), &om, sizeof(om));
  return k;
}
extern "C" {
// capture x = csweeps damped-Jacobi sweeps from x = 0 on c's stream; a refused capture leaves the
// plain launches in place (cgraph_failed)
int coarse_graph_capture(gls_ctx *c, gls_ctx *g, const double *b, double *x, double *y, int pre, double om) {
  auto &mg = c->mg;
  hipStream_t s = c->stream;
  GLS_TRY(ensure_diag(g));
  GLS_TRY(g->smooth_f32 ? ensure_qdata32(g, !g->smooth_oseen) : ensure_qdata(g));
  if (g->use_colors && g->acc.n != (size_t)g->n_dofs) GLS_TRY(g->acc.alloc((size_t)g->n_dofs));  // no malloc in capture
  const bool tim = g->timing;
  g->timing = false;  // no event records inside the capture
  hipGraph_t gr = nullptr;
  int rc = GLS_OK;
  hipError_t e = hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
  if (e == hipSuccess) {
    if (hipError_t e1 = gls::mg_jacobi_update(x, b, nullptr, g->diag.p, om, g->n_dofs, 1, s); e1 != hipSuccess)
      e = e1;
    for (int it = 1; it < pre && rc == GLS_OK && e == hipSuccess; ++it) rc = smoother_sweep(g, x, b, y, om);
    const hipError_t e2 = hipStreamEndCapture(s, &gr);
    if (e == hipSuccess) e = e2;
  }
  g->timing = tim;
  hipGraphExec_t ex = nullptr;
  if (rc == GLS_OK && e == hipSuccess && gr) e = hipGraphInstantiate(&ex, gr, nullptr, nullptr, 0);
  if (gr) (void)hipGraphDestroy(gr);
  if (rc != GLS_OK || e != hipSuccess || !ex) {
    (void)hipGetLastError();
    if (ex) (void)hipGraphExecDestroy(ex);
    mg.cgraph_failed = true;
    if (std::getenv("GLS_MG_VERBOSE")) std::printf("mg: coarse graph capture refused (%s)\n", hipGetErrorString(e));
    return GLS_OK;
  }
  mg.cgraph.h = ex;
  mg.cgraph_key = coarse_graph_key(g, b, x, y, pre, om);
  return GLS_OK;
}

// in-place sum over ranks of a device vector through c's transport (RCCL: one call; callback transports
// through their reduction buffer in chunks of GLS_RED_BUF_MIN values)
int dist_allreduce_vector(gls_ctx *c, double *v, int64_t n) {
  auto &D = c->dist;
  if (!D.on) return GLS_OK;
  if (D.comm) {
    if (D.allreduce(D.user, v, (int)n) != 0) return set_err(GLS_ECOMM, "vector all-reduce failed");
    return GLS_OK;
  }
  hipStream_t s = c->stream;
  for (int64_t o = 0; o < n; o += GLS_RED_BUF_MIN) {
    const int len = (int)std::min<int64_t>(GLS_RED_BUF_MIN, n - o);
    HIP_TRY(hipMemcpyAsync(D.red_buf, v + o, sizeof(double) * len, hipMemcpyDeviceToDevice, s));
    if (D.allreduce(D.user, D.red_buf, len) != 0) return set_err(GLS_ECOMM, "vector all-reduce failed");
    HIP_TRY(hipMemcpyAsync(v + o, D.red_buf, sizeof(double) * len, hipMemcpyDeviceToDevice, s));
  }
  return GLS_OK;
}
// the replica's copy of a fine-level state vector: each replica DoF takes its injection source's value on
// the one rank that owns that fine DoF (0 elsewhere), then the sum over ranks
int rep2_inject(gls_ctx *c, const double *loc, double *glob) {
  auto &mg = c->mg;
  const int64_t ng = mg.rep2->n_dofs, ni = (int64_t)mg.r2inj_c.n;
  HIP_TRY(gls::vec_fill(glob, ng, 0.0, c->stream));
  if (ni) {
    HIP_TRY(gls::vec_pack_dofs(loc, mg.r2inj_f.p, ni, mg.rep_tmp.p, c->stream));
    HIP_TRY(gls::vec_unpack_dofs(glob, mg.r2inj_c.p, ni, mg.rep_tmp.p, c->stream));
  }
  return dist_allreduce_vector(c, glob, ng);
}
// one V-cycle with the replica hierarchy below the distributed fine level (gls_mg_attach_replica)
int mg_vcycle_rep2(gls_ctx *c, const double *b, double *x) {
  auto &mg = c->mg;
  gls_ctx *r = mg.rep2;
  const int64_t n = c->n_dofs, ng = r->n_dofs;
  hipStream_t s = c->stream;
  GLS_TRY(ensure_diag(c));
  double *y = mgbuf(c, 0, MB_Y);
  double *zs = mg.ilu_smooth && c->ilu.on && !c->ilu.probe_only ? mgbuf(c, 0, MB_BOX) : nullptr;
  const int pre = mg.lpre[0], post = mg.lpost[0];
  if (pre > 0 && zs) {
    GLS_TRY(ensure_ilu(c));
    GLS_TRY(apply_ilu(c, b, x));
    for (int it = 1; it < pre; ++it) GLS_TRY(smoother_sweep(c, x, b, y, mg.omega, zs));
  } else if (pre > 0) {
    HIP_TRY(gls::mg_jacobi_update(x, b, nullptr, c->diag.p, mg.omega, n, 1, s));
    for (int it = 1; it < pre; ++it) GLS_TRY(smoother_sweep(c, x, b, y, mg.omega));
  } else {
    HIP_TRY(gls::vec_fill(x, n, 0.0, s));
  }
  if (pre > 0) GLS_TRY(smoother_apply(c, x, y, b));  // y = b - A x
  else HIP_TRY(gls::vec_copy(y, b, n, s));
  // restriction: the owned rows' part of P^T y on this rank, summed over ranks
  HIP_TRY(gls::vec_csr_spmv(mg.rep_b.p, y, mg.r2r_off.p, mg.r2r_col.p, mg.r2r_w.p, ng, false, s, mg.r2r_lane));
  GLS_TRY(dist_allreduce_vector(c, mg.rep_b.p, ng));
  HIP_TRY(gls::vec_set_indexed(mg.rep_b.p, r->con_dofs.p, nullptr, (int64_t)r->con_dofs.n, s));
  if (mg.direct_ok) {  // the replica level is the coarsest: its exact solve, every rank
    const double one = 1.0, zero = 0.0;
    if (rocblas_set_stream(mg.blas, s) != rocblas_status_success ||
        rocblas_dgemv(mg.blas, rocblas_operation_none, (rocblas_int)ng, (rocblas_int)ng, &one, mg.probe.p,
                      (rocblas_int)ng, mg.rep_b.p, 1, &zero, mg.rep_x.p, 1) != rocblas_status_success)
      return set_err(GLS_EHIP, "rocblas_dgemv failed");
  } else {
    GLS_TRY(gls_apply_preconditioner(r, mg.rep_b.p, mg.rep_x.p));  // the replica's own V-cycle, every rank
  }
  HIP_TRY(gls::vec_csr_spmv(y, mg.rep_x.p, mg.r2p_off.p, mg.r2p_col.p, mg.r2p_w.p, n, false, s, mg.r2p_lane));
  HIP_TRY(gls::vec_set_indexed(y, c->con_dofs.p, nullptr, (int64_t)c->con_dofs.n, s));
  HIP_TRY(gls::vec_axpy(x, 1.0, y, n, s));
  for (int it = 0; it < post; ++it) GLS_TRY(smoother_sweep(c, x, b, y, mg.omega, zs));
  return GLS_OK;
}

// glob (replica numbering, every rank) = the coarsest distributed level's vector loc: each rank scatters
// its owned rows into a zeroed copy, then one sum all-reduce (RCCL: in place; callback transports
// through their reduction buffer in chunks of 256 values)
int replica_gather(gls_ctx *c, const double *loc, double *glob) {
  auto &mg = c->mg;
  gls_ctx *g = mg.lev.back();
  auto &D = g->dist;
  const int64_t ng = mg.replica->n_dofs, no = (int64_t)mg.rep_own_loc.n;
  hipStream_t s = c->stream;
  HIP_TRY(gls::vec_fill(glob, ng, 0.0, s));
  if (no) {
    HIP_TRY(gls::vec_pack_dofs(loc, mg.rep_own_loc.p, no, mg.rep_tmp.p, s));
    HIP_TRY(gls::vec_unpack_dofs(glob, mg.rep_own_glob.p, no, mg.rep_tmp.p, s));
  }
  if (D.comm) {
    if (D.allreduce(D.user, glob, (int)ng) != 0) return set_err(GLS_ECOMM, "replica all-reduce failed");
    return GLS_OK;
  }
  for (int64_t o = 0; o < ng; o += 256) {
    const int len = (int)std::min<int64_t>(256, ng - o);
    HIP_TRY(hipMemcpyAsync(D.red_buf, glob + o, sizeof(double) * len, hipMemcpyDeviceToDevice, s));
    if (D.allreduce(D.user, D.red_buf, len) != 0) return set_err(GLS_ECOMM, "replica all-reduce failed");
    HIP_TRY(hipMemcpyAsync(glob + o, D.red_buf, sizeof(double) * len, hipMemcpyDeviceToDevice, s));
  }
  return GLS_OK;
}

// x = V-cycle(b) on level l (x, b are level-l vectors)
int mg_vcycle(gls_ctx *c, int l, const double *b, double *x) {
  auto &mg = c->mg;
  const int L = (int)mg.lev.size();
  gls_ctx *g = mg.lev[l];
  GLS_TRY(ensure_diag(g));
  const int64_t n = g->n_dofs;
  double *y = mgbuf(c, l, MB_Y);
  const double *d = g->diag.p;
  hipStream_t s = c->stream;
  if (l == L - 1 && mg.replica) {  // the replica's cycle on the gathered right-hand side, every rank
    GLS_TRY(replica_gather(c, b, mg.rep_b.p));
    GLS_TRY(gls_apply_preconditioner(mg.replica, mg.rep_b.p, mg.rep_x.p));
    HIP_TRY(gls::vec_pack_dofs(mg.rep_x.p, mg.rep_map.p, n, x, c->stream));
    return GLS_OK;
  }
  if (l == L - 1 && mg.direct_ok) GLS_TRY(coarse_lu32_finish(c));
  if (l == L - 1 && mg.direct_ok) {  // exact coarsest-level solve
    if (mg.lu32) {  // the FP32 factor / inverse, in the matrix's order (banded: the CSR's Cuthill-McKee order)
      const double *bb = b;
      double *xx = x;
      if (mg.lu_cm) {
        HIP_TRY(gls::vec_permute(mg.lu_tmp.p, b, g->ilu.perm.p, n, 0, c->stream));
        bb = xx = mg.lu_tmp.p;
      }
      if (mg.lu32_npvt) {  // x = U^-1 L^-1 b
        const int bl = mg.lu_cm ? (int)mg.lu_bl : -1, bu = mg.lu_cm ? (int)mg.lu_bu : -1;
        HIP_TRY(gls::vec_to_f32(bb, mg.x32.p, n, c->stream));
        HIP_TRY(gls::dense_lu_solve_f32(mg.probe32.p, (int)n, mg.x32.p, c->stream, bl, bu));
        if (mg.lu32_refine) {  // r = b - A x (the pinned FP64 matrix), x += LU^-1 r
          const double one = 1.0, mone = -1.0;
          double *r = mg.chk32.p, *x0 = mg.chk32.p + n;
          HIP_TRY(gls::vec_from_f32(mg.x32.p, x0, n, c->stream));
          HIP_TRY(gls::vec_copy(r, bb, n, c->stream));
          if (rocblas_set_stream(mg.blas, c->stream) != rocblas_status_success ||
              rocblas_dgemv(mg.blas, rocblas_operation_none, (rocblas_int)n, (rocblas_int)n, &mone, mg.probe.p,
                            (rocblas_int)n, x0, 1, &one, r, 1) != rocblas_status_success)
            return set_err(GLS_EHIP, "rocblas_dgemv failed");
          HIP_TRY(gls::vec_to_f32(r, mg.x32.p, n, c->stream));
          HIP_TRY(gls::dense_lu_solve_f32(mg.probe32.p, (int)n, mg.x32.p, c->stream, bl, bu));
          HIP_TRY(gls::vec_from_f32(mg.x32.p, xx, n, c->stream));
          HIP_TRY(gls::vec_axpy(xx, 1.0, x0, n, c->stream));
        } else {
          HIP_TRY(gls::vec_from_f32(mg.x32.p, xx, n, c->stream));
        }
      } else {  // x = A^-1 b
        const float one = 1.0f, zero = 0.0f;
        HIP_TRY(gls::vec_to_f32(bb, mg.b32.p, n, c->stream));
        if (rocblas_set_stream(mg.blas, c->stream) != rocblas_status_success ||
            rocblas_sgemv(mg.blas, rocblas_operation_none, (rocblas_int)n, (rocblas_int)n, &one, mg.probe32.p,
                          (rocblas_int)n, mg.b32.p, 1, &zero, mg.x32.p, 1) != rocblas_status_success)
          return set_err(GLS_EHIP, "rocblas_sgemv failed");
        HIP_TRY(gls::vec_from_f32(mg.x32.p, xx, n, c->stream));
      }
      if (mg.lu_cm) HIP_TRY(gls::vec_permute(x, mg.lu_tmp.p, g->ilu.perm.p, n, 1, c->stream));
      HIP_TRY(hipMemsetAsync(x + (int64_t)g->dim * g->n_vnodes, 0, sizeof(double), c->stream));  // pinned: no correction
      return GLS_OK;
    }
    if (mg.lu) {
      const double one = 1.0, zero = 0.0;
      if (rocblas_set_stream(mg.blas, c->stream) != rocblas_status_success ||
          rocblas_dgemv(mg.blas, rocblas_operation_none, (rocblas_int)n, (rocblas_int)n, &one, mg.probe.p,
                        (rocblas_int)n, b, 1, &zero, x, 1) != rocblas_status_success)
        return set_err(GLS_EHIP, "rocblas_dgemv failed");
    } else {
      HIP_TRY(gls::mg_dense_apply(mg.aug.p, (int)n, b, x, c->stream));
    }
    return GLS_OK;
  }
  const int pre = l == L - 1 ? mg.csweeps : mg.lpre[(size_t)l];
  const double om = l == L - 1 ? mg.comega : mg.omega;
  if (l == L - 1 && l > 0 && pre > 1 && coarse_graph_eligible(c, g, b, x)) {
    GLS_TRY(ensure_diag(g));  // contents the replay reads: current for this state
    GLS_TRY(g->smooth_f32 ? ensure_qdata32(g, !g->smooth_oseen) : ensure_qdata(g));
    if (mg.cgraph.h && mg.cgraph_key != coarse_graph_key(g, b, x, y, pre, om)) mg.cgraph.reset();
    if (!mg.cgraph.h) GLS_TRY(coarse_graph_capture(c, g, b, x, y, pre, om));
    if (mg.cgraph.h) {
      HIP_TRY(hipGraphLaunch(mg.cgraph.h, s));
      return GLS_OK;
    }
  }
  // one pre-sweep from 0 on a fused level: x = omega D^-1 b is formed inside the residual's J.v
  const bool first_fused = pre == 1 && l < L - 1 && first_sweep_fusable(g);
  double *zs = mg.ilu_smooth && g->ilu.on && !g->ilu.probe_only ? mgbuf(c, l, MB_BOX) : nullptr;  // ILU smoothing scratch
  if (pre > 0 && !first_fused && zs) {
    GLS_TRY(ensure_ilu(g));
    GLS_TRY(apply_ilu(g, b, x));  // first sweep from x = 0: x = M^-1 b
    for (int it = 1; it < pre; ++it) GLS_TRY(smoother_sweep(g, x, b, y, om, zs));
  } else if (pre > 0 && !first_fused) {
    HIP_TRY(gls::mg_jacobi_update(x, b, nullptr, d, om, n, 1, s));  // first sweep from x = 0
    for (int it = 1; it < pre; ++it) GLS_TRY(smoother_sweep(g, x, b, y, om));
  } else if (pre == 0) {
    HIP_TRY(gls::vec_fill(x, n, 0.0, s));
  }
  if (l == L - 1) return GLS_OK;
  // residual -> coarse right-hand side: restrict the owned rows, export-add coarse ghost rows
  if (first_fused) {
    GLS_TRY(jacobian_apply_f32(g, x, y, b, om, g->smooth_oseen));  // x = omega D^-1 b, y = b - A x
  } else if (pre > 0) {
    GLS_TRY(smoother_apply(g, x, y, b));  // y = b - A x
  } else {
    HIP_TRY(gls::vec_copy(y, b, n, s));  // x = 0: the residual is b
  }
  gls_ctx *h = mg.lev[l + 1];
  double *bc = mgbuf(c, l + 1, MB_B), *xc = mgbuf(c, l + 1, MB_X);
  GLS_TRY(mg_restrict(c, l, y, bc));
  HIP_TRY(gls::vec_set_indexed(bc, h->con_dofs.p, nullptr, (int64_t)h->con_dofs.n, s));
  GLS_TRY(mg_vcycle(c, l + 1, bc, xc));
  // prolongate the coarse correction (ghost values imported first). x += P xc in the transfer's
  // store on one rank: the coarse correction vanishes on the coarse Dirichlet rows (zero rhs rows,
  // D_c-scaled sweeps) and the nested Qk interpolation maps them onto the fine Dirichlet rows, so
  // P xc is exactly 0 there, as the zeroing below makes it in the general path
  if (mg_prolong_add_ok(c, l)) {
    GLS_TRY(mg_prolong(c, l, xc, x, true));
  } else {
    GLS_TRY(mg_prolong(c, l, xc, y));
    HIP_TRY(gls::vec_set_indexed(y, g->con_dofs.p, nullptr, (int64_t)g->con_dofs.n, s));
    HIP_TRY(gls::vec_axpy(x, 1.0, y, n, s));
  }
  for (int it = 0; it < mg.lpost[(size_t)l]; ++it) GLS_TRY(smoother_sweep(g, x, b, y, mg.omega, zs));
  return GLS_OK;
}

#define RS_TRY(x)                                                                        \
  do {                                                                                   \
    const rocsparse_status rs_ = (x);                                                    \
    if (rs_ != rocsparse_status_success) return set_err(GLS_EHIP, "%s: rocsparse status %d", #x, (int)rs_); \
  } while (0)

// assembled ILU(0): probe the operator into the CSR values (one J.v per color and DoF slot), perturb
// the diagonal, factor in place; once per Jacobian state (invalidated with the diagonal)
// the per-cell path on one rank: all probes in batches of B vectors, each step one launch over the batch
// (unit vectors, hanging-line values, the per-cell J.v with zero cell batches skipped, the ordered
// element-vector sums, condensation, constrained rows, extraction) -- the same operations per probe as
// gls_jacobian_apply, without one launch sequence per probe
static int ilu_probe_batched(gls_ctx *c) {
  auto &I = c->ilu;
  const int64_t n = c->n_dofs;
  hipStream_t s = c->stream;
  if (!c->u) return set_err(GLS_EINVAL, "gls_set_state was not called");
  GLS_TRY(ensure_element_maps(c));
  if (c->con_dofs.n) GLS_TRY(ensure_diag(c));
  const int dim = c->dim, nv = gls::ipow(c->k + 1, dim), np = gls::ipow(c->kp + 1, dim);
  const int64_t el = (int64_t)nv * dim + np, evs = (int64_t)c->n_cells * el;
  const char *bs = std::getenv("GLS_ILU_PROBE_BATCH");
  const int64_t budget = (int64_t)1 << 31;  // bytes of V, C V, Y and the element vectors per batch
  int B = bs ? std::atoi(bs) : (int)std::min<int64_t>(I.n_probes, std::max<int64_t>(1, budget / (8 * (3 * n + evs))));
  B = std::max(1, std::min(B, I.n_probes));
  if (I.bV.n < (size_t)B * n) {
    GLS_TRY(I.bV.alloc((size_t)B * n));
    GLS_TRY(I.bY.alloc((size_t)B * n));
  }
  if (c->hang.on && I.bC.n < (size_t)B * n) GLS_TRY(I.bC.alloc((size_t)B * n));
  if (c->bev.n < (size_t)B * evs) GLS_TRY(c->bev.alloc((size_t)B * evs));
  const int cb = gls::cell_kernel_cells_per_block(dim, c->k, c->nq1d, true), nblk = (c->n_cells + cb - 1) / cb;
  if (c->bact.n < (size_t)B * nblk) GLS_TRY(c->bact.alloc((size_t)B * nblk));
  if (I.fill > 0) HIP_TRY(gls::vec_fill(I.val.p, I.nnz, 0.0, s));  // fill-in positions start at 0
  // recorded activity (GLS_ILU_PROBE_LIST=0: every (probe, batch) block tests its vector, every time)
  const char *wl_env = std::getenv("GLS_ILU_PROBE_LIST");
  const bool wl_on = !(wl_env && wl_env[0] == '0');
  const bool use_list = wl_on && !I.woff.empty() && I.wB == B && I.wnblk == nblk;
  const bool record = wl_on && !use_list;
  // listed blocks read u, grad u, tau and R_s from the linearization cache of this state (the diagonal pass writes
  // it for every cell; not on forests, whose cache covers the cells outside the bricks only)
  bool cq_probe = use_list && cell_cache_on(c) && !c->oct.on;
  if (cq_probe) {
    GLS_TRY(ensure_diag(c));
    cq_probe = c->cq_valid && c->cq.n == cell_cache_size(c);
  }
  std::vector<int32_t> hlist;
  std::vector<int64_t> hoff;
  std::vector<uint8_t> hact;
  if (record) {
    GLS_TRY(I.wact.alloc((size_t)I.n_probes * nblk));
    hoff.push_back(0);
  }
  for (int p0 = 0; p0 < I.n_probes; p0 += B) {
    const int nb = std::min(B, I.n_probes - p0);
    HIP_TRY(gls::vec_fill(I.bV.p, (int64_t)nb * n, 0.0, s));
    const int64_t d0 = I.pdoff[(size_t)p0], d1 = I.pdoff[(size_t)(p0 + nb)];
    HIP_TRY(gls::probe_set_batched(I.bV.p, n, I.pdofs.p + d0, I.pdpid.p + d0, p0, d1 - d0, s));
    const double *Cv = I.bV.p;
    if (c->hang.on) {  // C v (hanging entries interpolated from their masters) in a copy: the constrained
      // rows below take the probe vector itself, as gls_jacobian_apply does
      HIP_TRY(gls::vec_copy(I.bC.p, I.bV.p, (int64_t)nb * n, s));
      HIP_TRY(gls::vec_csr_gather_set_b(I.bC.p, c->hang.dof.p, c->hang.ooff.p, c->hang.omaster.p, c->hang.ow.p,
                                        (int64_t)c->hang.dof.n, nb, n, s));
      Cv = I.bC.p;
    }
    gls::OpParams P = make_params(c, true);
    P.v = Cv;
    P.y = I.bY.p;
    P.hmask = c->hang.on ? c->hang.hmask.p : nullptr;
    P.ev = c->bev.p;
    // (the first, recording run re-derives the linearization in every (probe, cell batch) block: with all blocks
    // launched, reading the cache moved more bytes than the state gathers -- configs[4]'s ILU setup ran 1.4 ms per
    // Newton step slower; the listed runs read it, profiles/r05_ab_probe_cache.txt)
    P.bv_stride = n;
    P.bev_stride = evs;
    P.n_probe = nb;
    const int chunk = p0 / B;
    P.bact = use_list ? I.wact.p + (size_t)p0 * nblk : c->bact.p;
    if (use_list) {
      P.work = I.wlist.p + 2 * I.woff[(size_t)chunk];
      P.n_work = (int)(I.woff[(size_t)chunk + 1] - I.woff[(size_t)chunk]);
      if (cq_probe) {
        P.cq = c->cq.p;
        P.cq_mode = 2;
      }
    }
    if (!use_list || P.n_work > 0) {
      TimedLaunch t(c, (int)gls::MODE_JV);
      HIP_TRY(gls::launch_cell_kernel(c->dim, c->k, c->kp, c->nq1d, gls::MODE_JV, P, c->tables, s));
    }
    if (record) {  // this chunk's flags: kept on the device for the gathers, listed on the host
      HIP_TRY(hipMemcpyAsync(I.wact.p + (size_t)p0 * nblk, c->bact.p, (size_t)nb * nblk, hipMemcpyDeviceToDevice, s));
      hact.resize((size_t)nb * nblk);
      HIP_TRY(hipMemcpyAsync(hact.data(), c->bact.p, hact.size(), hipMemcpyDeviceToHost, s));
      HIP_TRY(hipStreamSynchronize(s));
      for (int v = 0; v < nb; ++v)
        for (int64_t b = 0; b < nblk; ++b)
          if (hact[(size_t)v * nblk + b]) {
            hlist.push_back(v);
            hlist.push_back((int32_t)b);
          }
      hoff.push_back((int64_t)hlist.size() / 2);
    }
    HIP_TRY(gls::gather_element_vectors_b(I.bY.p, c->bev.p, c->ev_voff.p, c->ev_vslot.p, c->n_vnodes, c->ev_poff.p,
                                          c->ev_pslot.p, c->n_pnodes, c->dim, nb, n, evs, P.bact, el, cb, nblk, s));
    if (c->hang.on)
      HIP_TRY(gls::vec_csr_condense_b(I.bY.p, c->hang.tm.p, c->hang.toff.p, c->hang.tdof.p, c->hang.tw.p,
                                      (int64_t)c->hang.tm.n, nb, n, s));
    HIP_TRY(gls::vec_gather_scale_set_b(I.bY.p, c->diag.p, I.bV.p, c->con_dofs.p, (int64_t)c->con_dofs.n, nb, n, s));
    const int64_t e0 = I.peoff[(size_t)p0], e1 = I.peoff[(size_t)(p0 + nb)];
    HIP_TRY(gls::probe_extract_batched(I.val.p, I.pent.p + e0, I.prow.p + e0, I.pepid.p + e0, p0, e1 - e0, I.bY.p, n, s));
  }
  if (I.ghost_diag.n) HIP_TRY(gls::vec_set_const_indexed64(I.val.p, I.ghost_diag.p, (int64_t)I.ghost_diag.n, 1.0, s));
  if (record) {
    GLS_TRY(I.wlist.upload(hlist.data(), hlist.size()));
    I.woff.swap(hoff);
    I.wB = B;
    I.wnblk = nblk;
  }
  return GLS_OK;
}

static int ilu_probe(gls_ctx *c) {  // I.val <- the operator's CSR values (gls_jacobian_apply)
  auto &I = c->ilu;
  const int64_t n = c->n_dofs;
  hipStream_t s = c->stream;
  if (!c->dist.on && !c->use_brick && !std::getenv("GLS_ILU_PROBE_LOOP")) return ilu_probe_batched(c);
  if (I.fill > 0 || c->dist.on) HIP_TRY(gls::vec_fill(I.val.p, I.nnz, 0.0, s));  // fill-in positions start at 0
  // across ranks the constrained rows' diagonal is the exchanged one: computed before the local probes
  if (c->dist.on && (c->con_dofs.n || I.complete)) GLS_TRY(ensure_diag(c));
  c->probe_local = c->dist.on;  // the probe's J.v: the rank's cells only, no ghost exchange
  struct ProbeLocalGuard {      // every exit path (errors included) restores the exchanging operator
    gls_ctx *c;
    ~ProbeLocalGuard() { c->probe_local = false; }
  } guard{c};
  auto &D = c->dist;
  const int rounds = I.complete ? I.n_rounds : I.n_probes;
  for (int p = 0; p < rounds; ++p) {
    if (p < I.n_probes) {
      HIP_TRY(gls::vec_fill(I.vbuf.p, n, 0.0, s));
      HIP_TRY(gls::vec_set_const_indexed(I.vbuf.p, I.pdofs.p + I.pdoff[(size_t)p],
                                         I.pdoff[(size_t)p + 1] - I.pdoff[(size_t)p], 1.0, s));
      GLS_TRY(gls_jacobian_apply(c, I.vbuf.p, I.ybuf.p));
      HIP_TRY(gls::csr_probe_extract(I.val.p, I.pent.p + I.peoff[(size_t)p], I.prow.p + I.peoff[(size_t)p],
                                     I.peoff[(size_t)p + 1] - I.peoff[(size_t)p], I.ybuf.p, s, c->dist.on));
    }
    if (!I.complete) continue;
    // ghost rows of this probe (the local cells' part of a neighbour's owned rows) to their owners
    if (p < I.n_probes) HIP_TRY(gls::vec_pack_dofs(I.ybuf.p, D.recv_nodes.p, D.n_recv, D.recv_buf, s));
    else if (D.n_recv) HIP_TRY(gls::vec_fill(D.recv_buf, D.n_recv, 0.0, s));
    if (D.xchg(D.user, 1) != 0) return set_err(GLS_ECOMM, "ILU probe exchange failed");
    const int64_t a = I.rr[(size_t)p], b = I.rr[(size_t)p + 1];
    if (b > a) HIP_TRY(gls::vec_add_pos_ordered(I.val.p, I.ru.p + a, I.ruoff.p + a, I.rslot.p, b - a, D.send_buf, s));
  }
  c->probe_local = false;
  if (I.ghost_diag.n) HIP_TRY(gls::vec_set_const_indexed64(I.val.p, I.ghost_diag.p, (int64_t)I.ghost_diag.n, 1.0, s));
  return GLS_OK;
}
static int apply_ilu(gls_ctx *c, const double *v, double *z);
static int ensure_ilu(gls_ctx *c) {
  auto &I = c->ilu;
  if (!I.on || I.valid) return GLS_OK;
  const int64_t n = c->n_dofs;
  hipStream_t s = c->stream;
  const bool verbose = std::getenv("GLS_ILU_VERBOSE") != nullptr;
  auto now = [&]() {
    if (verbose) (void)hipStreamSynchronize(s);
    return std::chrono::steady_clock::now();
  };
  const auto t0 = now();
  GLS_TRY(ilu_probe(c));
  HIP_TRY(gls::csr_diag_perturb(I.val.p, I.didx.p, n, I.athresh, I.rthresh, s));
  const auto t1 = now();
  const rocsparse_int m = (rocsparse_int)n, nnz = (rocsparse_int)I.nnz;
  if (I.h) RS_TRY(rocsparse_set_stream(I.h, s));  // (no handle past 2^31 entries: multicolor kernels only)
  if (I.mc_factor)
    HIP_TRY(gls::ilu_mc_factor(I.mc_grow.p, I.mc_cg.data(), (int)I.mc_cg.size() - 1, I.rowp.p, I.col.p, I.val.p,
                               I.mc_lsp.p, I.didx.p, I.boost_tol, I.boost_val, I.mc_moff.p,
                               I.mc_map.n ? I.mc_map.p : nullptr, I.mc_compact, I.rdiag.p, s));
  else
    RS_TRY(rocsparse_dcsrilu0(I.h, m, nnz, I.dA, I.val.p, I.rowp32.p, I.col.p, I.info, rocsparse_solve_policy_auto, I.work.p));
  I.valid = true;
  if (verbose) {
    const auto t2 = now();
    rocsparse_int zp = -1;
    const rocsparse_status st = I.h ? rocsparse_csrilu0_zero_pivot(I.h, I.info, &zp) : rocsparse_status_success;
    GLS_TRY(apply_ilu(c, I.ybuf.p, I.ybuf.p == nullptr ? nullptr : c->tmp1.p ? c->tmp1.p : I.ybuf.p));
    const auto t3 = now();
    std::printf("ilu: %d probes %.2f ms, csrilu0 %.2f ms (zero pivot status %d at %d), one apply %.3f ms\n", I.n_probes,
                std::chrono::duration<double, std::milli>(t1 - t0).count(),
                std::chrono::duration<double, std::milli>(t2 - t1).count(), (int)st, (int)zp,
                std::chrono::duration<double, std::milli>(t3 - t2).count());
  }
  return GLS_OK;
}
static int apply_ilu(gls_ctx *c, const double *v, double *z) {
  auto &I = c->ilu;
  const rocsparse_int m = (rocsparse_int)c->n_dofs, nnz = (rocsparse_int)I.nnz;
  const double one = 1.0;
  if (I.h) RS_TRY(rocsparse_set_stream(I.h, c->stream));
  // z = P^T U^-1 L^-1 P v (P: the Cuthill-McKee renumbering the factors live in)
  HIP_TRY(gls::vec_permute(I.vbuf.p, v, I.perm.p, c->n_dofs, 0, c->stream));
  if (I.mc_solve) {  // multicolor order: color-by-color solves (gls_ilu_kernels.hip)
    HIP_TRY(gls::ilu_mc_solve(I.mc_desc.p, I.mc_cg.data(), (int)I.mc_cg.size() - 1, I.col.p, I.val.p, I.vbuf.p,
                              I.tbuf.p, I.vbuf.p, I.mc_wl.data(), I.mc_wu.data(), c->stream));
    HIP_TRY(gls::vec_permute(z, I.vbuf.p, I.perm.p, c->n_dofs, 1, c->stream));
    return GLS_OK;
  }
  RS_TRY(rocsparse_dcsrsv_solve(I.h, rocsparse_operation_none, m, nnz, &one, I.dL, I.val.p, I.rowp32.p, I.col.p, I.info,
                                I.vbuf.p, I.tbuf.p, rocsparse_solve_policy_auto, I.work.p));
  RS_TRY(rocsparse_dcsrsv_solve(I.h, rocsparse_operation_none, m, nnz, &one, I.dU, I.val.p, I.rowp32.p, I.col.p, I.info,
                                I.tbuf.p, I.vbuf.p, rocsparse_solve_policy_auto, I.work.p));
  HIP_TRY(gls::vec_permute(z, I.vbuf.p, I.perm.p, c->n_dofs, 1, c->stream));
  return GLS_OK;
}

// z = M^{-1} v : Jacobi, assembled ILU(0) or a multigrid V-cycle when attached
int apply_prec(gls_ctx *c, const double *v, double *z) {
  if (c->mg.on && c->mg.rep_csr) return mg_vcycle_rep2(c, v, z);
  if (c->mg.on) return mg_vcycle(c, 0, v, z);
  if (c->ilu.on && !c->ilu.probe_only) return apply_ilu(c, v, z);
  HIP_TRY(gls::vec_div(z, v, c->diag.p, c->n_dofs, c->stream));
  return GLS_OK;
}
}  // namespace

int gls_apply_preconditioner(gls_ctx *c, const double *v, double *z) {
  GLS_TRY(check_ctx(c));
  if (!v || !z || v == z) return set_err(GLS_EINVAL, "v/z null or aliased");
  GLS_TRY(ensure_diag(c));
  if (c->mg.on) GLS_TRY(mg_prepare(c));
  GLS_TRY(ensure_ilu(c));
  return apply_prec(c, v, z);
}

int gls_mg_transfer(gls_ctx *c, int level, int direction, const double *in, double *out) {
  GLS_TRY(check_ctx(c));
  auto &mg = c->mg;
  if (!mg.on) return set_err(GLS_EINVAL, "gls_mg_transfer: no multigrid attached");
  if (level < 0 || level + 1 >= (int)mg.lev.size() || (direction != 0 && direction != 1) || !in || !out || in == out)
    return set_err(GLS_EINVAL, "gls_mg_transfer: bad level / direction / pointers");
  if (direction == 0) return mg_restrict(c, level, in, out);
  double *xc = mgbuf(c, level + 1, MB_X);  // ghost import writes into the coarse vector: work on a copy
  HIP_TRY(gls::vec_copy(xc, in, mg.lev[(size_t)level + 1]->n_dofs, c->stream));
  return mg_prolong(c, level, xc, out);
}

// --------------------------------------------------------------------------------------------
// Kelly error indicator (navier_stokes_base.cc:612-652)
// --------------------------------------------------------------------------------------------
namespace {
// face neighbours of a conforming mesh: faces match by their vertex node ids (periodic wraps share
// node ids, so a wrapped face has its periodic neighbour)
int build_face_neighbours(gls_ctx *c) {
  const int dim = c->dim, k = c->k, nv = gls::ipow(k + 1, dim);
  std::vector<int32_t> cn((size_t)c->n_cells * nv);
  if (!cn.empty() && hipMemcpy(cn.data(), c->cell_vnodes.p, cn.size() * sizeof(int32_t), hipMemcpyDeviceToHost) != hipSuccess)
    return set_err(GLS_EHIP, "cell map download failed");
  std::map<std::array<int32_t, 4>, std::pair<int, int>> open;  // face key -> (cell, face slot)
  std::vector<int32_t> nbr((size_t)c->n_cells * 2 * dim, -1);
  for (int cell = 0; cell < c->n_cells; ++cell)
    for (int d = 0; d < dim; ++d)
      for (int sd = 0; sd < 2; ++sd) {
        std::array<int32_t, 4> key = {-1, -1, -1, -1};
        int nk = 0;
        for (int v = 0; v < (1 << dim); ++v) {  // cell vertices with coordinate d on side sd
          if (((v >> d) & 1) != sd) continue;
          int a = 0, st = 1;
          for (int e = 0; e < dim; ++e, st *= k + 1) a += ((v >> e) & 1) * k * st;
          key[nk++] = cn[(size_t)cell * nv + a];
        }
        std::sort(key.begin(), key.begin() + nk);
        auto it = open.find(key);
        if (it == open.end()) {
          open.emplace(key, std::make_pair(cell, 2 * d + sd));
        } else {
          nbr[(size_t)cell * 2 * dim + 2 * d + sd] = it->second.first;
          nbr[(size_t)it->second.first * 2 * dim + it->second.second] = cell;
          open.erase(it);
        }
      }
  return c->face_nbr.upload(nbr.data(), nbr.size());
}

gls::KellyTables kelly_tables(int m, int nq) {
  gls::KellyTables T;
  std::memset(&T, 0, sizeof(T));
  double xq[gls::kMaxQ1D], wq[gls::kMaxQ1D], xn[gls::kMaxNodes1D];
  gauss_points(nq, xq, wq);
  lobatto_points(m, xn);
  T.nq = nq;
  for (int a = 0; a <= m; ++a) {
    double v, dd, s2;
    for (int q = 0; q < nq; ++q) {
      lagrange_1d(m, xn, a, xq[q], v, dd, s2);
      T.V[q][a] = v;
    }
    lagrange_1d(m, xn, a, 0.0, v, dd, s2);
    T.De[0][a] = dd;
    lagrange_1d(m, xn, a, 1.0, v, dd, s2);
    T.De[1][a] = dd;
  }
  for (int q = 0; q < nq; ++q) {
    T.w[q] = wq[q];
    T.xq[q] = xq[q];
  }
  for (int a = 0; a <= m; ++a) T.xn[a] = xn[a];
  return T;
}
}  // namespace

int gls_kelly_estimate(gls_ctx *c, const double *sol, int variable, double *eta) {
  GLS_TRY(check_ctx(c));
  if (!sol || !eta || (variable != 0 && variable != 1)) return set_err(GLS_EINVAL, "gls_kelly_estimate: bad arguments");
  if (c->hang.on) return set_err(GLS_EINVAL, "gls_kelly_estimate: conforming meshes only (no hanging nodes)");
  if (c->map_degree > 0) return set_err(GLS_EINVAL, "gls_kelly_estimate: axis-aligned box cells only");
  if (c->nq1d + 1 > gls::kMaxQ1D) return set_err(GLS_EINVAL, "gls_kelly_estimate: face rule too large");
  if (!c->face_nbr.p && c->n_cells > 0) GLS_TRY(build_face_neighbours(c));
  const bool pres = variable == 1;
  const int m = pres ? c->kp : c->k;
  const int32_t *nodes = pres && c->cell_pnodes.p ? c->cell_pnodes.p : c->cell_vnodes.p;
  const gls::KellyTables T = kelly_tables(m, c->nq1d + 1);  // QGauss<dim-1>(n_q + 1)
  HIP_TRY(gls::launch_kelly(c->dim, m, nodes, c->face_nbr.p, c->geo.p, sol, c->n_cells, pres ? 1 : c->dim,
                            pres ? (int64_t)c->dim * c->n_vnodes : 0, pres ? 1 : c->dim, T, eta, c->stream));
  return GLS_OK;
}

// Kelly indicator on meshes with hanging faces (gls_octree_faces lists the face pieces): the face
// integrals on the device, then eta_K = sqrt(diam(K)/24 * sum of K's pieces) in a fixed order
int gls_kelly_estimate_faces(gls_ctx *c, const double *sol, int variable, int64_t n_faces, const int32_t *fa,
                             const int32_t *fb, const int32_t *fdir, const double *rect_a, const double *rect_b,
                             double *eta) {
  GLS_TRY(check_ctx(c));
  if (!sol || !eta || (variable != 0 && variable != 1) || n_faces < 0 || (n_faces > 0 && (!fa || !fb || !fdir || !rect_a || !rect_b)))
    return set_err(GLS_EINVAL, "gls_kelly_estimate_faces: bad arguments");
  if (c->map_degree > 0) return set_err(GLS_EINVAL, "gls_kelly_estimate_faces: axis-aligned box cells only");
  for (int64_t e = 0; e < n_faces; ++e)
    if (fa[e] < 0 || fa[e] >= c->n_cells || fb[e] < 0 || fb[e] >= c->n_cells || fdir[e] < 0 || fdir[e] >= c->dim)
      return set_err(GLS_EINVAL, "gls_kelly_estimate_faces: face %lld out of range", (long long)e);
  const bool pres = variable == 1;
  const int m = pres ? c->kp : c->k;
  const int32_t *nodes = pres && c->cell_pnodes.p ? c->cell_pnodes.p : c->cell_vnodes.p;
  const gls::KellyTables T = kelly_tables(m, c->nq1d + 1);  // QGauss<dim-1>(n_q + 1) on every piece
  DevBuf<int32_t> dfa, dfb, dfd;
  DevBuf<double> dra, drb, dfi;
  GLS_TRY(dfa.upload(fa, (size_t)n_faces));
  GLS_TRY(dfb.upload(fb, (size_t)n_faces));
  GLS_TRY(dfd.upload(fdir, (size_t)n_faces));
  GLS_TRY(dra.upload(rect_a, (size_t)n_faces * 4));
  GLS_TRY(drb.upload(rect_b, (size_t)n_faces * 4));
  GLS_TRY(dfi.alloc((size_t)std::max<int64_t>(n_faces, 1)));
  HIP_TRY(gls::launch_kelly_faces(c->dim, m, nodes, c->geo.p, sol, n_faces, dfa.p, dfb.p, dfd.p, dra.p, drb.p,
                                  pres ? 1 : c->dim, pres ? (int64_t)c->dim * c->n_vnodes : 0, pres ? 1 : c->dim, T,
                                  dfi.p, c->stream));
  std::vector<double> fi((size_t)n_faces), geo((size_t)c->n_cells * 4), acc((size_t)c->n_cells, 0.0);
  HIP_TRY(hipMemcpyAsync(fi.data(), dfi.p, sizeof(double) * fi.size(), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipMemcpyAsync(geo.data(), c->geo.p, sizeof(double) * geo.size(), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  for (int64_t e = 0; e < n_faces; ++e) {  // each piece counts for both of its cells
    acc[(size_t)fa[e]] += fi[(size_t)e];
    acc[(size_t)fb[e]] += fi[(size_t)e];
  }
  for (int64_t k = 0; k < c->n_cells; ++k) {
    double d2 = 0.0;
    for (int d = 0; d < c->dim; ++d) d2 += geo[(size_t)k * 4 + d] * geo[(size_t)k * 4 + d];
    acc[(size_t)k] = std::sqrt(std::sqrt(d2) / 24.0 * acc[(size_t)k]);
  }
  HIP_TRY(hipMemcpyAsync(eta, acc.data(), sizeof(double) * acc.size(), hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return GLS_OK;
}

// Kelly indicator on mapped (MappingQ) meshes, conforming or with hanging faces: the face pieces
// and their per-point geometry from gls_fe_space_kelly_faces (host), the jump integrals on the
// device, eta_K = sqrt(diam(K)/24 * sum of K's pieces) in a fixed order (eta: DEVICE pointer)
int gls_kelly_estimate_mapped(gls_ctx *c, const double *sol, int variable, int64_t n_pieces, int nqf, const int32_t *ca,
                              const int32_t *cb, const double *xi, const double *g, const double *jxw,
                              const double *cell_diam, double *eta) {
  GLS_TRY(check_ctx(c));
  if (!sol || !eta || !cell_diam || (variable != 0 && variable != 1) || n_pieces < 0 ||
      (n_pieces > 0 && (!ca || !cb || !xi || !g || !jxw)))
    return set_err(GLS_EINVAL, "gls_kelly_estimate_mapped: bad arguments");
  const int nq = c->nq1d + 1;  // QGauss<dim-1>(n_q + 1)
  if (nqf != (c->dim == 3 ? nq * nq : nq))
    return set_err(GLS_EINVAL, "gls_kelly_estimate_mapped: %d face points per piece, the face rule has %d", nqf,
                   c->dim == 3 ? nq * nq : nq);
  for (int64_t e = 0; e < n_pieces; ++e)
    if (ca[e] < 0 || ca[e] >= c->n_cells || cb[e] < 0 || cb[e] >= c->n_cells)
      return set_err(GLS_EINVAL, "gls_kelly_estimate_mapped: piece %lld out of range", (long long)e);
  const bool pres = variable == 1;
  const int m = pres ? c->kp : c->k;
  const int32_t *nodes = pres && c->cell_pnodes.p ? c->cell_pnodes.p : c->cell_vnodes.p;
  const gls::KellyTables T = kelly_tables(m, nq);
  const size_t npts = (size_t)n_pieces * (size_t)nqf;
  DevBuf<int32_t> dca, dcb;
  DevBuf<double> dxi, dg, dj, dfi;
  GLS_TRY(dca.upload(ca, (size_t)n_pieces));
  GLS_TRY(dcb.upload(cb, (size_t)n_pieces));
  GLS_TRY(dxi.upload(xi, npts * 2 * c->dim));
  GLS_TRY(dg.upload(g, npts * 2 * c->dim));
  GLS_TRY(dj.upload(jxw, npts));
  GLS_TRY(dfi.alloc((size_t)std::max<int64_t>(n_pieces, 1)));
  HIP_TRY(gls::launch_kelly_mapped(c->dim, m, nodes, sol, n_pieces, nqf, dca.p, dcb.p, dxi.p, dg.p, dj.p,
                                   pres ? 1 : c->dim, pres ? (int64_t)c->dim * c->n_vnodes : 0, pres ? 1 : c->dim, T,
                                   dfi.p, c->stream));
  std::vector<double> fi((size_t)n_pieces), acc((size_t)c->n_cells, 0.0);
  HIP_TRY(hipMemcpyAsync(fi.data(), dfi.p, sizeof(double) * fi.size(), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  for (int64_t e = 0; e < n_pieces; ++e) {  // each piece counts for both of its cells
    acc[(size_t)ca[e]] += fi[(size_t)e];
    acc[(size_t)cb[e]] += fi[(size_t)e];
  }
  for (int64_t k = 0; k < c->n_cells; ++k) acc[(size_t)k] = std::sqrt(cell_diam[k] / 24.0 * acc[(size_t)k]);
  HIP_TRY(hipMemcpyAsync(eta, acc.data(), sizeof(double) * acc.size(), hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return GLS_OK;
}

int gls_set_lattice(gls_ctx *c, int n1d, const int64_t *l2g) {
  GLS_TRY(check_ctx(c));
  if (c->dim != 3 || n1d < 2 || !l2g) return set_err(GLS_EINVAL, "gls_set_lattice: 3D, n1d >= 2, map required");
  int lo[3] = {n1d, n1d, n1d}, hi[3] = {-1, -1, -1};
  for (int i = 0; i < c->n_vnodes; ++i) {
    const int64_t g = l2g[i];
    if (g < 0 || g >= (int64_t)n1d * n1d * n1d) return set_err(GLS_EINVAL, "lattice node out of range");
    const int x[3] = {(int)(g % n1d), (int)((g / n1d) % n1d), (int)(g / ((int64_t)n1d * n1d))};
    for (int a = 0; a < 3; ++a) { lo[a] = std::min(lo[a], x[a]); hi[a] = std::max(hi[a], x[a]); }
  }
  int bd[3];
  for (int a = 0; a < 3; ++a) bd[a] = hi[a] - lo[a] + 1;
  const int64_t nbox = (int64_t)bd[0] * bd[1] * bd[2];
  if (nbox != c->n_vnodes) return set_err(GLS_EINVAL, "local nodes do not fill a box (%lld != %d)", (long long)nbox, c->n_vnodes);
  std::vector<int32_t> map((size_t)nbox, -1);
  for (int i = 0; i < c->n_vnodes; ++i) {
    const int64_t g = l2g[i];
    const int64_t x = g % n1d - lo[0], y = (g / n1d) % n1d - lo[1], z = g / ((int64_t)n1d * n1d) - lo[2];
    int32_t &m = map[(size_t)((z * bd[1] + y) * bd[0] + x)];
    if (m >= 0) return set_err(GLS_EINVAL, "duplicate lattice node");
    m = i;
  }
  GLS_TRY(c->lat.map.upload(map.data(), map.size()));
  c->lat.n1d = n1d;
  for (int a = 0; a < 3; ++a) { c->lat.box0[a] = lo[a]; c->lat.bdim[a] = bd[a]; }
  c->lat.set = true;
  return GLS_OK;
}

// the sweep parameters, level buffers and the coarsest-level direct solve of an attached hierarchy
static int mg_attach_common(gls_ctx *c, const gls_mg_params *p) {
  auto &mg = c->mg;
  mg.k = c->k;
  mg.pre = p->pre_smooth > 0 ? p->pre_smooth : (p->pre_smooth < 0 ? 0 : 2);
  mg.post = p->post_smooth >= 0 ? p->post_smooth : 2;
  mg.csweeps = p->coarse_sweeps > 0 ? p->coarse_sweeps : 30;
  mg.omega = p->omega > 0 ? p->omega : 0.6;
  mg.comega = p->coarse_omega > 0 ? p->coarse_omega : mg.omega;
  mg.lpre.assign((size_t)p->n_levels, mg.pre);
  mg.lpost.assign((size_t)p->n_levels, mg.post);
  if (p->level_sweeps)
    for (int l = 0; l < p->n_levels; ++l) {
      if (p->level_sweeps[2 * l] < 0 || p->level_sweeps[2 * l + 1] < 0) return set_err(GLS_EINVAL, "mg: negative level sweeps");
      mg.lpre[(size_t)l] = p->level_sweeps[2 * l];
      mg.lpost[(size_t)l] = p->level_sweeps[2 * l + 1];
    }
  for (auto *g : mg.lev) g->smooth_f32 = p->mixed_precision != 0;
  // the smoother's operator: Newton's Jacobian, or its Oseen (Picard) part (FP32 brick levels only: the
  // pencil J.v drops the (grad u) v terms)
  {
    const bool os = p->smoother_operator == 1;
    if (p->smoother_operator < 0 || p->smoother_operator > 1) return set_err(GLS_EINVAL, "mg: smoother_operator 0 or 1");
    for (auto *g : mg.lev) g->smooth_oseen = os && g->smooth_f32;
  }
  mg.ilu_smooth = p->smoother == 1 || p->smoother == 2;
  if (p->smoother < 0 || p->smoother > 2 || (mg.ilu_smooth && !mg.csr))
    return set_err(GLS_EINVAL, "mg: smoother 0 (Jacobi), 1 (ILU) or 2 (ILU below the finest level; gls_mg_attach_transfers hierarchies)");
  for (int l = 0; l < p->n_levels; ++l)
    for (int b = 0; b < MB_N; ++b) {
      mg.bufs.emplace_back(new DevBuf<double>());
      const bool need = b == MB_BOX ? (mg.boxed || mg.ilu_smooth) : (l > 0 || b == MB_Y);
      if (need)
        GLS_TRY(mg.bufs.back()->alloc(b == MB_BOX && mg.boxed ? (size_t)(4 * mg_nbox(c, l)) : (size_t)mg.lev[l]->n_dofs));
    }
  if (mg.ilu_smooth)  // ILU(0) on every level above the coarsest (multicolor order); smoother 2: not the finest
    for (int l = p->smoother == 2 ? 1 : 0; l + 1 < p->n_levels; ++l) {
      gls_ctx *g = mg.lev[(size_t)l];
      // multicolor order on every level. As a smoother the color-by-color ILU(0) is both faster per sweep (no level-scheduled csrsv) and
      // stronger: configs[3] --precond hmg 38 -> 26 GMRES iterations, 3.97 -> 1.37 s wall, the linear solves
      // 1.72 -> 0.08 s (profiles/r05_app_configs3_hmg_ilu_order.txt)
      GLS_TRY(gls_ilu_set_options(g, GLS_ILU_ORDER_MULTICOLOR, 0));
      GLS_TRY(gls_ilu_attach(g, 0, 1e-12, 1.0));
      mg.ilu_levels.push_back(g);  // detached again by gls_mg_detach
    }
  // direct coarsest solve: single GPU, coarsest level up to kDirectMax DoFs (FP64 LU up to kDirectSmall, FP32 above)
  {
    const int64_t nco = mg.lev.back()->n_dofs;
    const int want = p->coarse_direct;
    if (want > 0 && (mg.boxed || nco > kDirectMax))
      return set_err(GLS_EINVAL, "mg: direct coarse solve needs one GPU, <= %lld DoFs", (long long)kDirectMax);
    mg.direct = want > 0 || (want == 0 && !mg.boxed && nco <= 2048);
    if (mg.direct) {
      GLS_TRY(mg.probe.alloc((size_t)(nco * nco)));
      if (nco > kDirectSmall) {
        GLS_TRY(mg.probe32.alloc((size_t)(nco * nco)));
        GLS_TRY(mg.b32.alloc((size_t)nco));
        GLS_TRY(mg.x32.alloc((size_t)nco));
      }
      if (std::getenv("GLS_MG_COARSE_SOLVER")) GLS_TRY(mg.aug.alloc((size_t)(2 * nco * nco)));  // gj experiments
      GLS_TRY(mg.ipiv.alloc((size_t)nco));
      GLS_TRY(mg.info.alloc(1));
      if (!mg.blas.h && rocblas_create_handle(&mg.blas.h) != rocblas_status_success)
        return set_err(GLS_EHIP, "rocblas_create_handle failed");
      rocblas_set_pointer_mode(mg.blas, rocblas_pointer_mode_host);
      GLS_TRY(mg.unit.alloc((size_t)nco));
      GLS_TRY(mg.status.alloc(1));
      GLS_TRY(mg_probe_setup(c, mg.lev.back()));
    }
  }
  mg.on = true;
  mg.dirty = true;
  // one stream for the whole V-cycle: the coarse levels' kernels are ordered with the transfers
  for (size_t l = 1; l < mg.lev.size(); ++l)
    if (mg.lev[l]->stream != c->stream) GLS_TRY(gls_set_stream(mg.lev[l], c->stream));
  return GLS_OK;
}

int gls_mg_attach(gls_ctx *c, const gls_mg_params *p) {
  GLS_TRY(check_ctx(c));
  if (!p || p->n_levels < 2 || !p->levels || p->levels[0] != c) return set_err(GLS_EINVAL, "mg: levels[0] must be ctx");
  if (c->dim != 3 || c->k > 2 || c->k != c->kp) return set_err(GLS_EINVAL, "mg: 3D Q1-Q1 / Q2-Q2 only");
  if (c->hang.on) return set_err(GLS_EINVAL, "mg: not with hanging-node constraints");
  if (c->map_degree > 0) return set_err(GLS_EINVAL, "mg: nested hyper_cube levels only (not mapped cells)");
  GLS_TRY(gls_mg_detach(c));  // a previous attach's levels / smoother ILUs
  auto &mg = c->mg;
  mg.boxed = c->dist.on;
  for (int l = 0; l < p->n_levels; ++l) {
    gls_ctx *g = p->levels[l];
    if (!g || g->dim != 3 || g->k != c->k || g->kp != c->kp || g->dist.on != mg.boxed)
      return set_err(GLS_EINVAL, "mg level %d: order / distribution differs from level 0", l);
    std::array<int, 3> dm;
    if (mg.boxed) {
      if (!g->lat.set) return set_err(GLS_EINVAL, "mg level %d: distributed level without gls_set_lattice", l);
      for (int a = 0; a < 3; ++a) dm[a] = g->lat.bdim[a];
      if (l > 0) {
        const gls_ctx *f = p->levels[l - 1];
        if (f->lat.n1d != 2 * g->lat.n1d - 1) return set_err(GLS_EINVAL, "mg level %d not nested", l);
        for (int a = 0; a < 3; ++a)
          if (f->lat.box0[a] != 2 * g->lat.box0[a] || f->lat.bdim[a] != 2 * g->lat.bdim[a] - 1)
            return set_err(GLS_EINVAL, "mg level %d: partition not nested (rank box %d)", l, a);
      }
    } else {
      const int n = (int)std::lround(std::cbrt((double)g->n_vnodes));
      if ((int64_t)n * n * n != g->n_vnodes) return set_err(GLS_EINVAL, "mg level %d is not an n^3 lattice", l);
      if (l > 0 && mg.dims.back()[0] != 2 * n - 1) return set_err(GLS_EINVAL, "mg level %d not nested", l);
      dm = {n, n, n};
    }
    mg.lev.push_back(g);
    mg.dims.push_back(dm);
  }
  // 1D transfer taps: fine lattice index i sits at x = i / (2k) coarse cells from the box origin;
  // prolongation interpolates the coarse Qk field of the parent cell (equidistant nodes, k <= 2)
  const int K = c->k;
  size_t xwork = 0;
  for (int l = 0; l + 1 < p->n_levels; ++l) {
    std::unique_ptr<gls_ctx::MG::Taps> T(new gls_ctx::MG::Taps);
    T->two_pass = true;
    xwork = std::max(xwork, (size_t)4 * mg.dims[l + 1][0] * mg.dims[l + 1][1] * mg.dims[l][2]);
    for (int a = 0; a < 3; ++a) {
      const int nf = mg.dims[l][a], nc = mg.dims[l + 1][a], ncc = (nf - 1) / (2 * K);
      std::vector<int32_t> pi((size_t)nf * 5, 0), ri((size_t)nc * 5, 0);
      std::vector<double> pw((size_t)nf * 5, 0.0), rw((size_t)nc * 5, 0.0);
      std::vector<int32_t> rn((size_t)nc, 0), pn((size_t)nf, 0);
      for (int i = 0; i < nf; ++i) {
        const double x = (double)i / (2.0 * K);
        const int cc = std::min((int)std::floor(x), ncc - 1);
        const double xi = x - cc;
        int np = 0;
        for (int q = 0; q <= K; ++q) {
          double L = 1.0;
          for (int b = 0; b <= K; ++b)
            if (b != q) L *= (xi * K - b) / (double)(q - b);
          if (L == 0.0) continue;
          const int j = cc * K + q;
          pi[(size_t)i * 5 + np] = j;
          pw[(size_t)i * 5 + np] = L;
          ++np;
          if (rn[(size_t)j] >= 5) return set_err(GLS_EINVAL, "mg: restriction stencil wider than 5");
          ri[(size_t)j * 5 + rn[(size_t)j]] = i;
          rw[(size_t)j * 5 + rn[(size_t)j]] = L;
          ++rn[(size_t)j];
        }
        pn[(size_t)i] = np;
      }
      if (a < 2)
        T->two_pass = T->two_pass && gls::mg_transfer_tile_fits(0, a, nf, pi.data(), pn.data()) &&
                      gls::mg_transfer_tile_fits(1, a, nc, ri.data(), rn.data());
      GLS_TRY(T->pi[a].upload(pi.data(), pi.size()));
      GLS_TRY(T->pw[a].upload(pw.data(), pw.size()));
      GLS_TRY(T->ri[a].upload(ri.data(), ri.size()));
      GLS_TRY(T->rw[a].upload(rw.data(), rw.size()));
      GLS_TRY(T->pc[a].upload(pn.data(), pn.size()));
      GLS_TRY(T->rc[a].upload(rn.data(), rn.size()));
    }
    mg.taps.push_back(std::move(T));
  }
  if (xwork) GLS_TRY(mg.xwork.alloc(xwork));
  return mg_attach_common(c, p);
}

int gls_mg_attach_transfers(gls_ctx *c, const gls_mg_params *p, const int64_t *const *p_off, const int32_t *const *p_col,
                            const double *const *p_w, const int64_t *const *inject) {
  GLS_TRY(check_ctx(c));
  if (!p || p->n_levels < 2 || !p->levels || p->levels[0] != c) return set_err(GLS_EINVAL, "mg: levels[0] must be ctx");
  if (!p_off || !p_col || !p_w || !inject) return set_err(GLS_EINVAL, "mg: transfer arrays missing");

  GLS_TRY(gls_mg_detach(c));  // a previous attach's levels / smoother ILUs
  auto &mg = c->mg;
  mg.csr = true;
  for (int l = 0; l < p->n_levels; ++l) {
    gls_ctx *g = p->levels[l];
    // the levels may differ in degree (h-p hierarchies: the CSR transfers carry the p-level pairs of
    // gls_fe_space_mg_transfer), not in dimension
    if (!g || g->dim != c->dim || g->dist.on)
      return set_err(GLS_EINVAL, "mg level %d: dimension differs from level 0, or distributed", l);
    mg.lev.push_back(g);
    mg.dims.push_back({0, 0, 0});
  }
  for (int l = 0; l + 1 < p->n_levels; ++l) {
    const int64_t nf = mg.lev[(size_t)l]->n_dofs, nc = mg.lev[(size_t)l + 1]->n_dofs;
    const int64_t *off = p_off[l];
    if (!off || !p_col[l] || !p_w[l] || !inject[l] || off[0] != 0) return set_err(GLS_EINVAL, "mg transfer %d: arrays", l);
    for (int64_t i = 0; i < nf; ++i)
      if (off[i + 1] < off[i]) return set_err(GLS_EINVAL, "mg transfer %d: offsets not monotone", l);
    const int64_t nnz = off[nf];
    std::vector<int64_t> rcnt((size_t)nc + 1, 0);
    for (int64_t j = 0; j < nnz; ++j) {
      if (p_col[l][j] < 0 || p_col[l][j] >= nc) return set_err(GLS_EINVAL, "mg transfer %d: column out of range", l);
      ++rcnt[(size_t)p_col[l][j] + 1];
    }
    for (int64_t j = 0; j < nc; ++j) rcnt[(size_t)j + 1] += rcnt[(size_t)j];
    // R = P^T, each coarse row's terms in ascending fine row order (deterministic sums)
    std::vector<int32_t> rcol((size_t)nnz);
    std::vector<double> rw((size_t)nnz);
    std::vector<int64_t> fill(rcnt.begin(), rcnt.end() - 1);
    for (int64_t i = 0; i < nf; ++i)
      for (int64_t j = off[i]; j < off[i + 1]; ++j) {
        const int64_t slot = fill[(size_t)p_col[l][j]]++;
        rcol[(size_t)slot] = (int32_t)i;
        rw[(size_t)slot] = p_w[l][j];
      }
    std::vector<int32_t> inj((size_t)nc);
    for (int64_t j = 0; j < nc; ++j) {
      if (inject[l][j] < 0 || inject[l][j] >= nf) return set_err(GLS_EINVAL, "mg transfer %d: injection out of range", l);
      inj[(size_t)j] = (int32_t)inject[l][j];
    }
    std::unique_ptr<gls_ctx::MG::Csr> X(new gls_ctx::MG::Csr);
    X->nf = nf;
    X->nc = nc;
    auto lanes = [](double mean) {  // ~2 entries per lane
      int L = 1;
      while (L < 16 && 2.0 * L < mean) L *= 2;
      return L;
    };
    X->plane = lanes((double)nnz / (double)std::max<int64_t>(nf, 1));
    X->rlane = lanes((double)nnz / (double)std::max<int64_t>(nc, 1));
    GLS_TRY(X->poff.upload(off, (size_t)nf + 1));
    GLS_TRY(X->pcol.upload(p_col[l], (size_t)std::max<int64_t>(nnz, 1)));
    GLS_TRY(X->pw.upload(p_w[l], (size_t)std::max<int64_t>(nnz, 1)));
    GLS_TRY(X->roff.upload(rcnt.data(), rcnt.size()));
    GLS_TRY(X->rcol.upload(rcol.data(), std::max<size_t>(rcol.size(), 1)));
    GLS_TRY(X->rw.upload(rw.data(), std::max<size_t>(rw.size(), 1)));
    GLS_TRY(X->inj.upload(inj.data(), inj.size()));
    mg.xfer.push_back(std::move(X));
  }
  return mg_attach_common(c, p);
}

int gls_mg_set_coarse_replica(gls_ctx *c, gls_ctx *replica, int64_t n_local, const int64_t *local_to_replica) {
  GLS_TRY(check_ctx(c));
  auto &mg = c->mg;
  if (!mg.on || mg.lev.size() < 2) return set_err(GLS_EINVAL, "coarse replica: attach the multigrid hierarchy first");
  gls_ctx *g = mg.lev.back();
  if (!replica || replica == c || replica->dist.on) return set_err(GLS_EINVAL, "coarse replica: a single-rank context");
  if (!g->dist.on) return set_err(GLS_EINVAL, "coarse replica: the coarsest level is not distributed");
  if (n_local != g->n_dofs || !local_to_replica) return set_err(GLS_EINVAL, "coarse replica: map of %lld rows expected",
                                                                (long long)g->n_dofs);
  const int64_t ng = replica->n_dofs;
  if (ng >= INT32_MAX) return set_err(GLS_EINVAL, "coarse replica too large");
  std::vector<int32_t> all((size_t)n_local), own_l, own_g;
  const int64_t dv = (int64_t)g->dim * g->n_vnodes;
  for (int64_t i = 0; i < n_local; ++i) {
    const int64_t t = local_to_replica[i];
    if (t < 0 || t >= ng) return set_err(GLS_EINVAL, "coarse replica: row %lld maps outside", (long long)i);
    all[(size_t)i] = (int32_t)t;
    const bool owned = i < dv ? i < (int64_t)g->dim * g->dist.n_owned : i - dv < g->dist.n_owned_p;
    if (owned) {
      own_l.push_back((int32_t)i);
      own_g.push_back((int32_t)t);
    }
  }
  GLS_TRY(mg.rep_map.upload(all.data(), all.size()));
  GLS_TRY(mg.rep_own_loc.upload(own_l.data(), own_l.size()));
  GLS_TRY(mg.rep_own_glob.upload(own_g.data(), own_g.size()));
  GLS_TRY(mg.rep_b.alloc((size_t)ng));
  GLS_TRY(mg.rep_x.alloc((size_t)ng));
  GLS_TRY(mg.rep_tmp.alloc(std::max<size_t>(own_l.size(), 1)));
  for (auto &u : mg.rep_u) GLS_TRY(u.alloc((size_t)ng));
  if (replica->stream != c->stream) GLS_TRY(gls_set_stream(replica, c->stream));
  mg.replica = replica;
  mg.dirty = true;
  return GLS_OK;
}

int gls_mg_attach_replica(gls_ctx *c, const gls_mg_params *p, gls_ctx *replica, const int64_t *p_off,
                          const int32_t *p_col, const double *p_w, const int64_t *inject) {
  GLS_TRY(check_ctx(c));
  if (!p || !replica || replica == c || replica->dist.on || !p_off || !p_col || !p_w || !inject)
    return set_err(GLS_EINVAL, "mg replica attach: arguments");
  if (!c->dist.on) return set_err(GLS_EINVAL, "mg replica attach: the fine context is not distributed");
  if (replica->dim != c->dim || replica->k != c->k || replica->kp != c->kp)
    return set_err(GLS_EINVAL, "mg replica attach: replica order / dimension differs");
  if (p->smoother < 0 || p->smoother > 1) return set_err(GLS_EINVAL, "mg replica attach: smoother 0 or 1");
  GLS_TRY(gls_mg_detach(c));
  auto &mg = c->mg;
  const int64_t n = c->n_dofs, ng = replica->n_dofs;
  if (ng >= INT32_MAX) return set_err(GLS_EINVAL, "mg replica attach: replica too large");
  const int64_t dv = (int64_t)c->dim * c->n_vnodes;
  auto owned = [&](int64_t i) { return i < dv ? i < (int64_t)c->dim * c->dist.n_owned : i - dv < c->dist.n_owned_p; };
  // P on the local rows; R = the owned rows' P^T (rows = replica DoFs, local fine columns in ascending order)
  const int64_t nnz = p_off[n];
  std::vector<int64_t> roff((size_t)ng + 1, 0);
  for (int64_t i = 0; i < n; ++i) {
    if (p_off[i + 1] < p_off[i]) return set_err(GLS_EINVAL, "mg replica attach: P offsets");
    for (int64_t e = p_off[i]; e < p_off[i + 1]; ++e) {
      if (p_col[e] < 0 || p_col[e] >= ng) return set_err(GLS_EINVAL, "mg replica attach: P column %d", p_col[e]);
      if (owned(i)) ++roff[(size_t)p_col[e] + 1];
    }
  }
  for (int64_t r = 0; r < ng; ++r) roff[(size_t)r + 1] += roff[(size_t)r];
  std::vector<int32_t> rcol((size_t)roff[(size_t)ng]);
  std::vector<double> rw(rcol.size());
  std::vector<int64_t> fill(roff.begin(), roff.end() - 1);
  for (int64_t i = 0; i < n; ++i)
    if (owned(i))
      for (int64_t e = p_off[i]; e < p_off[i + 1]; ++e) {
        const int64_t at = fill[(size_t)p_col[e]]++;
        rcol[(size_t)at] = (int32_t)i;
        rw[(size_t)at] = p_w[e];
      }
  std::vector<int32_t> ic, iff;
  for (int64_t r = 0; r < ng; ++r)
    if (inject[r] >= 0) {
      if (inject[r] >= n || !owned(inject[r])) return set_err(GLS_EINVAL, "mg replica attach: inject[%lld] not owned", (long long)r);
      ic.push_back((int32_t)r);
      iff.push_back((int32_t)inject[r]);
    }
  GLS_TRY(mg.r2p_off.upload(p_off, (size_t)n + 1));
  GLS_TRY(mg.r2p_col.upload(p_col, std::max<size_t>((size_t)nnz, 1)));
  GLS_TRY(mg.r2p_w.upload(p_w, std::max<size_t>((size_t)nnz, 1)));
  GLS_TRY(mg.r2r_off.upload(roff.data(), roff.size()));
  if (rcol.empty()) {
    rcol.push_back(0);
    rw.push_back(0.0);
  }
  GLS_TRY(mg.r2r_col.upload(rcol.data(), rcol.size()));
  GLS_TRY(mg.r2r_w.upload(rw.data(), rw.size()));
  auto lanes = [](double mean) { return mean > 24 ? 16 : mean > 6 ? 4 : 1; };
  mg.r2p_lane = lanes(n ? (double)nnz / (double)n : 0.0);
  mg.r2r_lane = lanes(ng ? (double)(roff[(size_t)ng]) / (double)ng : 0.0);
  if (ic.empty()) {
    ic.push_back(0);
    iff.push_back(0);
  }
  GLS_TRY(mg.r2inj_c.upload(ic.data(), ic.size()));
  GLS_TRY(mg.r2inj_f.upload(iff.data(), iff.size()));
  if (ic.size() == 1 && inject[ic[0]] < 0) mg.r2inj_c.n = mg.r2inj_f.n = 0;  // no owned source on this rank
  GLS_TRY(mg.rep_b.alloc((size_t)ng));
  GLS_TRY(mg.rep_x.alloc((size_t)ng));
  GLS_TRY(mg.rep_tmp.alloc(std::max<size_t>(ic.size(), 1)));
  for (auto &u : mg.rep_u) GLS_TRY(u.alloc((size_t)ng));
  // smoothing on the distributed fine level: damped Jacobi or ILU(0) (per-rank blocks, Ifpack overlap 0)
  mg.lev.assign(1, c);
  mg.pre = p->pre_smooth > 0 ? p->pre_smooth : (p->pre_smooth < 0 ? 0 : 2);
  mg.post = p->post_smooth >= 0 ? p->post_smooth : 2;
  mg.lpre.assign(1, mg.pre);
  mg.lpost.assign(1, mg.post);
  mg.omega = p->omega > 0 ? p->omega : 0.6;
  mg.comega = mg.omega;
  mg.ilu_smooth = p->smoother == 1;
  for (int b = 0; b < MB_N; ++b) {
    mg.bufs.emplace_back(new DevBuf<double>());
    if (b == MB_Y || (b == MB_BOX && mg.ilu_smooth)) GLS_TRY(mg.bufs.back()->alloc((size_t)n));
  }
  if (mg.ilu_smooth) {
    GLS_TRY(gls_ilu_set_options(c, GLS_ILU_ORDER_MULTICOLOR, 0));
    GLS_TRY(gls_ilu_attach(c, 0, 1e-12, 1.0));
    mg.ilu_levels.push_back(c);
  }
  // a replica without a hierarchy of its own is the coarsest level: exact LU when asked (coarse_direct > 0)
  if (p->coarse_direct > 0 && !replica->mg.on) {
    if (ng > 8192) return set_err(GLS_EINVAL, "mg replica attach: direct coarse solve needs <= 8192 DoFs");
    mg.direct = true;
    GLS_TRY(mg.probe.alloc((size_t)(ng * ng)));
    GLS_TRY(mg.ipiv.alloc((size_t)ng));
    GLS_TRY(mg.info.alloc(1));
    if (!mg.blas.h && rocblas_create_handle(&mg.blas.h) != rocblas_status_success)
      return set_err(GLS_EHIP, "rocblas_create_handle failed");
    rocblas_set_pointer_mode(mg.blas, rocblas_pointer_mode_host);
    GLS_TRY(mg.unit.alloc((size_t)ng));
    GLS_TRY(mg.status.alloc(1));
    GLS_TRY(mg_probe_setup(c, replica));
  }
  if (replica->stream != c->stream) GLS_TRY(gls_set_stream(replica, c->stream));
  mg.rep2 = replica;
  mg.rep_csr = true;
  mg.on = true;
  mg.dirty = true;
  return GLS_OK;
}

int gls_mg_detach(gls_ctx *c) {
  GLS_TRY(check_ctx(c));
  for (auto *g : c->mg.lev) g->smooth_f32 = g->smooth_oseen = false;
  // the ILU(0) smoothers the attach put on the levels (level 0 is this context) go with the multigrid, so
  // the preconditioner falls back to Jacobi (gls_native.h) and not to a leftover smoother ILU
  for (auto *g : c->mg.ilu_levels) GLS_TRY(gls_ilu_detach(g));
  c->mg.side.reset();  // (a coarse factorization in flight reads the buffers the assignment frees)
  c->mg = gls_ctx::MG();
  return GLS_OK;
}

// --------------------------------------------------------------------------------------------
// GMRES(m), right preconditioned (Jacobi, the V-cycle or the assembled ILU). Orthogonalisation:
// Gram-corrected classical Gram–Schmidt (one projection pass per iteration, see the loop) or, with
// gls_linear_params.orthogonalization = GLS_ORTHO_CGS2, classical Gram–Schmidt with one DGKS re-orthogonalisation
// pass; fused multi-dot /
// multi-axpy kernels (one pass over the Krylov basis per Gram–Schmidt sweep). Stopping test on the unpreconditioned residual
// ||b - A x|| <= max(rel*||b||, abs) (deal.II SolverControl / AztecOO AZ_noscaled).
// --------------------------------------------------------------------------------------------
// BiCGStab (solve_system_BiCGStab, gls_navier_stokes.cc:1293-1340: TrilinosWrappers::SolverBicgstab =
// AztecOO AZ_bicgstab with the same ILU, here with whatever preconditioner gls_solve_linear applies),
// right preconditioned (van der Vorst's BiCGStab on A M^-1, x = M^-1 y), so the recursively updated
// residual is the unpreconditioned b - A x the reference's tolerance rule tests:
// ||r|| <= max(rel ||b||, abs). One iteration = one BiCGStab step (two operator applications), as
// AztecOO counts. Breakdown (rho or (rhat, v) or (t, t) vanishing) stops with the current iterate.
static int solve_bicgstab(gls_ctx *c, const double *b, double *x, gls_linear_params *prm) {
  const int64_t n = c->n_dofs;
  hipStream_t s = c->stream;
  // work vectors: r, rhat, p, v, phat, shat, t (the GMRES basis storage when it is large enough)
  double *w[7];
  if (c->krylov.p && c->krylov.n >= (size_t)7 * n) {
    for (int i = 0; i < 7; ++i) w[i] = c->krylov.p + (int64_t)i * n;
  } else {
    if (c->bicg.n != (size_t)7 * n) GLS_TRY(c->bicg.alloc((size_t)7 * n));
    for (int i = 0; i < 7; ++i) w[i] = c->bicg.p + (int64_t)i * n;
  }
  double *r = w[0], *rh = w[1], *p = w[2], *v = w[3], *ph = w[4], *sh = w[5], *t = w[6];
  double bn2;
  GLS_TRY(device_dot(c, b, b, &bn2));
  const double tol = std::max(prm->relative_residual * std::sqrt(bn2), prm->minimum_residual);
  HIP_TRY(gls::vec_fill(x, n, 0.0, s));
  HIP_TRY(gls::vec_copy(r, b, n, s));
  HIP_TRY(gls::vec_copy(rh, b, n, s));
  HIP_TRY(gls::vec_fill(p, n, 0.0, s));
  HIP_TRY(gls::vec_fill(v, n, 0.0, s));
  double res = std::sqrt(bn2), rho = 1.0, alpha = 1.0, omega = 1.0;
  int it = 0;
  bool converged = res <= tol;
  while (!converged && it < prm->max_iterations) {
    double rho1;
    GLS_TRY(device_dot(c, rh, r, &rho1));
    if (rho1 == 0.0 || omega == 0.0) break;  // breakdown
    const double beta = (rho1 / rho) * (alpha / omega);
    rho = rho1;
    // p = r + beta (p - omega v)
    HIP_TRY(gls::vec_axpy(p, -omega, v, n, s));
    HIP_TRY(gls::vec_axpby(p, 1.0, r, beta, n, s));
    GLS_TRY(apply_prec(c, p, ph));
    GLS_TRY(gls_jacobian_apply(c, ph, v));
    double rhv;
    GLS_TRY(device_dot(c, rh, v, &rhv));
    if (rhv == 0.0) break;
    alpha = rho / rhv;
    HIP_TRY(gls::vec_axpy(r, -alpha, v, n, s));  // r <- s = r - alpha v
    HIP_TRY(gls::vec_axpy(x, alpha, ph, n, s));  // x += alpha M^-1 p
    ++it;
    double sn2;
    GLS_TRY(device_dot(c, r, r, &sn2));
    res = std::sqrt(sn2);
    if (res <= tol) {
      converged = true;
      break;
    }
    GLS_TRY(apply_prec(c, r, sh));
    GLS_TRY(gls_jacobian_apply(c, sh, t));
    double tt, ts;
    GLS_TRY(device_dot(c, t, t, &tt));
    GLS_TRY(device_dot(c, t, r, &ts));
    if (tt == 0.0) break;
    omega = ts / tt;
    HIP_TRY(gls::vec_axpy(x, omega, sh, n, s));  // x += omega M^-1 s
    HIP_TRY(gls::vec_axpy(r, -omega, t, n, s));  // r = s - omega t
    double rn2;
    GLS_TRY(device_dot(c, r, r, &rn2));
    res = std::sqrt(rn2);
    converged = res <= tol;
    if (getenv("GLS_GMRES_VERBOSE") && (it % 10 == 0 || it == 1))
      printf("  bicgstab it %d  res %.6e  (tol %.3e)\n", it, res, tol);
  }
  if (converged && prm->true_residual) {
    GLS_TRY(gls_jacobian_apply(c, x, t));
    HIP_TRY(gls::vec_axpby(t, 1.0, b, -1.0, n, s));
    double rn2;
    GLS_TRY(device_dot(c, t, t, &rn2));
    res = std::sqrt(rn2);
  }
  prm->iterations = it;
  prm->final_residual = res;
  if (!converged) return set_err(GLS_ENOCONV, "BiCGStab: %d iterations, residual %.3e > %.3e", it, res, tol);
  return GLS_OK;
}

int gls_solve_linear(gls_ctx *c, const double *b, double *x, gls_linear_params *prm) {
  GLS_TRY(check_ctx(c));
  if (!b || !x || !prm) return set_err(GLS_EINVAL, "null argument");
  const int m = prm->restart > 0 ? std::min(prm->restart, 200) : 30;
  const int64_t n = c->n_dofs;
  if (c->krylov_m != m || !c->krylov.p) {
    GLS_TRY(c->krylov.alloc((size_t)(m + 1) * n));
    GLS_TRY(c->coef.alloc((size_t)m + 8));
    if (c->scal.n < (size_t)m + 8) GLS_TRY(c->scal.alloc((size_t)m + 8));
    if (c->scal2.n < (size_t)m + 8) GLS_TRY(c->scal2.alloc((size_t)m + 8));
    if (c->hpin_n < 3 * ((size_t)m + 8)) {
      if (c->hpin) HIP_TRY(hipHostFree(c->hpin));
      c->hpin = nullptr;
      c->hpin_n = 0;
      HIP_TRY(hipHostMalloc(reinterpret_cast<void **>(&c->hpin), sizeof(double) * 3 * ((size_t)m + 8)));
      c->hpin_n = 3 * ((size_t)m + 8);
    }
    c->krylov_m = m;
  }
  if (!c->tmp1.p) {
    GLS_TRY(c->tmp1.alloc(n));
    GLS_TRY(c->tmp2.alloc(n));
  }
  GLS_TRY(ensure_diag(c));
  if (c->mg.on) GLS_TRY(mg_prepare(c));
  GLS_TRY(ensure_ilu(c));
  if (prm->method == GLS_LIN_BICGSTAB) return solve_bicgstab(c, b, x, prm);
  if (prm->method != GLS_LIN_GMRES) return set_err(GLS_EINVAL, "linear solver method %d unknown", prm->method);
  // with the V-cycle, keep Z = M^-1 V (flexible-GMRES storage): the update x += Z y then needs no
  // extra preconditioner application per restart cycle
  const bool keepz = c->mg.on;
  if (keepz && c->zbasis.n != (size_t)m * n) GLS_TRY(c->zbasis.alloc((size_t)m * n));
  double *V = c->krylov.p, *z = c->tmp1.p, *r = c->tmp2.p;
  hipStream_t s = c->stream;
  double bnorm2;
  GLS_TRY(device_dot(c, b, b, &bnorm2));
  const double tol = std::max(prm->relative_residual * std::sqrt(bnorm2), prm->minimum_residual);
  // x = 0: with the Z basis the first update writes x = Z y without reading it (x_zero), and the first
  // restart cycle starts from r = b itself (no copy)
  bool x_zero = keepz;
  if (!keepz) HIP_TRY(gls::vec_fill(x, n, 0.0, s));
  const double *rcur = b;
  double beta = std::sqrt(bnorm2);
  int it = 0;
  std::vector<double> H((size_t)(m + 1) * m), cs(m), sn(m), g(m + 1), hc2(m + 2), y(m);
  // Gram-corrected single-pass orthogonalisation (default; prm->orthogonalization = GLS_ORTHO_CGS2: classical
  // Gram-Schmidt with the DGKS second pass); Gm: measured off-diagonal part of V^T V of the current restart cycle
  const bool gram = prm->orthogonalization != GLS_ORTHO_CGS2;
  int ortho_repairs = 0;
  // test knobs (read per call): GLS_GMRES_REPAIR_TOL (default 1e-8; 0 repairs every column) and
  // GLS_GMRES_REPAIR_MEASURED=1 (the repair pass always normalises by the measured norm)
  const double repair_tol = std::getenv("GLS_GMRES_REPAIR_TOL") ? std::atof(std::getenv("GLS_GMRES_REPAIR_TOL")) : 1e-8;
  const bool repair_measured = std::getenv("GLS_GMRES_REPAIR_MEASURED") != nullptr;
  std::vector<double> Gm((size_t)(m + 1) * (m + 1), 0.0);
  bool converged = beta <= tol;
  const bool lverbose = std::getenv("GLS_ILU_VERBOSE") != nullptr;
  while (!converged && it < prm->max_iterations) {
    if (lverbose) std::printf("gmres: it %d residual %.6e (tol %.3e)\n", it, beta, tol);
    HIP_TRY(gls::vec_axpby(V, 1.0 / beta, rcur, 0.0, n, s));
    std::fill(Gm.begin(), Gm.end(), 0.);
    std::fill(g.begin(), g.end(), 0.);
    g[0] = beta;
    int j = 0;
    double res = beta;
    for (; j < m && it < prm->max_iterations; ++j) {
      double *vj = V + (int64_t)j * n, *w = V + (int64_t)(j + 1) * n;
      double *zj = keepz ? c->zbasis.p + (int64_t)j * n : z;
      GLS_TRY(apply_prec(c, vj, zj));
      GLS_TRY(gls_jacobian_apply(c, zj, w));
      // h = V[0..j]^T w and ||w||^2 in one pass. The Gram-Schmidt passes are chained on the stream:
      // each projection reads the previous pass's dots from device memory (scal / scal2 alternate),
      // the host copies arrive in pinned memory, and the host waits once per pass pair (after the
      // projection, and after the DGKS correction when it is taken) instead of once per pass.
      double *hp1 = c->hpin, *hp2 = c->hpin + (m + 8), *hp3 = c->hpin + 2 * (m + 8);
      const double *hdev = nullptr, *h2dev = nullptr, *h3dev = nullptr;
      GLS_TRY(multidot_async(c, V, n, j + 2, w, c->scal.p, hp1, &hdev));
      double wn2, wnorm, wnorm0;
      bool normalized = false;  // w already scaled to v_{j+1} (H(j+1, j) set) by the fused DGKS pass
      bool done = false;        // the Gram-corrected single projection below handled this column
      if (gram) {
        // Gram-corrected classical Gram-Schmidt: ONE projection pass with h = (2I - G) h1, where
        // h1 = V^T w and G = V^T V (unit diagonal, off-diagonal part Gm measured by the previous
        // projections' fused dots) -- the first-order inverse of G, so w - V h is orthogonal to the
        // basis up to O(|G - I|^2) and rounding, as after CGS2's second pass, without that pass over
        // V. The projection also normalises (est^2 = |w|^2 - 2 h.h1 + h^T G h) and returns V^T v_{j+1}
        // (the next column of Gm) and |v_{j+1}|^2; a DGKS pass repairs the rare column whose measured
        // orthogonality or norm is off by more than 1e-8 (catastrophic cancellation).
        HIP_TRY(hipStreamSynchronize(s));
        const double wn0sq = std::max(hp1[j + 1], 0.0);
        wnorm0 = std::sqrt(wn0sq);
        auto G = [&](int a, int b) { return Gm[(size_t)std::min(a, b) * (m + 1) + std::max(a, b)]; };
        double *hc = hp3;
        for (int i = 0; i <= j; ++i) {
          double t = hp1[i];
          for (int k = 0; k <= j; ++k)
            if (k != i) t -= G(i, k) * hp1[k];
          hc[i] = t;
        }
        double q = wn0sq;
        for (int i = 0; i <= j; ++i) q += hc[i] * hc[i] - 2.0 * hc[i] * hp1[i];
        for (int i = 0; i <= j; ++i)
          for (int k = i + 1; k <= j; ++k) q += 2.0 * hc[i] * hc[k] * G(i, k);
        if (q > 1e-20 * wn0sq && q > 0.) {
          const double est = std::sqrt(q);
          HIP_TRY(hipMemcpyAsync(c->coef.p, hc, sizeof(double) * (j + 1), hipMemcpyHostToDevice, s));
          if (j + 1 <= 8) {
            GLS_TRY(multiaxpy_dots_async(c, w, V, n, j + 1, c->coef.p, true, c->scal2.p, hp2, &h2dev, 1.0 / est));
          } else {
            HIP_TRY(gls::vec_multiaxpy(w, V, n, j + 1, c->coef.p, 1.0, n, s));
            HIP_TRY(gls::vec_scale(w, 1.0 / est, n, s));
            GLS_TRY(multidot_async(c, V, n, j + 2, w, c->scal2.p, hp2, &h2dev));
          }
          HIP_TRY(hipStreamSynchronize(s));
          for (int i = 0; i <= j; ++i) H[(size_t)i * m + j] = hc[i];
          H[(size_t)(j + 1) * m + j] = est;
          double gmax = 0., gg = 0.;
          for (int i = 0; i <= j; ++i) {
            gmax = std::max(gmax, std::fabs(hp2[i]));
            gg += hp2[i] * hp2[i];
          }
          const double nrm2 = hp2[j + 1];
          const double est2sq = nrm2 - gg;  // |v - V g|^2 if V were exactly orthonormal
          if (gmax > repair_tol || std::fabs(nrm2 - 1.0) > repair_tol) {
            // repair pass v' = (v - V g) / s: H column += est g, H(j+1, j) = est s. The first-order
            // estimate s = sqrt(|v|^2 - |g|^2) is used only when the cancellation leaves it well
            // above rounding (est2sq > 1e-4); otherwise the pass runs unscaled and s is the MEASURED
            // norm of its result. Either way the measured |v'|^2 returned by the pass decides: a
            // vector off unit length by more than 1e-8 is rescaled (with its H entry and Gram
            // column), and a vanishing one is a breakdown (the Krylov space is exhausted).
            const bool use_est = est2sq > 1e-4 && !repair_measured;
            const double est2 = use_est ? std::sqrt(est2sq) : 1.0;
            for (int i = 0; i <= j; ++i) H[(size_t)i * m + j] += est * hp2[i];
            if (j + 1 <= 8) {
              GLS_TRY(multiaxpy_dots_async(c, w, V, n, j + 1, h2dev, true, c->scal.p, hp1, &hdev, 1.0 / est2));
            } else {
              HIP_TRY(gls::vec_multiaxpy(w, V, n, j + 1, h2dev, 1.0, n, s));
              if (use_est) HIP_TRY(gls::vec_scale(w, 1.0 / est2, n, s));
              GLS_TRY(multidot_async(c, V, n, j + 2, w, c->scal.p, hp1, &hdev));
            }
            HIP_TRY(hipStreamSynchronize(s));
            const double nn = std::max(hp1[j + 1], 0.0);  // measured |v'|^2
            double sc = 1.0;                               // v_{j+1} = v' / sc
            if (nn <= 1e-28 * (use_est ? 1.0 : std::max(nrm2, 1e-300))) {
              sc = 0.0;  // breakdown: w lies in span(V) to rounding
            } else if (!use_est || std::fabs(nn - 1.0) > 1e-8) {
              sc = std::sqrt(nn);
              HIP_TRY(gls::vec_scale(w, 1.0 / sc, n, s));
            }
            H[(size_t)(j + 1) * m + j] = est * est2 * sc;
            for (int i = 0; i <= j; ++i) Gm[(size_t)i * (m + 1) + j + 1] = sc > 0. ? hp1[i] / sc : 0.;
            ++ortho_repairs;
          } else {
            for (int i = 0; i <= j; ++i) Gm[(size_t)i * (m + 1) + j + 1] = hp2[i];
          }
          wnorm = H[(size_t)(j + 1) * m + j];
          normalized = done = true;
        }
      }
      if (done) {
      } else if (j + 1 <= 8) {
        // projection fused with the DGKS dots and the norm: one pass over V instead of three
        GLS_TRY(multiaxpy_dots_async(c, w, V, n, j + 1, hdev, true, c->scal2.p, hp2, &h2dev));
        HIP_TRY(hipStreamSynchronize(s));
        wnorm0 = std::sqrt(std::max(hp1[j + 1], 0.0));
        for (int i = 0; i <= j; ++i) H[(size_t)i * m + j] = hp1[i];
        std::copy(hp2, hp2 + j + 2, hc2.begin());
        wnorm = std::sqrt(std::max(hc2[j + 1], 0.0));
        if (wnorm < 0.7071 * wnorm0) {  // DGKS re-orthogonalisation with the dots of the fused pass
          for (int i = 0; i <= j; ++i) H[(size_t)i * m + j] += hc2[i];
          // ||w''||^2 = ||w'||^2 - |V^T w'|^2 (V orthonormal): the correction pass also normalises,
          // v_{j+1} = w'' / est, and H(j+1, j) = est keeps A z_j = V H exactly (|v_{j+1}| = 1 + O(eps))
          double h2 = 0.;
          for (int i = 0; i <= j; ++i) h2 += hc2[i] * hc2[i];
          const double est2 = wnorm * wnorm - h2;
          if (est2 > 0.25 * wnorm * wnorm && est2 > 0.) {
            const double est = std::sqrt(est2);
            GLS_TRY(multiaxpy_dots_async(c, w, V, n, j + 1, h2dev, false, c->scal.p, hp3, &h3dev, 1.0 / est));
            HIP_TRY(hipStreamSynchronize(s));
            wn2 = hp3[0];
            H[(size_t)(j + 1) * m + j] = est;
            normalized = true;
            wnorm = est * std::sqrt(std::max(wn2, 0.0));
          } else {
            GLS_TRY(multiaxpy_dots_async(c, w, V, n, j + 1, h2dev, false, c->scal.p, hp3, &h3dev));
            HIP_TRY(hipStreamSynchronize(s));
            wn2 = hp3[0];
            wnorm = std::sqrt(std::max(wn2, 0.0));
          }
        }
      } else {
        HIP_TRY(gls::vec_multiaxpy(w, V, n, j + 1, hdev, 1.0, n, s));
        GLS_TRY(multidot_async(c, w, 0, 1, w, c->scal2.p, hp2, &h2dev));
        HIP_TRY(hipStreamSynchronize(s));
        wnorm0 = std::sqrt(std::max(hp1[j + 1], 0.0));
        for (int i = 0; i <= j; ++i) H[(size_t)i * m + j] = hp1[i];
        wn2 = hp2[0];
        wnorm = std::sqrt(std::max(wn2, 0.0));
        if (wnorm < 0.7071 * wnorm0) {  // DGKS re-orthogonalisation
          GLS_TRY(multidot_async(c, V, n, j + 1, w, c->scal.p, hp1, &hdev));
          HIP_TRY(gls::vec_multiaxpy(w, V, n, j + 1, hdev, 1.0, n, s));
          GLS_TRY(multidot_async(c, w, 0, 1, w, c->scal2.p, hp2, &h2dev));
          HIP_TRY(hipStreamSynchronize(s));
          for (int i = 0; i <= j; ++i) H[(size_t)i * m + j] += hp1[i];
          wn2 = hp2[0];
          wnorm = std::sqrt(std::max(wn2, 0.0));
        }
      }
      if (!normalized) {
        H[(size_t)(j + 1) * m + j] = wnorm;
        if (wnorm > 0) HIP_TRY(gls::vec_scale(w, 1.0 / wnorm, n, s));
      }
      // Givens
      for (int i = 0; i < j; ++i) {
        const double a = H[(size_t)i * m + j], bb = H[(size_t)(i + 1) * m + j];
        H[(size_t)i * m + j] = cs[i] * a + sn[i] * bb;
        H[(size_t)(i + 1) * m + j] = -sn[i] * a + cs[i] * bb;
      }
      const double a = H[(size_t)j * m + j], bb = H[(size_t)(j + 1) * m + j];
      const double rr = std::hypot(a, bb);
      cs[j] = rr > 0 ? a / rr : 1.0;
      sn[j] = rr > 0 ? bb / rr : 0.0;
      H[(size_t)j * m + j] = rr;
      H[(size_t)(j + 1) * m + j] = 0.;
      g[j + 1] = -sn[j] * g[j];
      g[j] = cs[j] * g[j];
      res = std::fabs(g[j + 1]);
      ++it;
      if (getenv("GLS_GMRES_VERBOSE") && (it % 10 == 0 || it == 1))
        printf("  gmres it %d  res %.6e  (tol %.3e)\n", it, res, tol);
      if (res <= tol || wnorm == 0.) { ++j; break; }
    }
    // back substitution and update x += M^{-1} V y
    const int kdim = j;
    for (int i = kdim - 1; i >= 0; --i) {
      double s_ = g[i];
      for (int l = i + 1; l < kdim; ++l) s_ -= H[(size_t)i * m + l] * y[l];
      y[i] = H[(size_t)i * m + i] != 0. ? s_ / H[(size_t)i * m + i] : 0.;
    }
    HIP_TRY(hipMemcpyAsync(c->coef.p, y.data(), sizeof(double) * kdim, hipMemcpyHostToDevice, s));
    if (keepz) {
      HIP_TRY(gls::vec_multiaxpy(x, c->zbasis.p, n, kdim, c->coef.p, -1.0, n, s, x_zero));  // x += Z y
      x_zero = false;
    } else {
      HIP_TRY(gls::vec_fill(r, n, 0.0, s));
      HIP_TRY(gls::vec_multiaxpy(r, V, n, kdim, c->coef.p, -1.0, n, s));  // r = V y
      GLS_TRY(apply_prec(c, r, z));
      HIP_TRY(gls::vec_axpy(x, 1.0, z, n, s));
    }
    // converged on the recurrence estimate: done (as deal.II's SolverGMRES, which recomputes the
    // true residual only at a restart)
    if (res <= tol) {
      beta = res;
      converged = true;
      if (prm->true_residual) {  // the caller asked for ||b - A x|| instead of the recurrence estimate
        GLS_TRY(gls_jacobian_apply(c, x, r));
        HIP_TRY(gls::vec_axpby(r, 1.0, b, -1.0, n, s));
        double rn2;
        GLS_TRY(device_dot(c, r, r, &rn2));
        beta = std::sqrt(rn2);
      }
      break;
    }
    // true residual r = b - A x
    GLS_TRY(gls_jacobian_apply(c, x, r));
    HIP_TRY(gls::vec_axpby(r, 1.0, b, -1.0, n, s));
    rcur = r;
    double rn2;
    GLS_TRY(device_dot(c, r, r, &rn2));
    beta = std::sqrt(rn2);
    converged = beta <= tol;
    if (beta == 0.) break;
  }
  if (x_zero) HIP_TRY(gls::vec_fill(x, n, 0.0, s));  // no update was made (b below the tolerance)
  prm->iterations = it;
  prm->final_residual = beta;
  if (ortho_repairs && std::getenv("GLS_GMRES_VERBOSE")) printf("  gmres: %d orthogonality repair passes\n", ortho_repairs);
  if (!converged) return set_err(GLS_ENOCONV, "GMRES: %d iterations, residual %.3e > %.3e", it, beta, tol);
  return GLS_OK;
}

// --------------------------------------------------------------------------------------------
// NewtonNonLinearSolver::solve (include/core/newton_non_linear_solver.h:74-139), one template
// driving any "physics" with the PhysicsSolver hooks (include/core/physics_solver.h:64-102).
// --------------------------------------------------------------------------------------------
}  // extern "C"

namespace {

struct NewtonStats {
  int outer = 0, linear = 0, residuals = 0;
  double final_res = 0.;
};

// SkipNewtonNonLinearSolver::solve (include/core/skip_newton_non_linear_solver.h:54-131): the
// Jacobian (and its preconditioner) is assembled only when consecutive_iters == 0, on the initial
// step or when forced, and only in the first outer iteration; every later iteration reuses it.
template <class Phys>
int skip_newton_template(Phys &ph, double tolerance, int max_iterations, int verbosity, int skip_iterations,
                         bool is_initial_step, bool force_matrix_renewal, int &consecutive, NewtonStats &st) {
  double current_res = 1.0, last_res = 1.0;
  int outer = 0;
  bool assembly_needed = consecutive == 0 || is_initial_step || force_matrix_renewal;
  while (current_res > tolerance && outer < max_iterations) {
    GLS_TRY(ph.evaluation_point_from_present());
    if (assembly_needed) {
      GLS_TRY(ph.assemble_matrix_and_rhs());
      ++st.residuals;
    } else if (outer == 0) {
      GLS_TRY(ph.assemble_rhs());
      ++st.residuals;
    }
    if (outer == 0) {
      GLS_TRY(ph.rhs_norm(current_res));
      last_res = current_res;
    }
    if (verbosity) printf("Newton iteration: %d  - Residual:  %g\n", outer, current_res);
    int lin_it = 0;
    GLS_TRY(ph.solve_linear_system(lin_it));  // renewed_matrix = assembly_needed: reused otherwise
    st.linear += lin_it;
    for (double alpha = 1.0; alpha > 1e-3; alpha *= 0.5) {
      GLS_TRY(ph.line_point(alpha));
      GLS_TRY(ph.assemble_rhs());
      ++st.residuals;
      GLS_TRY(ph.rhs_norm(current_res));
      if (verbosity) printf("\t\talpha = %6g res = %g\n", alpha, current_res);
      if (current_res < 0.9 * last_res || last_res < tolerance) break;
    }
    GLS_TRY(ph.present_from_evaluation_point());
    last_res = current_res;
    ++outer;
    assembly_needed = false;
  }
  if (!force_matrix_renewal) consecutive = (consecutive + 1) % std::max(skip_iterations, 1);
  st.outer = outer;
  st.final_res = current_res;
  return GLS_OK;
}

template <class Phys>
int newton_template(Phys &ph, double tolerance, int max_iterations, int verbosity, NewtonStats &st) {
  double current_res = 1.0, last_res = 1.0;
  int outer = 0;
  while (current_res > tolerance && outer < max_iterations) {
    GLS_TRY(ph.evaluation_point_from_present());          // evaluation_point = present_solution
    GLS_TRY(ph.assemble_matrix_and_rhs());
    ++st.residuals;
    if (outer == 0) {
      GLS_TRY(ph.rhs_norm(current_res));
      last_res = current_res;
    }
    if (verbosity) printf("Newton iteration: %d  - Residual:  %g\n", outer, current_res);
    int lin_it = 0;
    GLS_TRY(ph.solve_linear_system(lin_it));
    st.linear += lin_it;
    for (double alpha = 1.0; alpha > 1e-3; alpha *= 0.5) {
      GLS_TRY(ph.line_point(alpha));  // local_eval = present + alpha*update; apply_constraints; eval = local_eval
      GLS_TRY(ph.assemble_rhs());
      ++st.residuals;
      GLS_TRY(ph.rhs_norm(current_res));
      if (verbosity) printf("\t\talpha = %6g res = %g\n", alpha, current_res);
      if (current_res < 0.9 * last_res || last_res < tolerance) break;
    }
    GLS_TRY(ph.present_from_evaluation_point());  // present_solution = evaluation_point
    last_res = current_res;
    ++outer;
  }
  st.outer = outer;
  st.final_res = current_res;
  return GLS_OK;
}

// one TimerOutput::Scope of the reference (gls_navier_stokes.cc:921, 1028, 1165, 1274): host wall
// time of the section with the context stream drained on entry and exit (the reference's sections
// are synchronous host code); no cost while the timer is off
struct SectionScope {
  gls_ctx *c;
  int s;
  std::chrono::steady_clock::time_point t0;
  SectionScope(gls_ctx *c_, int s_) : c(c_), s(s_) {
    if (c->sec_on) {
      (void)hipStreamSynchronize(c->stream);
      t0 = std::chrono::steady_clock::now();
    }
  }
  ~SectionScope() {
    if (!c->sec_on) return;
    (void)hipStreamSynchronize(c->stream);
    c->sec_t[s] += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    ++c->sec_n[s];
  }
};

// GLS physics on device vectors (the GLSNavierStokesSolver side of the plugin API)
struct DevicePhysics {
  gls_ctx *c;
  double *present, *eval, *update, *rhs;
  const double *u1, *u2, *u3;
  gls_linear_params lin;
  int verbosity;
  bool skip = false;  // skip_newton: the Jacobian is frozen between assemblies (gls_freeze_jacobian)
  int linear_failures = 0;
  int evaluation_point_from_present() {
    // the state IS present (no copy): the assembly reads it, the line search writes eval; the frozen-
    // Jacobian renewal (skip) re-states eval, so it keeps the reference's copy
    if (!skip) return gls_set_state(c, present, u1, u2, u3);
    HIP_TRY(gls::vec_copy(eval, present, c->n_dofs, c->stream));
    return gls_set_state(c, eval, u1, u2, u3);
  }
  int assemble_matrix_and_rhs() {  // matrix-free: residual + the Jacobian diagonal at this state
    SectionScope t(c, GLS_SEC_ASSEMBLE_SYSTEM);
    if (skip) {  // renew the frozen Jacobian at this evaluation point
      GLS_TRY(gls_freeze_jacobian(c, 0));
      GLS_TRY(gls_set_state(c, eval, u1, u2, u3));
    }
    GLS_TRY(gls_residual_and_diagonal(c, rhs, nullptr));
    return skip ? gls_freeze_jacobian(c, 1) : GLS_OK;
  }
  int assemble_rhs() {
    SectionScope t(c, GLS_SEC_ASSEMBLE_RHS);
    return gls_residual(c, rhs);
  }
  int rhs_norm(double &r) {
    double r2;
    GLS_TRY(device_dot(c, rhs, rhs, &r2));
    r = std::sqrt(r2);
    return GLS_OK;
  }
  int solve_linear_system(int &its) {
    gls_linear_params lp = lin;
    if (c->mg.on) {  // preconditioner setup first (setup_ILU / setup_AMG, gls_navier_stokes.cc:1165, 1182)
      SectionScope t(c, GLS_SEC_SETUP_GMG);
      GLS_TRY(ensure_diag(c));
      GLS_TRY(mg_prepare(c));
    } else if (c->ilu.on && !c->ilu.probe_only) {
      SectionScope t(c, GLS_SEC_SETUP_ILU);
      GLS_TRY(ensure_diag(c));
      GLS_TRY(ensure_ilu(c));
    }
    SectionScope t(c, GLS_SEC_SOLVE_LINEAR);
    const int rc = gls_solve_linear(c, rhs, update, &lp);
    if (rc < 0 && rc != GLS_ENOCONV) return rc;
    if (rc == GLS_ENOCONV) {
      ++linear_failures;
      if (verbosity) printf("  -Iterative solver did not converge: %d steps, residual %g\n", lp.iterations, lp.final_residual);
    }
    its = lp.iterations;
    if (verbosity) printf("  -Iterative solver took : %d steps \n", lp.iterations);
    // zero_constraints.distribute(solution): constrained entries of the update are 0
    HIP_TRY(gls::vec_set_indexed(update, c->con_dofs.p, nullptr, (int64_t)c->con_dofs.n, c->stream));
    return GLS_OK;
  }
  int line_point(double alpha) {
    HIP_TRY(gls::vec_waxpy(eval, present, alpha, update, c->n_dofs, c->stream));  // eval = present + alpha update
    GLS_TRY(gls_apply_dirichlet(c, eval));  // nonzero_constraints.distribute
    return gls_set_state(c, eval, u1, u2, u3);
  }
  int present_from_evaluation_point() {
    HIP_TRY(gls::vec_copy(present, eval, c->n_dofs, c->stream));
    return GLS_OK;
  }
};

// the reference's fake physics (tests/core/non_linear_test_system_01.h:50-129)
struct KatPhysics {
  double present[2] = {1., 0.}, eval[2] = {0, 0}, update[2] = {0, 0}, rhs[2] = {0, 0};
  double J[2][2] = {{0, 0}, {0, 0}};
  int evaluation_point_from_present() { eval[0] = present[0]; eval[1] = present[1]; return GLS_OK; }
  int assemble_matrix_and_rhs() {
    J[0][0] = 2 * eval[0]; J[0][1] = 1; J[1][0] = 0; J[1][1] = 2;
    return assemble_rhs();
  }
  int assemble_rhs() {
    rhs[0] = -(eval[0] * eval[0] + eval[1]);
    rhs[1] = -(2 * eval[1] + 3);
    return GLS_OK;
  }
  int rhs_norm(double &r) { r = std::sqrt(rhs[0] * rhs[0] + rhs[1] * rhs[1]); return GLS_OK; }
  int solve_linear_system(int &its) {
    const double det = J[0][0] * J[1][1] - J[0][1] * J[1][0];
    if (det == 0.) return set_err(GLS_EINVAL, "singular KAT Jacobian");
    update[0] = (rhs[0] * J[1][1] - J[0][1] * rhs[1]) / det;
    update[1] = (J[0][0] * rhs[1] - J[1][0] * rhs[0]) / det;
    its = 1;
    return GLS_OK;
  }
  int line_point(double a) { eval[0] = present[0] + a * update[0]; eval[1] = present[1] + a * update[1]; return GLS_OK; }
  int present_from_evaluation_point() { present[0] = eval[0]; present[1] = eval[1]; return GLS_OK; }
};

}  // namespace

extern "C" {

int gls_newton_solve(gls_ctx *c, double *present, const double *u1, const double *u2, const double *u3,
                     gls_newton_params *prm) {
  GLS_TRY(check_ctx(c));
  if (!present || !prm) return set_err(GLS_EINVAL, "null argument");
  const int64_t n = c->n_dofs;
  if (!c->tmp3.p) {
    GLS_TRY(c->tmp3.alloc(n));  // evaluation_point
    GLS_TRY(c->tmp4.alloc(n));  // newton_update
    GLS_TRY(c->tmp5.alloc(n));  // system_rhs
  }
  DevicePhysics ph{c, present, c->tmp3.p, c->tmp4.p, c->tmp5.p, u1, u2, u3, prm->lin, prm->verbosity};
  NewtonStats st;
  if (prm->solver == GLS_SKIP_NEWTON) {
    ph.skip = true;
    GLS_TRY(skip_newton_template(ph, prm->tolerance, prm->max_iterations, prm->verbosity, prm->skip_iterations,
                                 prm->is_initial_step != 0, prm->force_matrix_renewal != 0, c->skip_consecutive, st));
  } else {
    GLS_TRY(gls_freeze_jacobian(c, 0));
    GLS_TRY(newton_template(ph, prm->tolerance, prm->max_iterations, prm->verbosity, st));
  }
  HIP_TRY(hipStreamSynchronize(c->stream));
  prm->newton_iterations = st.outer;
  prm->linear_iterations = st.linear;
  prm->residual_evaluations = st.residuals;
  prm->final_residual = st.final_res;
  prm->linear_failures = ph.linear_failures;
  return GLS_OK;
}

int gls_section_timing(gls_ctx *c, int enable) {
  GLS_TRY(check_ctx(c));
  c->sec_on = enable != 0;
  for (int i = 0; i < GLS_N_SECTIONS; ++i) {
    c->sec_t[i] = 0.;
    c->sec_n[i] = 0;
  }
  return GLS_OK;
}
int gls_section_get(const gls_ctx *c, int section, double *seconds, int *calls) {
  if (!c) return set_err(GLS_EINVAL, "null context");
  if (section < 0 || section >= GLS_N_SECTIONS) return set_err(GLS_EINVAL, "section %d", section);
  if (seconds) *seconds = c->sec_t[section];
  if (calls) *calls = c->sec_n[section];
  return GLS_OK;
}

// Newton KAT (tests/core/newton_non_linear_solver_01.cc: tol 1e-8, max 10 iterations)
int gls_newton_selftest(double xo[2]) {
  if (!xo) return set_err(GLS_EINVAL, "null");
  KatPhysics ph;
  NewtonStats st;
  GLS_TRY(newton_template(ph, 1e-8, 10, 0, st));
  xo[0] = ph.present[0];
  xo[1] = ph.present[1];
  return GLS_OK;
}

// SkipNewton KAT (tests/core/skip_newton_non_linear_solver_01.cc: tol 1e-8, max 10 iterations,
// skip iterations as given; solve_non_linear_system(steady, true, true))
int gls_skip_newton_selftest(int skip_iterations, double xo[2]) {
  if (!xo || skip_iterations < 1) return set_err(GLS_EINVAL, "gls_skip_newton_selftest arguments");
  KatPhysics ph;
  NewtonStats st;
  int consecutive = 0;
  GLS_TRY(skip_newton_template(ph, 1e-8, 10, 0, skip_iterations, true, true, consecutive, st));
  xo[0] = ph.present[0];
  xo[1] = ph.present[1];
  return GLS_OK;
}

// --------------------------------------------------------------------------------------------
// hyper_cube + refine_global, Morton (z-order) cells, lexicographic nodes
// --------------------------------------------------------------------------------------------
int gls_mesh_hyper_cube_sizes(int dim, int n, int k, int kp, int pmask, int64_t *nc, int64_t *nv, int64_t *np) {
  if ((dim != 2 && dim != 3) || n <= 0 || k <= 0 || kp <= 0) return set_err(GLS_EINVAL, "mesh args");
  int64_t c = 1, v = 1, p = 1;
  for (int d = 0; d < dim; ++d) {
    const bool per = (pmask >> d) & 1;
    c *= n;
    v *= (int64_t)k * n + (per ? 0 : 1);
    p *= (int64_t)kp * n + (per ? 0 : 1);
  }
  if (nc) *nc = c;
  if (nv) *nv = v;
  if (np) *np = p;
  return GLS_OK;
}

int gls_mesh_hyper_cube(int dim, int n, int k, int kp, double lo, double hi, int pmask, int32_t *cv, int32_t *cp,
                        double *x0, double *h) {
  int64_t nc, nv, np;
  GLS_TRY(gls_mesh_hyper_cube_sizes(dim, n, k, kp, pmask, &nc, &nv, &np));
  if (nv > INT32_MAX || np > INT32_MAX) return set_err(GLS_EINVAL, "mesh too large for int32 node ids");
  int L = 0;
  while ((1 << L) < n) ++L;
  const double hc = (hi - lo) / n;
  int vsh[3], psh[3];
  for (int d = 0; d < 3; ++d) {
    const bool per = (pmask >> d) & 1;
    vsh[d] = k * n + (per ? 0 : 1);
    psh[d] = kp * n + (per ? 0 : 1);
  }
  const int nvl = gls::ipow(k + 1, dim), npl = gls::ipow(kp + 1, dim);
  int64_t cell = 0;
  const int64_t total = (int64_t)1 << (dim * L);
  for (int64_t mcode = 0; mcode < total; ++mcode) {
    int ijk[3] = {0, 0, 0};
    for (int b = 0; b < L; ++b)
      for (int d = 0; d < dim; ++d) ijk[d] |= (int)((mcode >> (b * dim + d)) & 1) << b;
    bool inside = true;
    for (int d = 0; d < dim; ++d) inside = inside && ijk[d] < n;
    if (!inside) continue;
    for (int a = 0; a < nvl; ++a) {
      int loc[3] = {a % (k + 1), (a / (k + 1)) % (k + 1), a / ((k + 1) * (k + 1))};
      int64_t id = 0, stride = 1;
      for (int d = 0; d < dim; ++d) {
        id += (int64_t)((ijk[d] * k + loc[d]) % vsh[d]) * stride;
        stride *= vsh[d];
      }
      cv[cell * nvl + a] = (int32_t)id;
    }
    if (cp) {
      for (int a = 0; a < npl; ++a) {
        int loc[3] = {a % (kp + 1), (a / (kp + 1)) % (kp + 1), a / ((kp + 1) * (kp + 1))};
        int64_t id = 0, stride = 1;
        for (int d = 0; d < dim; ++d) {
          id += (int64_t)((ijk[d] * kp + loc[d]) % psh[d]) * stride;
          stride *= psh[d];
        }
        cp[cell * npl + a] = (int32_t)id;
      }
    }
    for (int d = 0; d < dim; ++d) {
      if (x0) x0[cell * dim + d] = lo + ijk[d] * hc;
      if (h) h[cell * dim + d] = hc;
    }
    ++cell;
  }
  return cell == nc ? GLS_OK : set_err(GLS_EINVAL, "morton enumeration mismatch");
}

// --------------------------------------------------------------------------------------------
// timing
// --------------------------------------------------------------------------------------------
int gls_timing_enable(gls_ctx *c, int en) {
  GLS_TRY(check_ctx(c));
  c->timing = en != 0;
  return GLS_OK;
}
int gls_timing_reset(gls_ctx *c) {
  GLS_TRY(check_ctx(c));
  HIP_TRY(hipStreamSynchronize(c->stream));
  for (auto &e : c->events) { (void)hipEventDestroy(e.a); (void)hipEventDestroy(e.b); }
  c->events.clear();
  for (int i = 0; i < 6; ++i) { c->t_ms[i] = 0; c->t_n[i] = 0; }
  return GLS_OK;
}
int gls_timing_get(gls_ctx *c, int which, double *ms, int64_t *cnt) {
  GLS_TRY(check_ctx(c));
  if (which < 0 || which > 5) return set_err(GLS_EINVAL, "which");
  HIP_TRY(hipStreamSynchronize(c->stream));
  for (auto &e : c->events) {
    float t = 0;
    HIP_TRY(hipEventElapsedTime(&t, e.a, e.b));
    c->t_ms[e.which] += t;
    c->t_n[e.which] += 1;
    (void)hipEventDestroy(e.a);
    (void)hipEventDestroy(e.b);
  }
  c->events.clear();
  if (ms) *ms = c->t_ms[which];
  if (cnt) *cnt = c->t_n[which];
  return GLS_OK;
}

}  // extern "C"


// ---------------------------------------------------------------------------------------------
// gls_ilu_attach: the reference's ILU-preconditioned GMRES (linear solver method gmres with 'ilu
// preconditioner fill / absolute tolerance / relative tolerance', setup_ILU gls_navier_stokes.cc:
// 1161-1176: Ifpack ILU(k) with athresh / rthresh, no overlap) on the assembled Jacobian. The matrix
// is never formed by a CPU: it is probed from the device operator with distance-2-colored unit
// vectors (no two DoFs of a probe share a row). Its graph is the reference's system-matrix sparsity
// (make_sparsity_pattern with nonzero_constraints, keep_constrained_dofs = false,
// gls_navier_stokes.cc:208-211): a constrained row / column holds its diagonal only, lines
// (hanging nodes, slip on curved walls) couple their masters. The DoFs are renumbered like
// DoFRenumbering::Cuthill_McKee (gls_navier_stokes.cc:70), the level-of-fill pattern of ILU(fill)
// is inserted with explicit zeros, and rocSPARSE csrilu0 on that pattern computes ILU(fill).
// ---------------------------------------------------------------------------------------------
extern "C" int gls_ilu_attach(gls_ctx *c, int fill, double athresh, double rthresh) {
  GLS_TRY(check_ctx(c));
  auto &I = c->ilu;
  I.probe_only = false;  // a caller's attach: a preconditioner (mg_probe_setup marks its own afterwards)
  if (c->dist.on && !c->dist.dofs) return set_err(GLS_EINVAL, "gls_ilu_attach: brick-partitioned contexts use the multigrid");
  if (c->mg.on) return set_err(GLS_EINVAL, "gls_ilu_attach: a multigrid preconditioner is attached");
  if (fill < 0 || fill > GLS_ILU_MAX_FILL)
    return set_err(GLS_EINVAL, "gls_ilu_attach: ilu preconditioner fill %d not supported (0..%d)", fill, GLS_ILU_MAX_FILL);
  const int dim = c->dim, nvc = gls::ipow(c->k + 1, dim);
  const bool sep = c->cell_pnodes.p != nullptr;
  const int npc = sep ? gls::ipow(c->kp + 1, dim) : 0;
  const int64_t nv = c->n_vnodes, np = c->n_pnodes, nc = c->n_cells, n = c->n_dofs;
  if (n >= INT32_MAX) return set_err(GLS_EINVAL, "gls_ilu_attach: too many DoFs for 32-bit CSR");
  std::vector<int32_t> cv((size_t)nc * nvc), cp((size_t)nc * npc);
  HIP_TRY(hipMemcpy(cv.data(), c->cell_vnodes.p, cv.size() * sizeof(int32_t), hipMemcpyDeviceToHost));
  if (sep) HIP_TRY(hipMemcpy(cp.data(), c->cell_pnodes.p, cp.size() * sizeof(int32_t), hipMemcpyDeviceToHost));
  // unified nodes: velocity nodes [0, nv), separate pressure nodes [nv, nv + np)
  const int64_t nu = nv + (sep ? np : 0);
  const int ncn = nvc + npc;
  auto cell_node = [&](int64_t cell, int a) -> int64_t {
    return a < nvc ? cv[(size_t)(cell * nvc + a)] : nv + cp[(size_t)(cell * npc + a - nvc)];
  };
  // DoFs of a unified node and their probe slot (component; dim = pressure)
  auto node_dofs = [&](int64_t x, int64_t *d, int *slot) -> int {
    if (x >= nv) { d[0] = dim * nv + (x - nv); slot[0] = dim; return 1; }
    int m = 0;
    for (int cc = 0; cc < dim; ++cc) { d[m] = x * dim + cc; slot[m++] = cc; }
    if (!sep) { d[m] = dim * nv + x; slot[m++] = dim; }
    return m;
  };
  const int64_t nvd = (int64_t)dim * nv;
  auto unode = [&](int64_t d) { return d < nvd ? d / dim : (sep ? nv + (d - nvd) : d - nvd); };
  // constrained DoFs (zero_constraints: Dirichlet + lines) and the operator lines (Dirichlet masters
  // drop out, as in the closed AffineConstraints)
  std::vector<char> cons((size_t)n, 0), isline((size_t)n, 0);
  {
    std::vector<int64_t> cd(c->con_dofs.n);
    if (!cd.empty()) HIP_TRY(hipMemcpy(cd.data(), c->con_dofs.p, cd.size() * sizeof(int64_t), hipMemcpyDeviceToHost));
    for (int64_t d : cd) cons[(size_t)d] = 1;
  }
  std::vector<int64_t> lidx((size_t)n, -1);
  if (c->hang.on)
    for (size_t i = 0; i + 1 < c->hang.h_off.size(); ++i) {
      lidx[(size_t)c->hang.h_dof[i]] = (int64_t)i;
      isline[(size_t)c->hang.h_dof[i]] = 1;
    }
  // across ranks (Ifpack additive Schwarz, overlap 0, as the reference runs with MPI): each rank
  // factors its owned rows and columns; ghost DoFs are identity rows and drop out of the pattern
  auto ghost = [&](int64_t d) {
    if (!c->dist.on) return false;
    return d < nvd ? d / dim >= c->dist.n_owned : d - nvd >= c->dist.n_owned_p;
  };
  const std::vector<char> fcons = cons;  // constrained DoFs before the ghosts join them (complete rows)
  for (int64_t d = 0; d < n; ++d)
    if (ghost(d)) cons[(size_t)d] = 1;
  auto dirichlet = [&](int64_t d) { return (cons[(size_t)d] && !isline[(size_t)d]) || ghost(d); };
  // effective DoFs of each cell: its unconstrained DoFs and the (non-Dirichlet) masters of its lines
  std::vector<int64_t> effoff((size_t)nc + 1, 0), eff;
  {
    std::vector<int64_t> buf;
    for (int64_t e = 0; e < nc; ++e) {
      buf.clear();
      for (int a = 0; a < ncn; ++a) {
        int64_t d[4];
        int sl[4];
        const int m = node_dofs(cell_node(e, a), d, sl);
        for (int j = 0; j < m; ++j) {
          const int64_t li = lidx[(size_t)d[j]];
          if (li >= 0 && !ghost(d[j])) {
            for (int64_t t = c->hang.h_off[(size_t)li]; t < c->hang.h_off[(size_t)li + 1]; ++t)
              if (!dirichlet(c->hang.h_master[(size_t)t])) buf.push_back(c->hang.h_master[(size_t)t]);
          } else if (!cons[(size_t)d[j]]) {
            buf.push_back(d[j]);
          }
        }
      }
      std::sort(buf.begin(), buf.end());
      buf.erase(std::unique(buf.begin(), buf.end()), buf.end());
      eff.insert(eff.end(), buf.begin(), buf.end());
      effoff[(size_t)e + 1] = (int64_t)eff.size();
    }
  }
  // DoF -> cells whose effective list holds it
  std::vector<int64_t> dcoff((size_t)n + 1, 0), dcell;
  for (int64_t d : eff) ++dcoff[(size_t)d + 1];
  for (int64_t i = 0; i < n; ++i) dcoff[(size_t)i + 1] += dcoff[(size_t)i];
  dcell.resize((size_t)dcoff[(size_t)n]);
  {
    std::vector<int64_t> f(dcoff.begin(), dcoff.end() - 1);
    for (int64_t e = 0; e < nc; ++e)
      for (int64_t t = effoff[(size_t)e]; t < effoff[(size_t)e + 1]; ++t) dcell[(size_t)f[(size_t)eff[(size_t)t]]++] = e;
  }
  // rows of the system matrix (old numbering, sorted): an unconstrained DoF couples the effective DoFs
  // of its cells; a constrained DoF only itself
  std::vector<int64_t> aoff((size_t)n + 1, 0), acol;
  {
    std::vector<int64_t> stamp((size_t)n, -1), buf;
    for (int64_t i = 0; i < n; ++i) {
      buf.clear();
      buf.push_back(i);
      stamp[(size_t)i] = i;
      if (!cons[(size_t)i])
        for (int64_t t = dcoff[(size_t)i]; t < dcoff[(size_t)i + 1]; ++t) {
          const int64_t e = dcell[(size_t)t];
          for (int64_t u = effoff[(size_t)e]; u < effoff[(size_t)e + 1]; ++u) {
            const int64_t j = eff[(size_t)u];
            if (stamp[(size_t)j] != i) { stamp[(size_t)j] = i; buf.push_back(j); }
          }
        }
      std::sort(buf.begin(), buf.end());
      acol.insert(acol.end(), buf.begin(), buf.end());
      aoff[(size_t)i + 1] = (int64_t)acol.size();
    }
  }
  // node graph of that pattern (x ~ y when a row of x holds a DoF of y) for the distance-2 coloring
  std::vector<int64_t> n1off((size_t)nu + 1, 0), n1;
  {
    std::vector<int64_t> stamp((size_t)nu, -1), buf;
    for (int64_t x = 0; x < nu; ++x) {
      buf.clear();
      buf.push_back(x);
      stamp[(size_t)x] = x;
      int64_t d[4];
      int sl[4];
      const int m = node_dofs(x, d, sl);
      for (int j = 0; j < m; ++j)
        for (int64_t t = aoff[(size_t)d[j]]; t < aoff[(size_t)d[j] + 1]; ++t) {
          const int64_t y = unode(acol[(size_t)t]);
          if (stamp[(size_t)y] != x) { stamp[(size_t)y] = x; buf.push_back(y); }
        }
      std::sort(buf.begin(), buf.end());
      n1.insert(n1.end(), buf.begin(), buf.end());
      n1off[(size_t)x + 1] = (int64_t)n1.size();
    }
  }
  // greedy distance-2 coloring of the unified nodes
  std::vector<int> color((size_t)nu, -1), mark;
  int ncol = 0;
  for (int64_t x = 0; x < nu; ++x) {
    for (int64_t t = n1off[(size_t)x]; t < n1off[(size_t)x + 1]; ++t) {
      const int64_t z = n1[(size_t)t];
      for (int64_t u = n1off[(size_t)z]; u < n1off[(size_t)z + 1]; ++u) {
        const int cy = color[(size_t)n1[(size_t)u]];
        if (cy >= 0) {
          if ((int)mark.size() <= cy) mark.resize((size_t)cy + 1, -1);
          mark[(size_t)cy] = (int)x;
        }
      }
    }
    int col = 0;
    while (col < (int)mark.size() && mark[(size_t)col] == (int)x) ++col;
    color[(size_t)x] = col;
    ncol = std::max(ncol, col + 1);
  }
  // Across ranks, complete owned rows (the rows of Ifpack's distributed matrix, restricted to the owned
  // columns as its additive Schwarz with overlap 0 does): the owned x owned block also receives the
  // neighbours' cells. Every rank probes its cells' operator on ALL its DoFs (owned and ghost) with a
  // distance-2 coloring of that full local pattern; the ghost rows of each probe go to their owners
  // through the export exchange, tagged once (here) with the column as its position in the owner's
  // send list. Probe rounds run to the largest probe count of any rank (collective).
  std::vector<char> aown;  // per system-matrix entry: probed on this rank (else a neighbour's entry only)
  struct RemoteEntry {
    int32_t round, slot;
    int64_t i, j;
  };
  std::vector<RemoteEntry> remote;
  int n_rounds = 0;
  const bool cmpl = c->dist.on && c->dist.dofs;
  if (cmpl) {
    auto fdir = [&](int64_t d) { return fcons[(size_t)d] && !isline[(size_t)d]; };
    std::vector<int64_t> feoff((size_t)nc + 1, 0), feff, buf;
    for (int64_t e = 0; e < nc; ++e) {
      buf.clear();
      for (int a = 0; a < ncn; ++a) {
        int64_t d[4];
        int sl[4];
        const int m = node_dofs(cell_node(e, a), d, sl);
        for (int j = 0; j < m; ++j) {
          const int64_t li = lidx[(size_t)d[j]];
          if (li >= 0) {
            for (int64_t t = c->hang.h_off[(size_t)li]; t < c->hang.h_off[(size_t)li + 1]; ++t)
              if (!fdir(c->hang.h_master[(size_t)t])) buf.push_back(c->hang.h_master[(size_t)t]);
          } else if (!fcons[(size_t)d[j]]) {
            buf.push_back(d[j]);
          }
        }
      }
      std::sort(buf.begin(), buf.end());
      buf.erase(std::unique(buf.begin(), buf.end()), buf.end());
      feff.insert(feff.end(), buf.begin(), buf.end());
      feoff[(size_t)e + 1] = (int64_t)feff.size();
    }
    std::vector<int64_t> fdoff((size_t)n + 1, 0), fdcell;
    for (int64_t d : feff) ++fdoff[(size_t)d + 1];
    for (int64_t i = 0; i < n; ++i) fdoff[(size_t)i + 1] += fdoff[(size_t)i];
    fdcell.resize((size_t)fdoff[(size_t)n]);
    {
      std::vector<int64_t> f(fdoff.begin(), fdoff.end() - 1);
      for (int64_t e = 0; e < nc; ++e)
        for (int64_t t = feoff[(size_t)e]; t < feoff[(size_t)e + 1]; ++t) fdcell[(size_t)f[(size_t)feff[(size_t)t]]++] = e;
    }
    std::vector<int64_t> faoff((size_t)n + 1, 0), facol;
    {
      std::vector<int64_t> stamp((size_t)n, -1);
      for (int64_t i = 0; i < n; ++i) {
        buf.clear();
        buf.push_back(i);
        stamp[(size_t)i] = i;
        if (!fcons[(size_t)i])
          for (int64_t t = fdoff[(size_t)i]; t < fdoff[(size_t)i + 1]; ++t) {
            const int64_t e = fdcell[(size_t)t];
            for (int64_t u = feoff[(size_t)e]; u < feoff[(size_t)e + 1]; ++u) {
              const int64_t j = feff[(size_t)u];
              if (stamp[(size_t)j] != i) { stamp[(size_t)j] = i; buf.push_back(j); }
            }
          }
        std::sort(buf.begin(), buf.end());
        facol.insert(facol.end(), buf.begin(), buf.end());
        faoff[(size_t)i + 1] = (int64_t)facol.size();
      }
    }
    // distance-2 coloring of the full pattern's node graph (replaces the owned-block coloring)
    std::vector<int64_t> g1off((size_t)nu + 1, 0), g1;
    {
      std::vector<int64_t> stamp((size_t)nu, -1);
      for (int64_t x = 0; x < nu; ++x) {
        buf.clear();
        buf.push_back(x);
        stamp[(size_t)x] = x;
        int64_t d[4];
        int sl[4];
        const int m = node_dofs(x, d, sl);
        for (int j = 0; j < m; ++j)
          for (int64_t t = faoff[(size_t)d[j]]; t < faoff[(size_t)d[j] + 1]; ++t) {
            const int64_t y = unode(facol[(size_t)t]);
            if (stamp[(size_t)y] != x) { stamp[(size_t)y] = x; buf.push_back(y); }
          }
        std::sort(buf.begin(), buf.end());
        g1.insert(g1.end(), buf.begin(), buf.end());
        g1off[(size_t)x + 1] = (int64_t)g1.size();
      }
    }
    std::fill(color.begin(), color.end(), -1);
    mark.clear();
    ncol = 0;
    for (int64_t x = 0; x < nu; ++x) {
      for (int64_t t = g1off[(size_t)x]; t < g1off[(size_t)x + 1]; ++t) {
        const int64_t z = g1[(size_t)t];
        for (int64_t u = g1off[(size_t)z]; u < g1off[(size_t)z + 1]; ++u) {
          const int cy = color[(size_t)g1[(size_t)u]];
          if (cy >= 0) {
            if ((int)mark.size() <= cy) mark.resize((size_t)cy + 1, -1);
            mark[(size_t)cy] = (int)x;
          }
        }
      }
      int col = 0;
      while (col < (int)mark.size() && mark[(size_t)col] == (int)x) ++col;
      color[(size_t)x] = col;
      ncol = std::max(ncol, col + 1);
    }
    auto pof = [&](int64_t d) { return color[(size_t)unode(d)] * (dim + 1) + (d < nvd ? (int)(d % dim) : dim); };
    const int nprobe_local = ncol * (dim + 1);
    // the column tags: per round, each ghost row's probed column as its position in the owner's list
    auto &D = c->dist;
    const int nn = (int)D.h_soff.size() - 1;
    const int64_t ns = D.n_send, nr = D.n_recv;
    std::vector<int32_t> gnb((size_t)n, -1), gk((size_t)n, -1);
    for (int t = 0; t < nn; ++t)
      for (int64_t q = D.h_roff[(size_t)t]; q < D.h_roff[(size_t)t + 1]; ++q) {
        gnb[(size_t)D.h_recv[(size_t)q]] = t;
        gk[(size_t)D.h_recv[(size_t)q]] = (int32_t)(q - D.h_roff[(size_t)t]);
      }
    std::vector<double> hpos((size_t)std::max<int64_t>(nr, 1)), hin((size_t)std::max<int64_t>(ns, 1));
    for (int p = 0;; ++p) {
      double flag = p < nprobe_local ? 1.0 : 0.0;
      HIP_TRY(hipMemcpy(D.red_buf, &flag, sizeof(double), hipMemcpyHostToDevice));
      if (D.allreduce(D.user, D.red_buf, 1) != 0) return set_err(GLS_ECOMM, "gls_ilu_attach: allreduce failed");
      HIP_TRY(hipStreamSynchronize(c->stream));
      HIP_TRY(hipMemcpy(&flag, D.red_buf, sizeof(double), hipMemcpyDeviceToHost));
      if (flag == 0.0) break;
      ++n_rounds;
      for (int64_t q = 0; q < nr; ++q) {
        const int64_t i = D.h_recv[(size_t)q];
        double pos = -1.0;
        if (p < nprobe_local && !fcons[(size_t)i])
          for (int64_t t = faoff[(size_t)i]; t < faoff[(size_t)i + 1]; ++t) {
            const int64_t j = facol[(size_t)t];
            if (pof(j) != p) continue;
            if (gnb[(size_t)j] == gnb[(size_t)i]) pos = (double)gk[(size_t)j];
            break;
          }
        hpos[(size_t)q] = pos;
      }
      if (nr) HIP_TRY(hipMemcpy(D.recv_buf, hpos.data(), sizeof(double) * (size_t)nr, hipMemcpyHostToDevice));
      HIP_TRY(hipDeviceSynchronize());
      if (D.xchg(D.user, 1) != 0) return set_err(GLS_ECOMM, "gls_ilu_attach: exchange failed");
      HIP_TRY(hipStreamSynchronize(c->stream));
      if (ns) HIP_TRY(hipMemcpy(hin.data(), D.send_buf, sizeof(double) * (size_t)ns, hipMemcpyDeviceToHost));
      for (int t = 0; t < nn; ++t)
        for (int64_t q = D.h_soff[(size_t)t]; q < D.h_soff[(size_t)t + 1]; ++q) {
          const int64_t pos = (int64_t)hin[(size_t)q];
          if (pos < 0) continue;
          if (pos >= D.h_soff[(size_t)t + 1] - D.h_soff[(size_t)t]) return set_err(GLS_ECOMM, "gls_ilu_attach: bad column tag");
          const int64_t i = D.h_send[(size_t)q], j = D.h_send[(size_t)(D.h_soff[(size_t)t] + pos)];
          if (cons[(size_t)i] || cons[(size_t)j]) continue;
          remote.push_back({p, (int32_t)q, i, j});
        }
    }
    // the system matrix's rows gain the neighbours' couplings
    std::vector<std::vector<int64_t>> extra((size_t)n);
    for (const auto &r : remote) extra[(size_t)r.i].push_back(r.j);
    std::vector<int64_t> noff((size_t)n + 1, 0), ncl_;
    for (int64_t i = 0; i < n; ++i) {
      const size_t s0 = ncl_.size();
      for (int64_t t = aoff[(size_t)i]; t < aoff[(size_t)i + 1]; ++t) ncl_.push_back(acol[(size_t)t]);
      auto &x = extra[(size_t)i];
      std::sort(x.begin(), x.end());
      for (int64_t j : x)
        if (!std::binary_search(acol.begin() + aoff[(size_t)i], acol.begin() + aoff[(size_t)i + 1], j)) ncl_.push_back(j);
      std::sort(ncl_.begin() + (std::ptrdiff_t)s0, ncl_.end());
      ncl_.erase(std::unique(ncl_.begin() + (std::ptrdiff_t)s0, ncl_.end()), ncl_.end());
      noff[(size_t)i + 1] = (int64_t)ncl_.size();
    }
    aown.assign(ncl_.size(), 0);
    for (int64_t i = 0; i < n; ++i)
      for (int64_t t = noff[(size_t)i]; t < noff[(size_t)i + 1]; ++t)
        aown[(size_t)t] = std::binary_search(acol.begin() + aoff[(size_t)i], acol.begin() + aoff[(size_t)i + 1], ncl_[(size_t)t]);
    aoff.swap(noff);
    acol.swap(ncl_);
  } else {
    aown.assign(acol.size(), 1);
  }
  // Cuthill-McKee (deal.II) on the unconstrained cell-coupling graph of the DoF handler. Its nodes
  // carry deal.II's per-support-point DoF groups: a velocity node's components followed by the
  // pressure DoF at the same point (Q(k)-Q(kp) with kp | k: a pressure node sits on the velocity node
  // of the same lexicographic position in every cell; the map is checked cell by cell)
  std::vector<int64_t> p_at((size_t)std::max<int64_t>(np, 1), -1);  // pressure node -> velocity node
  bool p_map = sep && c->k % c->kp == 0;
  if (p_map) {
    const int r = c->k / c->kp, k1 = c->k + 1, kp1 = c->kp + 1;
    for (int64_t e = 0; e < nc && p_map; ++e)
      for (int a = 0; a < npc; ++a) {
        const int ax = a % kp1, ay = (a / kp1) % kp1, az = dim == 3 ? a / (kp1 * kp1) : 0;
        const int va = ax * r + k1 * (ay * r) + (dim == 3 ? k1 * k1 * az * r : 0);
        const int64_t pn = cp[(size_t)(e * npc + a)], vn = cv[(size_t)(e * nvc + va)];
        if (p_at[(size_t)pn] < 0) p_at[(size_t)pn] = vn;
        else if (p_at[(size_t)pn] != vn) { p_map = false; break; }
      }
  }
  // CM nodes: velocity nodes (+ their pressure DoF), then unmapped pressure nodes
  std::vector<int64_t> cmnode((size_t)nu, -1);  // unified node -> CM node
  int64_t ncm = 0;
  for (int64_t x = 0; x < nv; ++x) cmnode[(size_t)x] = ncm++;
  if (sep)
    for (int64_t pn = 0; pn < np; ++pn)  // (a ghost pressure node in no local cell -- a line master only -- is its own node)
      cmnode[(size_t)(nv + pn)] = p_map && p_at[(size_t)pn] >= 0 ? cmnode[(size_t)p_at[(size_t)pn]] : ncm++;
  std::vector<int64_t> cm_doff((size_t)ncm + 1, 0), cm_dofs((size_t)n);
  for (int64_t x = 0; x < nu; ++x) {
    int64_t d[4];
    int sl[4];
    cm_doff[(size_t)cmnode[(size_t)x] + 1] += node_dofs(x, d, sl);
  }
  for (int64_t y = 0; y < ncm; ++y) cm_doff[(size_t)y + 1] += cm_doff[(size_t)y];
  {
    std::vector<int64_t> f(cm_doff.begin(), cm_doff.end() - 1);
    for (int64_t x = 0; x < nu; ++x) {  // velocity nodes come first: their components precede p
      int64_t d[4];
      int sl[4];
      const int m = node_dofs(x, d, sl);
      for (int j = 0; j < m; ++j) cm_dofs[(size_t)f[(size_t)cmnode[(size_t)x]]++] = d[j];
    }
  }
  std::vector<int64_t> cadj_off((size_t)ncm + 1, 0), cadj;
  {
    std::vector<int64_t> ccoff((size_t)ncm + 1, 0), ccell;  // CM node -> cells
    for (int64_t e = 0; e < nc; ++e)
      for (int a = 0; a < ncn; ++a) ++ccoff[(size_t)cmnode[(size_t)cell_node(e, a)] + 1];
    for (int64_t y = 0; y < ncm; ++y) ccoff[(size_t)y + 1] += ccoff[(size_t)y];
    ccell.resize((size_t)ccoff[(size_t)ncm]);
    std::vector<int64_t> f(ccoff.begin(), ccoff.end() - 1);
    for (int64_t e = 0; e < nc; ++e)
      for (int a = 0; a < ncn; ++a) ccell[(size_t)f[(size_t)cmnode[(size_t)cell_node(e, a)]]++] = e;
    std::vector<int64_t> stamp((size_t)ncm, -1), buf;
    for (int64_t y = 0; y < ncm; ++y) {
      buf.clear();
      buf.push_back(y);
      stamp[(size_t)y] = y;
      for (int64_t t = ccoff[(size_t)y]; t < ccoff[(size_t)y + 1]; ++t)
        for (int a = 0; a < ncn; ++a) {
          const int64_t z = cmnode[(size_t)cell_node(ccell[(size_t)t], a)];
          if (stamp[(size_t)z] != y) { stamp[(size_t)z] = y; buf.push_back(z); }
        }
      std::sort(buf.begin(), buf.end());
      cadj.insert(cadj.end(), buf.begin(), buf.end());
      cadj_off[(size_t)y + 1] = (int64_t)cadj.size();
    }
  }
  std::vector<int64_t> order;
  gls::cuthill_mckee_nodes(ncm, cadj_off, cadj, cm_doff, cm_dofs, order);
  if ((int64_t)order.size() != n) return set_err(GLS_EINVAL, "gls_ilu_attach: renumbering covers %lld of %lld DoFs", (long long)order.size(), (long long)n);
  {
    std::vector<char> seen((size_t)n, 0);
    for (int64_t d : order)
      if (d < 0 || d >= n || seen[(size_t)d]++) return set_err(GLS_EINVAL, "gls_ilu_attach: renumbering is not a permutation");
  }
  // subdomains (Ifpack's additive Schwarz with overlap 0, which the reference runs with one block per
  // MPI rank): contiguous ranges of the cell order (space-filling: leaf order of the forest / Morton
  // bricks), a DoF in the block of its lowest cell; couplings between blocks are dropped, each block
  // is factored on its own, the blocks' triangular solves run side by side
  const int nblk = I.block_dofs > 0 ? (int)std::min<int64_t>(std::max<int64_t>((n + I.block_dofs - 1) / I.block_dofs, 1), nc) : 1;
  std::vector<int32_t> dblk((size_t)n, 0);
  std::vector<int64_t> dnode_((size_t)n, 0);  // DoF -> unified node
  for (int64_t x = 0; x < nu; ++x) {
    int64_t d[4];
    int sl[4];
    const int m = node_dofs(x, d, sl);
    for (int j = 0; j < m; ++j) dnode_[(size_t)d[j]] = x;
  }
  if (nblk > 1) {
    std::vector<int32_t> nodeblk((size_t)nu, INT32_MAX);
    for (int64_t e = 0; e < nc; ++e) {
      const int32_t b = (int32_t)(e * nblk / nc);
      for (int a = 0; a < ncn; ++a) {
        int32_t &nb_ = nodeblk[(size_t)cell_node(e, a)];
        nb_ = std::min(nb_, b);
      }
    }
    for (int64_t d = 0; d < n; ++d) {
      const int32_t b = nodeblk[(size_t)dnode_[(size_t)d]];
      dblk[(size_t)d] = b == INT32_MAX ? 0 : b;
    }
  }
  std::vector<int32_t> dcolor;  // multicolor: each DoF's color (its node's)
  if (I.ordering == GLS_ILU_ORDER_MULTICOLOR) {
    // multicolor order: a greedy distance-1 coloring of the node graph of the system matrix (nodes
    // visited in Cuthill-McKee order); DoFs sorted by (color, node's first Cuthill-McKee position,
    // position), so a node's DoFs stay consecutive. Same-colored nodes share no matrix entry: each
    // color's diagonal block is block-diagonal by node, and the triangular solves' dependency chain
    // is ~colors x DoFs per node. (Blocks only drop couplings here: the colors stay outermost.)
    std::vector<int> c1((size_t)nu, -1), used;
    int ncl = 0;
    // visit order of the greedy coloring: Cuthill-McKee (smallest-last ordering gave 36 instead of 46 colors but
    // 104 instead of 60 GMRES iterations, profiles/r03_ilu_coloring_ab.txt)
    std::vector<int64_t> visit;
    visit.reserve((size_t)nu);
    std::vector<char> seen((size_t)nu, 0);
    for (int64_t t = 0; t < n; ++t) {
      const int64_t x = dnode_[(size_t)order[(size_t)t]];
      if (!seen[(size_t)x]) {
        seen[(size_t)x] = 1;
        visit.push_back(x);
      }
    }
    for (const int64_t x : visit) {
      if (c1[(size_t)x] >= 0) continue;
      for (int64_t u = n1off[(size_t)x]; u < n1off[(size_t)x + 1]; ++u) {
        const int cy = c1[(size_t)n1[(size_t)u]];
        if (cy >= 0) {
          if ((int)used.size() <= cy) used.resize((size_t)cy + 1, -1);
          used[(size_t)cy] = (int)x;
        }
      }
      int col = 0;
      while (col < (int)used.size() && used[(size_t)col] == (int)x) ++col;
      c1[(size_t)x] = col;
      ncl = std::max(ncl, col + 1);
    }
    I.n_order_colors = ncl;
    std::vector<int64_t> npos((size_t)nu, INT64_MAX), pos((size_t)n);
    for (int64_t t = 0; t < n; ++t) {
      pos[(size_t)order[(size_t)t]] = t;
      int64_t &np_ = npos[(size_t)dnode_[(size_t)order[(size_t)t]]];
      np_ = std::min(np_, t);
    }
    dcolor.assign((size_t)n, 0);
    for (int64_t d = 0; d < n; ++d) dcolor[(size_t)d] = c1[(size_t)dnode_[(size_t)d]];
    std::sort(order.begin(), order.end(), [&](int64_t a, int64_t b) {
      if (dcolor[(size_t)a] != dcolor[(size_t)b]) return dcolor[(size_t)a] < dcolor[(size_t)b];
      const int64_t pa = npos[(size_t)dnode_[(size_t)a]], pb = npos[(size_t)dnode_[(size_t)b]];
      if (pa != pb) return pa < pb;
      return pos[(size_t)a] < pos[(size_t)b];
    });
  } else if (nblk > 1) {
    std::stable_sort(order.begin(), order.end(), [&](int64_t a, int64_t b) { return dblk[(size_t)a] < dblk[(size_t)b]; });
  }
  std::vector<int32_t> newidx((size_t)n, -1), olddof((size_t)n);
  for (int64_t r = 0; r < n; ++r) {
    newidx[(size_t)order[(size_t)r]] = (int32_t)r;
    olddof[(size_t)r] = (int32_t)order[(size_t)r];
  }
  // the system matrix's pattern in the new numbering, then its ILU(fill) pattern
  std::vector<int64_t> arow((size_t)n + 1, 0);
  std::vector<int32_t> acl;
  std::vector<char> aclown;  // entry probed on this rank (pent / prow); else filled by the neighbours only
  acl.reserve(acol.size());
  {
    std::vector<std::pair<int32_t, char>> rowbuf;
    for (int64_t r = 0; r < n; ++r) {
      const int64_t i = olddof[(size_t)r];
      rowbuf.clear();
      for (int64_t t = aoff[(size_t)i]; t < aoff[(size_t)i + 1]; ++t)
        if (dblk[(size_t)acol[(size_t)t]] == dblk[(size_t)i]) rowbuf.push_back({newidx[(size_t)acol[(size_t)t]], aown[(size_t)t]});
      std::sort(rowbuf.begin(), rowbuf.end());
      for (const auto &e : rowbuf) {
        acl.push_back(e.first);
        aclown.push_back(e.second);
      }
      arow[(size_t)r + 1] = (int64_t)acl.size();
    }
  }
  std::vector<int64_t> rowp;
  std::vector<int32_t> col;
  if (gls::iluk_pattern<int64_t>(n, arow.data(), acl.data(), fill, rowp, col) != GLS_OK)
    return set_err(GLS_EINVAL, "gls_ilu_attach: ILU(%d) pattern", fill);
  std::vector<int64_t> didx((size_t)n, -1);
  for (int64_t r = 0; r < n; ++r) {
    const auto b = col.begin() + rowp[(size_t)r], e = col.begin() + rowp[(size_t)r + 1];
    const auto it = std::lower_bound(b, e, (int32_t)r);
    if (it == e || *it != r) return set_err(GLS_EINVAL, "gls_ilu_attach: row %lld has no diagonal", (long long)r);
    didx[(size_t)r] = (int64_t)(it - col.begin());
  }
  // multicolor solves: node groups (consecutive rows of one node), per color their range, per row
  // the split of its entries into other colors / own node; valid while no entry couples two nodes of
  // one color (fill 0; fill-in can create such entries: then rocSPARSE csrsv solves)
  I.mc_solve = false;
  I.mc_factor = false;
  I.mc_compact = false;
  std::vector<int64_t> mc_moff_h;  // position map offsets (empty: no map)
  if (I.ordering == GLS_ILU_ORDER_MULTICOLOR) {
    const int ncl = I.n_order_colors;
    std::vector<int32_t> cstart((size_t)ncl + 2, (int32_t)n), grow, cg((size_t)ncl + 1, 0);
    std::vector<int64_t> lsp((size_t)n), usp((size_t)n);
    for (int64_t r = n - 1; r >= 0; --r) cstart[(size_t)dcolor[(size_t)olddof[(size_t)r]]] = (int32_t)r;
    for (int c = ncl - 1; c >= 0; --c) cstart[(size_t)c] = std::min(cstart[(size_t)c], cstart[(size_t)c + 1]);
    bool ok = true;
    for (int64_t r = 0; r < n && ok; ++r) {
      const int64_t x = dnode_[(size_t)olddof[(size_t)r]];
      if (r == 0 || x != dnode_[(size_t)olddof[(size_t)r - 1]]) grow.push_back((int32_t)r);
      if (r + 1 - grow.back() > gls::kMaxGroupRows) ok = false;
      const int cr = dcolor[(size_t)olddof[(size_t)r]];
      int64_t e = rowp[(size_t)r];
      while (e < rowp[(size_t)r + 1] && col[(size_t)e] < cstart[(size_t)cr]) ++e;
      lsp[(size_t)r] = e;
      while (e < rowp[(size_t)r + 1] && col[(size_t)e] < cstart[(size_t)cr + 1]) {
        if (dnode_[(size_t)olddof[(size_t)col[(size_t)e]]] != x) ok = false;  // same color, other node
        ++e;
      }
      usp[(size_t)r] = e;
    }
    if (ok) {
      grow.push_back((int32_t)n);
      for (int c = 0, g = 0; c <= ncl; ++c) {
        while (g + 1 < (int)grow.size() && grow[(size_t)g] < cstart[(size_t)c]) ++g;
        cg[(size_t)c] = c == ncl ? (int)grow.size() - 1 : g;
      }
      GLS_TRY(I.mc_grow.upload(grow.data(), grow.size()));
      GLS_TRY(I.mc_lsp.upload(lsp.data(), lsp.size()));
      GLS_TRY(I.mc_usp.upload(usp.data(), usp.size()));
      {
        const size_t ng = grow.size() - 1;
        std::vector<int64_t> desc(ng * gls::kGroupDesc, 0);
        for (size_t g = 0; g < ng; ++g) {
          int64_t *d = &desc[g * gls::kGroupDesc];
          const int32_t r0 = grow[g], nr = grow[g + 1] - r0;
          d[0] = r0;
          d[1] = nr;
          d[2] = rowp[(size_t)r0];
          d[3] = rowp[(size_t)(r0 + nr)];
          for (int t = 1; t < 4; ++t) d[3 + t] = t < nr ? rowp[(size_t)(r0 + t)] : INT64_MAX;
          for (int t = 0; t < nr; ++t) {
            d[8 + t] = lsp[(size_t)(r0 + t)];
            d[12 + t] = usp[(size_t)(r0 + t)];
            d[16 + t] = didx[(size_t)(r0 + t)];
            d[20 + t] = rowp[(size_t)(r0 + t) + 1];
          }
        }
        GLS_TRY(I.mc_desc.upload(desc.data(), desc.size()));
      }
      I.mc_cg = cg;
      I.mc_solve = true;
      int64_t maxrow = 0;
      for (int64_t r = 0; r < n; ++r) maxrow = std::max(maxrow, rowp[(size_t)r + 1] - rowp[(size_t)r]);
      I.mc_factor = maxrow <= gls::kIluMaxRow && rowp.back() < (int64_t(1) << 35) && !std::getenv("GLS_ILU_ROCSPARSE_FACTOR");
      I.mc_compact = maxrow <= gls::kIluCompactRow;
      if (I.mc_factor) GLS_TRY(I.rdiag.alloc((size_t)n));
      if (I.mc_factor) {  // the position map (uint16 per entry), when it fits a quarter of free memory
        mc_moff_h.assign((size_t)n + 1, 0);
        for (int64_t r = 0; r < n; ++r) {
          int64_t m = 0;
          for (int64_t e = rowp[(size_t)r]; e < lsp[(size_t)r]; ++e) {
            const int32_t k = col[(size_t)e];
            m += (rowp[(size_t)k + 1] - didx[(size_t)k] - 1 + 3) & ~3;  // segments padded to quads
          }
          mc_moff_h[(size_t)r + 1] = mc_moff_h[(size_t)r] + m;
        }
        size_t fr = 0, tot = 0;
        const char *me = std::getenv("GLS_ILU_FACTOR_MAP");
        if ((me && std::atoi(me) == 0) || hipMemGetInfo(&fr, &tot) != hipSuccess ||
            (double)mc_moff_h[(size_t)n] * 2.0 > 0.25 * (double)fr)
          mc_moff_h.clear();
      }
      // per color and direction: one wavefront per node group while a group's other-color entries
      // fit a few passes of 64 lanes, else four (long rows: the late colors' L parts, the early
      // colors' U parts)
      I.mc_wl.assign((size_t)ncl, 1);
      I.mc_wu.assign((size_t)ncl, 1);
      for (int c = 0; c < ncl; ++c) {
        const int32_t ra = grow[(size_t)cg[(size_t)c]], rb = grow[(size_t)cg[(size_t)c + 1]];
        const int ng = cg[(size_t)c + 1] - cg[(size_t)c];
        int64_t nlo = 0, nup = 0;
        for (int32_t r = ra; r < rb; ++r) {
          nlo += lsp[(size_t)r] - rowp[(size_t)r];
          nup += rowp[(size_t)r + 1] - usp[(size_t)r];
        }
        I.mc_wl[(size_t)c] = (uint8_t)(ng && nlo > 256 * (int64_t)ng ? 4 : 1);
        I.mc_wu[(size_t)c] = (uint8_t)(ng && nup > 256 * (int64_t)ng ? 4 : 1);
      }
    }
  }
  // probes: one per (color, slot); every entry of the system matrix is read from the probe of its
  // column DoF (entry position in the ILU pattern, row's original DoF)
  const int nprobe = ncol * (dim + 1);
  std::vector<int> dslot((size_t)n, 0);
  std::vector<int64_t> dnode((size_t)n, 0);
  for (int64_t x = 0; x < nu; ++x) {
    int64_t d[4];
    int sl[4];
    const int m = node_dofs(x, d, sl);
    for (int j = 0; j < m; ++j) { dslot[(size_t)d[j]] = sl[j]; dnode[(size_t)d[j]] = x; }
  }
  auto probe_of = [&](int64_t d) { return color[(size_t)dnode[(size_t)d]] * (dim + 1) + dslot[(size_t)d]; };
  std::vector<int64_t> pdoff((size_t)nprobe + 1, 0), peoff((size_t)nprobe + 1, 0);
  for (int64_t d = 0; d < n; ++d) ++pdoff[(size_t)probe_of(d) + 1];
  for (int64_t r = 0; r < n; ++r)
    for (int64_t t = arow[(size_t)r]; t < arow[(size_t)r + 1]; ++t)
      if (aclown[(size_t)t]) ++peoff[(size_t)probe_of(olddof[(size_t)acl[(size_t)t]]) + 1];
  for (int p = 0; p < nprobe; ++p) {
    pdoff[(size_t)p + 1] += pdoff[(size_t)p];
    peoff[(size_t)p + 1] += peoff[(size_t)p];
  }
  std::vector<int32_t> pdofs((size_t)pdoff[(size_t)nprobe]), prow((size_t)peoff[(size_t)nprobe]);
  std::vector<int64_t> pent(prow.size());
  {
    std::vector<int64_t> f1(pdoff.begin(), pdoff.end() - 1), f2(peoff.begin(), peoff.end() - 1);
    // (complete rows: the unconstrained ghost DoFs are probed too)
    for (int64_t d = 0; d < n; ++d)
      pdofs[(size_t)f1[(size_t)probe_of(d)]++] = ghost(d) && !(cmpl && !fcons[(size_t)d]) ? -1 : (int32_t)d;
    for (int64_t r = 0; r < n; ++r) {
      int64_t pos = rowp[(size_t)r];
      for (int64_t t = arow[(size_t)r]; t < arow[(size_t)r + 1]; ++t) {
        while (col[(size_t)pos] < acl[(size_t)t]) ++pos;  // both rows sorted; A's pattern is a subset
        if (!aclown[(size_t)t]) continue;
        const int64_t k = f2[(size_t)probe_of(olddof[(size_t)acl[(size_t)t]])]++;
        pent[(size_t)k] = pos;
        prow[(size_t)k] = olddof[(size_t)r];  // the probe result is indexed by the original DoF
      }
    }
  }
  I.release();
  GLS_TRY(I.rowp.upload(rowp.data(), rowp.size()));
  GLS_TRY(I.col.upload(col.data(), col.size()));
  GLS_TRY(I.didx.upload(didx.data(), didx.size()));
  GLS_TRY(I.perm.upload(newidx.data(), newidx.size()));
  I.mc_map.release();
  I.mc_moff.release();
  if (!mc_moff_h.empty()) {
    GLS_TRY(I.mc_moff.upload(mc_moff_h.data(), mc_moff_h.size()));
    GLS_TRY(I.mc_map.alloc((size_t)mc_moff_h.back() + 256));  // + the clamped index of empty stages
    HIP_TRY(gls::ilu_mc_factor_map(n, I.rowp.p, I.col.p, I.mc_lsp.p, I.didx.p, I.mc_moff.p, I.mc_map.p, c->stream));
  }
  // ghost DoFs are not probed (identity rows): drop them from the unit lists, remember their diagonals
  {
    std::vector<int32_t> pd2;
    std::vector<int64_t> pdoff2((size_t)nprobe + 1, 0);
    for (int p = 0; p < nprobe; ++p) {
      for (int64_t t = pdoff[(size_t)p]; t < pdoff[(size_t)p + 1]; ++t)
        if (pdofs[(size_t)t] >= 0) pd2.push_back(pdofs[(size_t)t]);
      pdoff2[(size_t)p + 1] = (int64_t)pd2.size();
    }
    pdofs.swap(pd2);
    pdoff.swap(pdoff2);
    std::vector<int64_t> gd;
    for (int64_t r = 0; r < n; ++r)
      if (ghost(olddof[(size_t)r])) gd.push_back(didx[(size_t)r]);
    GLS_TRY(I.ghost_diag.upload(gd.data(), gd.size()));
  }
  // the neighbours' entries: per round, each CSR entry's send_buf slots in (round, neighbour, slot) order
  {
    std::vector<std::pair<int64_t, int64_t>> key;  // (round * nnz + entry, record) sorted stably
    const int64_t nnz = (int64_t)col.size();
    for (size_t q = 0; q < remote.size(); ++q) {
      const auto &e = remote[q];
      if (dblk[(size_t)e.i] != dblk[(size_t)e.j]) continue;
      const int32_t r = newidx[(size_t)e.i], cj = newidx[(size_t)e.j];
      const auto b = col.begin() + rowp[(size_t)r], en = col.begin() + rowp[(size_t)r + 1];
      const auto it = std::lower_bound(b, en, cj);
      if (it == en || *it != cj) return set_err(GLS_EINVAL, "gls_ilu_attach: a neighbour's entry is not in the pattern");
      key.push_back({(int64_t)e.round * nnz + (int64_t)(it - col.begin()), (int64_t)q});
    }
    std::stable_sort(key.begin(), key.end(), [](const std::pair<int64_t, int64_t> &a, const std::pair<int64_t, int64_t> &b) {
      return a.first < b.first;
    });
    std::vector<int64_t> ru;
    std::vector<int32_t> ruoff{0}, rslot;
    std::vector<int64_t> rr((size_t)std::max(n_rounds, 0) + 1, 0);
    for (size_t t = 0; t < key.size(); ++t) {
      if (t == 0 || key[t].first != key[t - 1].first) {
        if (t) ruoff.push_back((int32_t)rslot.size());
        ru.push_back(key[t].first % nnz);
        ++rr[(size_t)(key[t].first / nnz) + 1];
      }
      rslot.push_back(remote[(size_t)key[t].second].slot);
    }
    if (!key.empty()) ruoff.push_back((int32_t)rslot.size());
    for (int p = 0; p < n_rounds; ++p) rr[(size_t)p + 1] += rr[(size_t)p];
    ru.push_back(0);  // (padding: no zero-sized device buffers)
    rslot.push_back(0);
    GLS_TRY(I.ru.upload(ru.data(), ru.size()));
    GLS_TRY(I.ruoff.upload(ruoff.data(), ruoff.size()));
    GLS_TRY(I.rslot.upload(rslot.data(), rslot.size()));
    I.rr = rr;
    I.complete = cmpl;
    I.n_rounds = n_rounds;
  }
  GLS_TRY(I.pdofs.upload(pdofs.data(), pdofs.size()));
  GLS_TRY(I.pent.upload(pent.data(), pent.size()));
  GLS_TRY(I.prow.upload(prow.data(), prow.size()));
  {  // probe of every unit DoF and every extracted entry (batched probing)
    std::vector<int32_t> pdp(std::max<size_t>(pdofs.size(), 1)), pep(std::max<size_t>(pent.size(), 1));
    for (int p = 0; p < nprobe; ++p) {
      for (int64_t t = pdoff[(size_t)p]; t < pdoff[(size_t)p + 1]; ++t) pdp[(size_t)t] = p;
      for (int64_t t = peoff[(size_t)p]; t < peoff[(size_t)p + 1]; ++t) pep[(size_t)t] = p;
    }
    GLS_TRY(I.pdpid.upload(pdp.data(), pdp.size()));
    GLS_TRY(I.pepid.upload(pep.data(), pep.size()));
  }
  GLS_TRY(I.val.alloc(col.size() + 256));  // + the factorization's whole-quad loads past a row's end
  HIP_TRY(hipMemset(I.val.p, 0, col.size() * sizeof(double)));
  GLS_TRY(I.vbuf.alloc((size_t)n));
  GLS_TRY(I.ybuf.alloc((size_t)n));
  GLS_TRY(I.tbuf.alloc((size_t)n));
  I.pdoff = pdoff;
  I.woff.clear();  // new probes: their activity is recorded again
  I.peoff = peoff;
  I.n_probes = nprobe;
  I.nnz = (int64_t)col.size();
  I.nnz_a = (int64_t)acl.size();
  I.fill = fill;
  I.n_blocks = nblk;
  I.athresh = athresh;
  I.rthresh = rthresh;
  // the multicolor kernels factor and solve: no rocSPARSE state (its csrilu0 / csrsv analyses were a setup cost of
  // ~0.9 s at 1.7 M DoFs, a radix sort each, for solves that never ran); past 2^31 entries they are the only route
  // (rocSPARSE takes 32-bit CSR)
  if (I.nnz >= INT32_MAX || (I.mc_factor && I.mc_solve)) {
    if (!I.mc_factor || !I.mc_solve)
      return set_err(GLS_EINVAL, "gls_ilu_attach: %lld entries (> 2^31): the multicolor order with fill 0 is needed",
                     (long long)I.nnz);
    I.boost_tol = athresh > 0 ? athresh : 1e-300;  // as below, read by the multicolor factorization
    I.boost_val = athresh > 0 ? athresh : 1e-12;
    I.valid = false;
    I.on = true;
    return GLS_OK;
  }
  {
    std::vector<int32_t> rp32(rowp.begin(), rowp.end());
    GLS_TRY(I.rowp32.upload(rp32.data(), rp32.size()));
  }
  RS_TRY(rocsparse_create_handle(&I.h));
  RS_TRY(rocsparse_set_stream(I.h, c->stream));
  RS_TRY(rocsparse_create_mat_descr(&I.dA));
  RS_TRY(rocsparse_create_mat_descr(&I.dL));
  RS_TRY(rocsparse_set_mat_fill_mode(I.dL, rocsparse_fill_mode_lower));
  RS_TRY(rocsparse_set_mat_diag_type(I.dL, rocsparse_diag_type_unit));
  RS_TRY(rocsparse_create_mat_descr(&I.dU));
  RS_TRY(rocsparse_set_mat_fill_mode(I.dU, rocsparse_fill_mode_upper));
  RS_TRY(rocsparse_set_mat_diag_type(I.dU, rocsparse_diag_type_non_unit));
  RS_TRY(rocsparse_create_mat_info(&I.info));
  const rocsparse_int m = (rocsparse_int)n, nnz = (rocsparse_int)I.nnz;
  size_t b0 = 0, b1 = 0, b2 = 0;
  RS_TRY(rocsparse_dcsrilu0_buffer_size(I.h, m, nnz, I.dA, I.val.p, I.rowp32.p, I.col.p, I.info, &b0));
  RS_TRY(rocsparse_dcsrsv_buffer_size(I.h, rocsparse_operation_none, m, nnz, I.dL, I.val.p, I.rowp32.p, I.col.p, I.info, &b1));
  RS_TRY(rocsparse_dcsrsv_buffer_size(I.h, rocsparse_operation_none, m, nnz, I.dU, I.val.p, I.rowp32.p, I.col.p, I.info, &b2));
  GLS_TRY(I.work.alloc(std::max(std::max(b0, b1), std::max(b2, (size_t)16))));
  RS_TRY(rocsparse_dcsrilu0_analysis(I.h, m, nnz, I.dA, I.val.p, I.rowp32.p, I.col.p, I.info, rocsparse_analysis_policy_reuse,
                                     rocsparse_solve_policy_auto, I.work.p));
  RS_TRY(rocsparse_dcsrsv_analysis(I.h, rocsparse_operation_none, m, nnz, I.dL, I.val.p, I.rowp32.p, I.col.p, I.info,
                                   rocsparse_analysis_policy_reuse, rocsparse_solve_policy_auto, I.work.p));
  RS_TRY(rocsparse_dcsrsv_analysis(I.h, rocsparse_operation_none, m, nnz, I.dU, I.val.p, I.rowp32.p, I.col.p, I.info,
                                   rocsparse_analysis_policy_reuse, rocsparse_solve_policy_auto, I.work.p));
  // pivots that end below athresh in magnitude are boosted to athresh (enclosed-flow pressure mode)
  // (rocsparse stores the two pointers and reads them at every csrilu0: they must outlive this call;
  // stack locals here gave the first factorization whatever the stack later held)
  I.boost_tol = athresh > 0 ? athresh : 1e-300;
  I.boost_val = athresh > 0 ? athresh : 1e-12;
  RS_TRY(rocsparse_dcsrilu0_numeric_boost(I.h, I.info, 1, &I.boost_tol, &I.boost_val));
  I.on = true;
  I.valid = false;
  if (std::getenv("GLS_ILU_VERBOSE"))
    std::printf("ilu attach: n %lld fill %d blocks %d ordering %s (%d colors%s) nnz(A) %lld nnz(ILU) %lld probe colors "
                "%d probes %d\n", (long long)n, fill, nblk, I.ordering == GLS_ILU_ORDER_CM ? "cuthill-mckee" : "multicolor",
                I.n_order_colors, I.mc_solve ? ", color solves" : "", (long long)I.nnz_a, (long long)I.nnz, ncol, nprobe);
  return GLS_OK;
}
extern "C" int gls_ilu_set_options(gls_ctx *c, int ordering, int64_t block_dofs) {
  GLS_TRY(check_ctx(c));
  if (block_dofs < 0) return set_err(GLS_EINVAL, "gls_ilu_set_options: negative block size");
  if (ordering != GLS_ILU_ORDER_CM && ordering != GLS_ILU_ORDER_MULTICOLOR)
    return set_err(GLS_EINVAL, "gls_ilu_set_options: ordering %d", ordering);
  c->ilu.block_dofs = block_dofs;
  c->ilu.ordering = ordering;
  return GLS_OK;
}
extern "C" int gls_ilu_detach(gls_ctx *c) {
  GLS_TRY(check_ctx(c));
  c->ilu.on = false;
  c->ilu.probe_only = false;
  c->ilu.release();
  return GLS_OK;
}
// the probed (unfactored, unperturbed) operator matrix, for tests: host CSR arrays of gls_ilu_info's nnz
extern "C" int gls_ilu_matrix(gls_ctx *c, int32_t *rowp, int32_t *col, double *val) {
  GLS_TRY(check_ctx(c));
  auto &I = c->ilu;
  if (!I.on) return set_err(GLS_EINVAL, "no ILU attached");
  GLS_TRY(ilu_probe(c));
  HIP_TRY(hipStreamSynchronize(c->stream));
  // renumbered CSR on the device; returned in the context's DoF numbering
  const int64_t n = c->n_dofs;
  if (I.nnz >= INT32_MAX) return set_err(GLS_EINVAL, "gls_ilu_matrix: %lld entries do not fit its 32-bit CSR", (long long)I.nnz);
  std::vector<int64_t> rp((size_t)n + 1);
  std::vector<int32_t> cl((size_t)I.nnz), pm((size_t)n);
  std::vector<double> vl((size_t)I.nnz);
  HIP_TRY(hipMemcpy(rp.data(), I.rowp.p, sizeof(int64_t) * rp.size(), hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(cl.data(), I.col.p, sizeof(int32_t) * cl.size(), hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(vl.data(), I.val.p, sizeof(double) * vl.size(), hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(pm.data(), I.perm.p, sizeof(int32_t) * pm.size(), hipMemcpyDeviceToHost));
  std::vector<int32_t> old((size_t)n);
  for (int64_t i = 0; i < n; ++i) old[(size_t)pm[(size_t)i]] = (int32_t)i;
  std::vector<std::vector<std::pair<int32_t, double>>> rows((size_t)n);
  for (int64_t r = 0; r < n; ++r)
    for (int64_t e = rp[(size_t)r]; e < rp[(size_t)r + 1]; ++e) rows[(size_t)old[(size_t)r]].push_back({old[(size_t)cl[(size_t)e]], vl[(size_t)e]});
  int64_t k = 0;
  if (rowp) rowp[0] = 0;
  for (int64_t i = 0; i < n; ++i) {
    std::sort(rows[(size_t)i].begin(), rows[(size_t)i].end());
    for (auto &pr : rows[(size_t)i]) {
      if (col) col[k] = pr.first;
      if (val) val[k] = pr.second;
      ++k;
    }
    if (rowp) rowp[i + 1] = (int32_t)k;
  }
  I.valid = false;  // the values now hold the unfactored matrix
  return GLS_OK;
}
// the factored ILU(fill) (after the diagonal perturbation) in the factorization's numbering, for
// tests: perm[dof] = its row; rowp / col / val of gls_ilu_info's nnz entries (unit-diagonal L below
// the diagonal, U on and above it, as rocSPARSE csrilu0 stores them)
extern "C" int gls_ilu_factors(gls_ctx *c, int32_t *perm, int32_t *rowp, int32_t *col, double *val) {
  GLS_TRY(check_ctx(c));
  auto &I = c->ilu;
  if (!I.on) return set_err(GLS_EINVAL, "no ILU attached");
  GLS_TRY(ensure_diag(c));
  GLS_TRY(ensure_ilu(c));
  HIP_TRY(hipStreamSynchronize(c->stream));
  if (perm) HIP_TRY(hipMemcpy(perm, I.perm.p, sizeof(int32_t) * (size_t)c->n_dofs, hipMemcpyDeviceToHost));
  if (I.nnz >= INT32_MAX) return set_err(GLS_EINVAL, "gls_ilu_factors: %lld entries do not fit its 32-bit CSR", (long long)I.nnz);
  if (rowp) {
    std::vector<int64_t> rp((size_t)c->n_dofs + 1);
    HIP_TRY(hipMemcpy(rp.data(), I.rowp.p, sizeof(int64_t) * rp.size(), hipMemcpyDeviceToHost));
    for (size_t i = 0; i < rp.size(); ++i) rowp[i] = (int32_t)rp[i];
  }
  if (col) HIP_TRY(hipMemcpy(col, I.col.p, sizeof(int32_t) * (size_t)I.nnz, hipMemcpyDeviceToHost));
  if (val) HIP_TRY(hipMemcpy(val, I.val.p, sizeof(double) * (size_t)I.nnz, hipMemcpyDeviceToHost));
  return GLS_OK;
}
extern "C" int gls_ilu_info(const gls_ctx *c, int64_t *nnz, int *n_probes) {
  if (!c) return set_err(GLS_EINVAL, "null context");
  if (nnz) *nnz = c->ilu.nnz;
  if (n_probes) *n_probes = c->ilu.n_probes;
  return c->ilu.on ? GLS_OK : set_err(GLS_EINVAL, "no ILU attached");
}


// ---------------------------------------------------------------------------------------------
// In-library RCCL over xGMI (the reference's Trilinos ghost import / compress(add) and
// MPI_Allreduce, gls_navier_stokes.cc:186-202, 774-776): one communicator per process, shared by
// the contexts of every multigrid level; exchanges and reductions are enqueued on the context
// stream (RCCL orders them with the pack / unpack kernels), so no exchange blocks the host.
// ---------------------------------------------------------------------------------------------
struct gls_rccl {
  ncclComm_t comm = nullptr;
  int rank = 0, world = 1;
};
namespace {
int rccl_exchange(void *user, int phase) { return rccl_exchange_on(static_cast<gls_ctx *>(user), phase, static_cast<gls_ctx *>(user)->stream); }
int rccl_allreduce(void *user, double *buf, int n) {
  gls_ctx *c = static_cast<gls_ctx *>(user);
  return ncclAllReduce(buf, buf, (size_t)n, ncclDouble, ncclSum, c->dist.comm, c->stream) == ncclSuccess ? 0 : -1;
}
int rccl_exchange_on(gls_ctx *c, int phase, hipStream_t stream) {
  auto &D = c->dist;
  // phase 0 (import): send send_buf segments (owned nodes others ghost), receive into recv_buf;
  // phase 1 (export-add): the reverse (ghost partial sums back to their owners)
  double *sb = phase == 0 ? D.send_buf : D.recv_buf, *rb = phase == 0 ? D.recv_buf : D.send_buf;
  const std::vector<int64_t> &so = phase == 0 ? D.soff : D.roff, &ro = phase == 0 ? D.roff : D.soff;
  if (ncclGroupStart() != ncclSuccess) return -1;
  for (size_t i = 0; i < D.nbrs.size(); ++i) {
    const int w = D.width;
    const size_t ns = (size_t)(w * (so[i + 1] - so[i])), nr = (size_t)(w * (ro[i + 1] - ro[i]));
    if (ns && ncclSend(sb + w * so[i], ns, ncclDouble, D.nbrs[i], D.comm, stream) != ncclSuccess) return -1;
    if (nr && ncclRecv(rb + w * ro[i], nr, ncclDouble, D.nbrs[i], D.comm, stream) != ncclSuccess) return -1;
  }
  return ncclGroupEnd() == ncclSuccess ? 0 : -1;
}
}  // namespace

extern "C" int gls_rccl_unique_id(unsigned char *id_out) {
  if (!id_out) return set_err(GLS_EINVAL, "gls_rccl_unique_id: null output");
  ncclUniqueId id;
  const ncclResult_t r = ncclGetUniqueId(&id);
  if (r != ncclSuccess) return set_err(GLS_ECOMM, "ncclGetUniqueId: %s", ncclGetErrorString(r));
  static_assert(sizeof(id) == GLS_RCCL_ID_BYTES, "ncclUniqueId size");
  std::memcpy(id_out, &id, sizeof(id));
  return GLS_OK;
}
extern "C" int gls_rccl_create(const unsigned char *id_in, int rank, int world, gls_rccl **out) {
  if (!id_in || !out || world < 1 || rank < 0 || rank >= world) return set_err(GLS_EINVAL, "gls_rccl_create: bad arguments");
  ncclUniqueId id;
  std::memcpy(&id, id_in, sizeof(id));
  auto r = std::make_unique<gls_rccl>();
  const ncclResult_t e = ncclCommInitRank(&r->comm, world, id, rank);
  if (e != ncclSuccess) return set_err(GLS_ECOMM, "ncclCommInitRank(%d of %d): %s", rank, world, ncclGetErrorString(e));
  r->rank = rank;
  r->world = world;
  *out = r.release();
  return GLS_OK;
}
// the communicator's own view (ncclCommUserRank / ncclCommCount): what bench.py reports as rccl_ranks
extern "C" int gls_rccl_info(const gls_rccl *r, int *rank, int *world) {
  if (!r || !r->comm) return set_err(GLS_EINVAL, "gls_rccl_info: no communicator");
  int rk = -1, n = 0;
  if (ncclCommUserRank(r->comm, &rk) != ncclSuccess || ncclCommCount(r->comm, &n) != ncclSuccess)
    return set_err(GLS_ECOMM, "gls_rccl_info: ncclCommUserRank / ncclCommCount failed");
  if (rank) *rank = rk;
  if (world) *world = n;
  return GLS_OK;
}
extern "C" int gls_rccl_destroy(gls_rccl *r) {
  if (!r) return GLS_OK;
  if (r->comm) (void)ncclCommDestroy(r->comm);
  delete r;
  return GLS_OK;
}
extern "C" int gls_dist_attach_rccl(gls_ctx *c, gls_rccl *r, int64_t n_owned_nodes, int n_nbrs, const int *nbr_ranks,
                                    const int64_t *send_offsets, const int32_t *send_nodes, const int64_t *recv_offsets,
                                    const int32_t *recv_nodes) {
  GLS_TRY(check_ctx(c));
  if (!r || !r->comm || n_nbrs < 0 || (n_nbrs > 0 && (!nbr_ranks || !send_offsets || !recv_offsets)))
    return set_err(GLS_EINVAL, "gls_dist_attach_rccl: bad arguments");
  auto &D = c->dist;
  const int64_t ns = n_nbrs ? send_offsets[n_nbrs] : 0, nr = n_nbrs ? recv_offsets[n_nbrs] : 0;
  for (int i = 0; i < n_nbrs; ++i)
    if (nbr_ranks[i] < 0 || nbr_ranks[i] >= r->world || nbr_ranks[i] == r->rank)
      return set_err(GLS_EINVAL, "gls_dist_attach_rccl: neighbour rank %d", nbr_ranks[i]);
  GLS_TRY(D.own_send.alloc((size_t)std::max<int64_t>(4 * ns, 1)));
  GLS_TRY(D.own_recv.alloc((size_t)std::max<int64_t>(4 * nr, 1)));
  GLS_TRY(D.own_red.alloc(256));
  GLS_TRY(gls_dist_attach(c, n_owned_nodes, n_nbrs, send_offsets, send_nodes, recv_offsets, recv_nodes, D.own_send.p,
                          D.own_recv.p, D.own_red.p, rccl_exchange, rccl_allreduce, c));
  D.comm = r->comm;
  if (!D.xstream) {
    HIP_TRY(hipStreamCreateWithFlags(&D.xstream, hipStreamNonBlocking));
    HIP_TRY(hipEventCreateWithFlags(&D.ev_ready, hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&D.ev_done, hipEventDisableTiming));
  }
  D.nbrs.assign(nbr_ranks, nbr_ranks + n_nbrs);
  D.soff.assign(send_offsets, send_offsets + n_nbrs + 1);
  D.roff.assign(recv_offsets, recv_offsets + n_nbrs + 1);
  if (n_nbrs == 0) {
    D.soff.assign(1, 0);
    D.roff.assign(1, 0);
  }
  return GLS_OK;
}

extern "C" int gls_dist_attach_dofs_rccl(gls_ctx *c, gls_rccl *r, int64_t n_owned_vnodes, int64_t n_owned_pnodes,
                                         int n_nbrs, const int *nbr_ranks, const int64_t *send_offsets,
                                         const int32_t *send_dofs, const int64_t *recv_offsets, const int32_t *recv_dofs) {
  GLS_TRY(check_ctx(c));
  if (!r || !r->comm || n_nbrs < 0 || (n_nbrs > 0 && (!nbr_ranks || !send_offsets || !recv_offsets)))
    return set_err(GLS_EINVAL, "gls_dist_attach_dofs_rccl: bad arguments");
  auto &D = c->dist;
  const int64_t ns = n_nbrs ? send_offsets[n_nbrs] : 0, nr = n_nbrs ? recv_offsets[n_nbrs] : 0;
  for (int i = 0; i < n_nbrs; ++i)
    if (nbr_ranks[i] < 0 || nbr_ranks[i] >= r->world || nbr_ranks[i] == r->rank)
      return set_err(GLS_EINVAL, "gls_dist_attach_dofs_rccl: neighbour rank %d", nbr_ranks[i]);
  GLS_TRY(D.own_send.alloc((size_t)std::max<int64_t>(ns, 1)));
  GLS_TRY(D.own_recv.alloc((size_t)std::max<int64_t>(nr, 1)));
  GLS_TRY(D.own_red.alloc(256));
  GLS_TRY(gls_dist_attach_dofs(c, n_owned_vnodes, n_owned_pnodes, n_nbrs, send_offsets, send_dofs, recv_offsets, recv_dofs,
                               D.own_send.p, D.own_recv.p, D.own_red.p, rccl_exchange, rccl_allreduce, c));
  D.comm = r->comm;
  D.nbrs.assign(nbr_ranks, nbr_ranks + n_nbrs);
  D.soff.assign(send_offsets, send_offsets + n_nbrs + 1);
  D.roff.assign(recv_offsets, recv_offsets + n_nbrs + 1);
  if (n_nbrs == 0) {
    D.soff.assign(1, 0);
    D.roff.assign(1, 0);
  }
  return GLS_OK;
}
