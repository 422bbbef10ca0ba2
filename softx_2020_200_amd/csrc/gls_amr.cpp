// gls_amr.cpp — locally refined hyper_cube with hanging-node constraints (host C++17).
//
// The reference builds its meshes on a p4est forest and refines them adaptively
// (navier_stokes_base.cc:592-780); every refinement level difference leaves hanging nodes, which
// setup_dofs constrains with DoFTools::make_hanging_node_constraints (gls_navier_stokes.cc:84, 143)
// before the boundary conditions (interpolate_boundary_values skips DoFs already constrained).
// This builder produces the one-level case: hyper_cube(lo, hi) refined to n cells per direction,
// then the flagged cells refined once more (2^dim children, lexicographic). A node of a refined
// cell that lies on the boundary of an unrefined neighbour without being one of its nodes is
// hanging: its value is the neighbour's Qk interpolant there, i.e. the neighbour's tensor-product
// Lagrange basis (support points a/k: Gauss-Lobatto = equidistant for k <= 2) evaluated at the
// node, which is what make_hanging_node_constraints yields for FE_Q. Nodes live on the fine
// lattice of spacing h_fine / k; ids follow lexicographic lattice order (x fastest) over the used
// points. Velocity and pressure spaces are built separately (kp may be < k).
#include <algorithm>
#include <limits>
#include <cmath>
#include <functional>
#include <cstdint>
#include <cstring>
#include <memory>
#include <vector>

#include "../../include/gls_native.h"

int gls_io_set_error(int code, const char *fmt, ...);  // gls_api.cpp

namespace {

struct RefinedMeshImpl {
  gls_refined_mesh pub{};
  std::vector<int32_t> cell_vnodes, cell_pnodes, cell_level;
  std::vector<double> cell_x0, cell_h, vnode_x, pnode_x;
  std::vector<int64_t> vh_node, vh_off, vh_master, ph_node, ph_off, ph_master;
  std::vector<double> vh_w, ph_w;
};

struct Cell {
  int f0[3];  // origin in fine-cell units
  int s;      // extent in fine cells: 2 (unrefined) or 1 (child of a refined cell)
};

double lagrange(int k, int a, double xi) {  // degree-k Lagrange basis a on the nodes b/k, at xi
  double v = 1.0;
  for (int b = 0; b <= k; ++b)
    if (b != a) v *= (xi - (double)b / k) / ((double)(a - b) / k);
  return v;
}

// nodes, cell -> node table and hanging lines of the FE_Q(kk) space on the refined mesh
int build_space(int dim, int n, int kk, double lo, double hf, const std::vector<Cell> &cells,
                std::vector<int32_t> &cell_nodes, std::vector<double> &node_x, std::vector<int64_t> &hnode,
                std::vector<int64_t> &hoff, std::vector<double> &hw, std::vector<int64_t> &hmaster) {
  const int64_t np1 = (int64_t)kk * 2 * n + 1;  // lattice points per direction
  int64_t npts = 1;
  for (int d = 0; d < dim; ++d) npts *= np1;
  if (npts > ((int64_t)1 << 31)) return gls_io_set_error(GLS_EINVAL, "refined mesh lattice too large");
  auto lat = [&](const int64_t *p) {
    int64_t id = 0, st = 1;
    for (int d = 0; d < dim; ++d) {
      id += p[d] * st;
      st *= np1;
    }
    return id;
  };
  const int K1 = kk + 1;
  int npc = 1;
  for (int d = 0; d < dim; ++d) npc *= K1;
  std::vector<int32_t> id((size_t)npts, -1);
  // lattice point of local node a of a cell: kk * f0 + a * s (an unrefined cell's nodes sit every 2 points)
  auto cell_point = [&](const Cell &c, int a, int64_t *p) {
    int r = a;
    for (int d = 0; d < dim; ++d) {
      p[d] = (int64_t)kk * c.f0[d] + (int64_t)(r % K1) * c.s;
      r /= K1;
    }
  };
  for (const Cell &c : cells)
    for (int a = 0; a < npc; ++a) {
      int64_t p[3];
      cell_point(c, a, p);
      id[(size_t)lat(p)] = 0;
    }
  int32_t next = 0;
  node_x.clear();
  for (int64_t t = 0; t < npts; ++t)
    if (id[(size_t)t] == 0) {
      id[(size_t)t] = next++;
      int64_t r = t;
      for (int d = 0; d < dim; ++d) {
        node_x.push_back(lo + (double)(r % np1) * hf / kk);
        r /= np1;
      }
    }
  cell_nodes.resize(cells.size() * (size_t)npc);
  for (size_t ci = 0; ci < cells.size(); ++ci)
    for (int a = 0; a < npc; ++a) {
      int64_t p[3];
      cell_point(cells[ci], a, p);
      cell_nodes[ci * npc + a] = id[(size_t)lat(p)];
    }
  // hanging nodes: used lattice points on the closed box of an unrefined cell that are not its
  // nodes (an odd offset along the face); only a refined neighbour can use such a point
  std::vector<char> done((size_t)next, 0);
  hnode.clear();
  hoff.assign(1, 0);
  hw.clear();
  hmaster.clear();
  const int64_t span = 2 * (int64_t)kk;  // lattice intervals across an unrefined cell
  int64_t nbox = 1;
  for (int d = 0; d < dim; ++d) nbox *= span + 1;
  for (const Cell &c : cells) {
    if (c.s != 2) continue;
    for (int64_t b = 0; b < nbox; ++b) {
      int64_t off[3] = {0, 0, 0}, p[3] = {0, 0, 0}, r = b;
      bool on_boundary = false, is_node = true;
      for (int d = 0; d < dim; ++d) {
        off[d] = r % (span + 1);
        r /= span + 1;
        on_boundary = on_boundary || off[d] == 0 || off[d] == span;
        is_node = is_node && off[d] % 2 == 0;
        p[d] = (int64_t)kk * c.f0[d] + off[d];
      }
      if (!on_boundary || is_node) continue;
      const int32_t nid = id[(size_t)lat(p)];
      if (nid < 0 || done[(size_t)nid]) continue;  // unused point, or constrained already
      done[(size_t)nid] = 1;
      hnode.push_back(nid);
      for (int a = 0; a < npc; ++a) {
        double w = 1.0;
        int rr = a;
        int64_t q[3] = {0, 0, 0};
        for (int d = 0; d < dim; ++d) {
          const int ad = rr % K1;
          rr /= K1;
          w *= lagrange(kk, ad, (double)off[d] / span);
          q[d] = (int64_t)kk * c.f0[d] + 2 * ad;
        }
        if (std::fabs(w) < 1e-13) continue;
        hmaster.push_back(id[(size_t)lat(q)]);
        hw.push_back(w);
      }
      hoff.push_back((int64_t)hmaster.size());
    }
  }
  return GLS_OK;
}

}  // namespace

extern "C" {

int gls_mesh_refined_create(int dim, int n, int k, int kp, double lo, double hi, const int32_t *refine,
                            gls_refined_mesh **out) {
  if (!out) return gls_io_set_error(GLS_EINVAL, "null output");
  *out = nullptr;
  if ((dim != 2 && dim != 3) || n < 1 || k < 1 || k > 2 || kp < 1 || kp > k || !(hi > lo))
    return gls_io_set_error(GLS_EINVAL, "gls_mesh_refined_create: dim 2/3, n >= 1, 1 <= kp <= k <= 2");
  std::unique_ptr<RefinedMeshImpl> M(new RefinedMeshImpl);
  int64_t ncoarse = 1;
  for (int d = 0; d < dim; ++d) ncoarse *= n;
  std::vector<Cell> cells;
  for (int64_t c = 0; c < ncoarse; ++c) {
    int ijk[3] = {0, 0, 0};
    int64_t r = c;
    for (int d = 0; d < dim; ++d) {
      ijk[d] = (int)(r % n);
      r /= n;
    }
    if (refine && refine[c]) {
      for (int ch = 0; ch < (1 << dim); ++ch) {
        Cell cc{};
        for (int d = 0; d < dim; ++d) cc.f0[d] = 2 * ijk[d] + ((ch >> d) & 1);
        cc.s = 1;
        cells.push_back(cc);
      }
    } else {
      Cell cc{};
      for (int d = 0; d < dim; ++d) cc.f0[d] = 2 * ijk[d];
      cc.s = 2;
      cells.push_back(cc);
    }
  }
  const double hf = (hi - lo) / (2.0 * n);
  int rc = build_space(dim, n, k, lo, hf, cells, M->cell_vnodes, M->vnode_x, M->vh_node, M->vh_off, M->vh_w,
                       M->vh_master);
  if (rc != GLS_OK) return rc;
  rc = build_space(dim, n, kp, lo, hf, cells, M->cell_pnodes, M->pnode_x, M->ph_node, M->ph_off, M->ph_w,
                   M->ph_master);
  if (rc != GLS_OK) return rc;
  for (const Cell &c : cells) {
    for (int d = 0; d < dim; ++d) {
      M->cell_x0.push_back(lo + c.f0[d] * hf);
      M->cell_h.push_back(c.s * hf);
    }
    M->cell_level.push_back(c.s == 1 ? 1 : 0);
  }
  gls_refined_mesh &p = M->pub;
  p.dim = dim;
  p.k = k;
  p.kp = kp;
  p.n_cells = (int64_t)cells.size();
  p.n_vnodes = (int64_t)M->vnode_x.size() / dim;
  p.n_pnodes = (int64_t)M->pnode_x.size() / dim;
  p.cell_vnodes = M->cell_vnodes.data();
  p.cell_pnodes = M->cell_pnodes.data();
  p.cell_level = M->cell_level.data();
  p.cell_x0 = M->cell_x0.data();
  p.cell_h = M->cell_h.data();
  p.vnode_x = M->vnode_x.data();
  p.pnode_x = M->pnode_x.data();
  p.n_vhang = (int64_t)M->vh_node.size();
  p.vhang_node = M->vh_node.data();
  p.vhang_off = M->vh_off.data();
  p.vhang_master = M->vh_master.data();
  p.vhang_w = M->vh_w.data();
  p.n_phang = (int64_t)M->ph_node.size();
  p.phang_node = M->ph_node.data();
  p.phang_off = M->ph_off.data();
  p.phang_master = M->ph_master.data();
  p.phang_w = M->ph_w.data();
  p.impl_ = M.get();
  *out = &M.release()->pub;
  return GLS_OK;
}

int gls_mesh_refined_destroy(gls_refined_mesh *m) {
  if (m) delete static_cast<RefinedMeshImpl *>(m->impl_);
  return GLS_OK;
}

// dealii::GridRefinement::refine (deal.II 9.2 source/grid/grid_refinement.cc, not vendored), the
// marking step both refinement rules end in: nothing is flagged when every indicator is zero;
// a zero threshold is raised to the smallest positive indicator, the scan starting from
// criteria[0] as deal.II's does (so a leading zero keeps it at 0); cells with |c| >= threshold
// are flagged. Returns the number flagged.
static int refine_mark(int64_t n_cells, const float *criteria, double threshold, int32_t *flags, double *used) {
  bool all_zero = true;
  for (int64_t i = 0; i < n_cells && all_zero; ++i) all_zero = criteria[i] == 0.0f;
  if (used) *used = threshold;
  if (all_zero) return 0;
  double thr = threshold;
  if (thr == 0.0) {
    thr = criteria[0];
    for (int64_t i = 1; i < n_cells; ++i)
      if (criteria[i] > 0 && criteria[i] < thr) thr = criteria[i];
  }
  if (used) *used = thr;
  int cnt = 0;
  for (int64_t i = 0; i < n_cells; ++i)
    if (std::fabs(criteria[i]) >= thr) {
      flags[i] = 1;
      ++cnt;
    }
  return cnt;
}

// GridRefinement::refine_and_coarsen_fixed_number, refinement part (navier_stokes_base.cc:654-661 with
// the serial deal.II rule): n_refine = int(top_fraction * n_cells); threshold = the n_refine-th largest
// indicator (std::nth_element); every cell with criteria >= threshold is flagged (GridRefinement::refine).
int gls_refine_fixed_number(int64_t n_cells, const float *criteria, double top_fraction, int32_t *flags) {
  if (n_cells < 0 || (n_cells && (!criteria || !flags)) || top_fraction < 0 || top_fraction > 1)
    return gls_io_set_error(GLS_EINVAL, "gls_refine_fixed_number: bad arguments");
  for (int64_t i = 0; i < n_cells; ++i) flags[i] = 0;
  const int64_t nr = (int64_t)(top_fraction * (double)n_cells);
  if (nr <= 0) return 0;
  std::vector<float> tmp(criteria, criteria + n_cells);
  std::nth_element(tmp.begin(), tmp.begin() + (nr - 1), tmp.end(), std::greater<float>());
  const float thr = tmp[(size_t)(nr - 1)];
  return refine_mark(n_cells, criteria, thr, flags, nullptr);
}

// compute_threshold of parallel::distributed::GridRefinement (RefineAndCoarsenFixedNumber /
// RefineAndCoarsenFixedFraction, deal.II 9.2 source/distributed/grid_refinement.cc, not vendored):
// bisection between the slightly widened indicator extremes (geometric mean while the lower end is
// > 0), 25 steps at most; the number (fraction_type 0) or summed indicator (1) of cells strictly
// above the test value decides the half kept.
static double pd_threshold(int64_t n_cells, const float *criteria, int fraction_type, double lo, double hi,
                           double target) {
  const double gmax = hi;
  // adjust_interesting_range
  if (lo > 0) lo *= 0.99;
  if (hi > 0) hi *= 1.01;
  else hi += 0.01 * (hi - lo);
  for (int it = 0;; ++it) {
    if (lo == hi) return fraction_type == 1 ? std::min(lo, gmax) : lo;
    const double test = lo > 0 ? std::sqrt(lo * hi) : (lo + hi) / 2;
    double above = 0.0;
    for (int64_t i = 0; i < n_cells; ++i)
      if (criteria[i] > test) above += fraction_type == 0 ? 1.0 : (double)criteria[i];
    if (above > target) lo = test;
    else if (above < target) hi = test;
    else lo = hi = test;
    if (it + 1 == 25) lo = hi = test;
  }
}

// parallel::distributed::GridRefinement::refine_and_coarsen_fixed_number / _fixed_fraction, the call
// refine_mesh_kelly makes (navier_stokes_base.cc:654-667). Fixed number: the fractions are first
// capped by GridRefinement::adjust_refine_and_coarsen_number_fraction<dim> so that the mesh grows to
// at most max_n_cells (when it is already larger, coarsen (n - max) / (1 - 2^-dim) cells and refine
// none); top threshold: int(top * n) cells above it; bottom threshold: int((1 - bottom) * n) cells
// above it. Fixed fraction: top * (summed indicator) / (1 - bottom) * (summed indicator) above the
// thresholds. A zero bottom fraction gives the lowest representable threshold (no coarsening).
// mark_cells: GridRefinement::refine (criteria >= top, see refine_mark), then GridRefinement::coarsen
// (|criteria| <= bottom on cells not flagged for refinement). The summed quantities are global sums,
// so with per-rank indicators the caller gathers them first (the app adapts on one process).
int gls_refine_coarsen_pd(int64_t n_cells, const float *criteria, int dim, int fraction_type, double top_fraction,
                          double bottom_fraction, int64_t max_n_cells, int32_t *refine, int32_t *coarsen,
                          double *thresholds) {
  if (n_cells < 0 || (n_cells && (!criteria || !refine)) || (dim != 2 && dim != 3) || top_fraction < 0 ||
      top_fraction > 1 || bottom_fraction < 0 || bottom_fraction > 1 ||
      top_fraction + bottom_fraction > 1 + 1e-15 || (fraction_type != 0 && fraction_type != 1) || max_n_cells < 0 ||
      (bottom_fraction > 0 && n_cells && !coarsen))
    return gls_io_set_error(GLS_EINVAL, "gls_refine_coarsen_pd: bad arguments");
  for (int64_t i = 0; i < n_cells; ++i) refine[i] = 0;
  if (coarsen)
    for (int64_t i = 0; i < n_cells; ++i) coarsen[i] = 0;
  if (thresholds) thresholds[0] = thresholds[1] = 0.0;
  if (n_cells == 0) return 0;
  double lo = criteria[0], hi = criteria[0];
  float total = 0.0f;  // compute_global_sum accumulates in the indicator type
  for (int64_t i = 0; i < n_cells; ++i) {
    if (!(criteria[i] >= 0.0f)) return gls_io_set_error(GLS_EINVAL, "gls_refine_coarsen_pd: criteria must be >= 0");
    lo = std::min(lo, (double)criteria[i]);
    hi = std::max(hi, (double)criteria[i]);
    total += criteria[i];
  }
  double top = top_fraction, bottom = bottom_fraction, t_top, t_bottom;
  const double nc = (double)n_cells;
  if (fraction_type == 0) {
    const double inc = (double)((1 << dim) - 1), dec = 1.0 - 1.0 / (double)(1 << dim);
    const double rc = nc * top_fraction, cc = nc * bottom_fraction;
    if (n_cells >= max_n_cells) {
      top = 0.0;
      bottom = std::min((nc - (double)max_n_cells) / dec / nc, 1.0);
    } else if ((int64_t)(nc + rc * inc - cc * dec) > max_n_cells) {
      const double alpha = ((double)max_n_cells - nc) / (rc * inc - cc * dec);
      top = alpha * top_fraction;
      bottom = alpha * bottom_fraction;
    }
    t_top = (double)(int64_t)(top * nc);
    t_bottom = (double)(int64_t)((1.0 - bottom) * nc);
  } else {
    t_top = top_fraction * total;
    t_bottom = (1.0 - bottom_fraction) * total;
  }
  const double thr = pd_threshold(n_cells, criteria, fraction_type, lo, hi, t_top);
  double used = thr;
  const int nr = refine_mark(n_cells, criteria, thr, refine, &used);
  double bthr = -std::numeric_limits<float>::max();  // std::numeric_limits<Number>::lowest(), Number = float
  if (bottom > 0 && coarsen) {  // refinement-only callers pass no coarsen flags
    bthr = pd_threshold(n_cells, criteria, fraction_type, lo, hi, t_bottom);
    for (int64_t i = 0; i < n_cells; ++i)
      if (std::fabs(criteria[i]) <= bthr && !refine[i]) {
        coarsen[i] = 1;
      }
  }
  if (thresholds) {
    thresholds[0] = used;
    thresholds[1] = bthr;
  }
  return nr;
}

// the refinement-only call (fraction coarsening = 0): flags of gls_refine_coarsen_pd, threshold = top.
int gls_refine_pd(int64_t n_cells, const float *criteria, int dim, int fraction_type, double top_fraction,
                  int64_t max_n_cells, int32_t *flags, double *threshold) {
  double th[2];
  const int rc = gls_refine_coarsen_pd(n_cells, criteria, dim, fraction_type, top_fraction, 0.0, max_n_cells, flags,
                                       nullptr, th);
  if (rc >= 0 && threshold) *threshold = th[0];
  return rc;
}

// SolutionTransfer::interpolate for the first refinement of a uniform mesh (navier_stokes_base.cc:
// 689-733): every node of the refined mesh lies in a cell of hyper_cube(n, lo, hi), whose Qk
// interpolant it samples (exact for the refined space, which contains the coarse one).
int gls_mesh_refined_interpolate(const gls_refined_mesh *m, int n, double lo, double hi, const double *coarse,
                                 double *fine) {
  if (!m || !coarse || !fine || n < 1 || !(hi > lo)) return gls_io_set_error(GLS_EINVAL, "gls_mesh_refined_interpolate: bad arguments");
  const int dim = m->dim;
  const double hc = (hi - lo) / n;
  auto sample = [&](int kk, const double *x, int ncomp, int64_t base, int stride, double *out) {
    const int64_t np1 = (int64_t)kk * n + 1;
    int cidx[3] = {0, 0, 0};
    double xi[3] = {0, 0, 0};
    for (int d = 0; d < dim; ++d) {
      const double t = (x[d] - lo) / hc;
      cidx[d] = std::min(std::max((int)std::floor(t), 0), n - 1);
      xi[d] = t - cidx[d];
    }
    for (int c = 0; c < ncomp; ++c) out[c] = 0.0;
    const int na = dim == 3 ? (kk + 1) * (kk + 1) * (kk + 1) : (kk + 1) * (kk + 1);
    for (int a = 0; a < na; ++a) {
      const int ai[3] = {a % (kk + 1), (a / (kk + 1)) % (kk + 1), dim == 3 ? a / ((kk + 1) * (kk + 1)) : 0};
      double w = 1.0;
      int64_t node = 0, st = 1;
      for (int d = 0; d < dim; ++d) {
        w *= lagrange(kk, ai[d], xi[d]);
        node += ((int64_t)cidx[d] * kk + ai[d]) * st;
        st *= np1;
      }
      if (w == 0.0) continue;
      for (int c = 0; c < ncomp; ++c) out[c] += w * coarse[base + node * stride + c];
    }
  };
  int64_t nvc = 1, npc = 1;
  for (int d = 0; d < dim; ++d) {
    nvc *= (int64_t)m->k * n + 1;
    npc *= (int64_t)m->kp * n + 1;
  }
  (void)npc;
  for (int64_t i = 0; i < m->n_vnodes; ++i) sample(m->k, m->vnode_x + i * dim, dim, 0, dim, fine + i * dim);
  const int64_t fvoff = (int64_t)dim * m->n_vnodes, cvoff = (int64_t)dim * nvc;
  for (int64_t i = 0; i < m->n_pnodes; ++i) sample(m->kp, m->pnode_x + i * dim, 1, cvoff, 1, fine + fvoff + i);
  return GLS_OK;
}

}  // extern "C"
