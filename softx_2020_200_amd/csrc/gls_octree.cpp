// gls_octree.cpp — multi-level adaptive refinement of a hyper_cube (host C++17).
//
// The reference adapts a p4est forest (parallel::distributed::Triangulation with
// smoothing_on_refinement | smoothing_on_coarsening, navier_stokes_base.cc:55-60, 592-780):
// refine / coarsen flags from the Kelly thresholds, at most one level of difference between cells
// that share a vertex (limit_level_difference_at_vertices = p4est corner balance), coarsening only
// of complete sibling groups, then DoFTools::make_hanging_node_constraints with chains closed by
// AffineConstraints::close (gls_navier_stokes.cc:84, 143) and SolutionTransfer.
// Here the forest is one tree over hyper_cube(lo, hi) with n^dim level-0 cells; a leaf of level l
// covers a block of 2^(L-l) cells of the finest level L. Leaves are kept in depth-first Morton
// order (children lexicographic, x fastest), which is p4est's order for a single tree.
// gls_octree_mesh builds the FE_Q(k) / FE_Q(kp) node spaces on the finest node lattice with
// hanging lines whose masters are all unconstrained (chains resolved).
// Periodic directions (gls_octree_set_periodic; GridTools::collect_periodic_faces +
// add_periodicity, gls_navier_stokes.cc:130-134, 164-168): the forest's neighbourhoods wrap around
// them -- the 2:1 vertex balance, the smoothing's face neighbours and vertex levels, the Kelly faces --
// and the node lattice identifies the max face with the min face, so the hanging lines of a coarse
// cell also constrain a finer periodic neighbour's face nodes (periodicity and hanging constraints
// together, as make_periodicity_constraints + make_hanging_node_constraints close them). Restated, no
// reference golden covers it (no reference case combines periodicity with adaptation).
#include <algorithm>
#include <array>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <map>
#include <memory>
#include <unordered_map>
#include <vector>

#include "../../include/gls_native.h"

int gls_io_set_error(int code, const char *fmt, ...);  // gls_api.cpp

struct gls_octree {
  int dim = 3, n = 1;
  int pmask = 0;  // periodic directions (bit d)
  struct Leaf {
    int level;
    int64_t x[3];  // origin in units of its own level's cells
  };
  std::vector<Leaf> leaves;
  int max_level() const {
    int L = 0;
    for (const Leaf &c : leaves) L = std::max(L, c.level);
    return L;
  }
};

namespace {

using Leaf = gls_octree::Leaf;

// Morton key of a leaf's origin at level L (interleaved bits; base-grid index in the high bits)
uint64_t morton_key(const gls_octree &t, const Leaf &c, int L) {
  int64_t p[3] = {0, 0, 0};
  for (int d = 0; d < t.dim; ++d) p[d] = c.x[d] << (L - c.level);
  // base cell (level 0 block) lexicographic first, then the Morton order inside it
  const int64_t s = (int64_t)1 << L;
  int64_t base = 0, st = 1;
  for (int d = 0; d < t.dim; ++d) {
    base += (p[d] / s) * st;
    st *= t.n;
  }
  uint64_t m = 0;
  for (int b = L - 1; b >= 0; --b)
    for (int d = t.dim - 1; d >= 0; --d) m = (m << 1) | (uint64_t)(((p[d] % s) >> b) & 1);
  return ((uint64_t)base << (t.dim * L)) | m;
}
void sort_leaves(gls_octree &t) {
  const int L = t.max_level();
  std::stable_sort(t.leaves.begin(), t.leaves.end(),
                   [&](const Leaf &a, const Leaf &b) { return morton_key(t, a, L) < morton_key(t, b, L); });
}

// level of the leaf covering every finest-level cell (a dense grid: small trees only)
struct LevelGrid {
  int dim, L, pmask = 0;
  int64_t N;  // finest cells per direction
  std::vector<int8_t> lev;
  int at(const int64_t *p) const {
    int64_t id = 0, st = 1;
    for (int d = 0; d < dim; ++d) {
      int64_t q = p[d];
      if ((pmask >> d) & 1) q = ((q % N) + N) % N;  // periodic: the neighbourhood wraps
      else if (q < 0 || q >= N) return -1;
      id += q * st;
      st *= N;
    }
    return lev[(size_t)id];
  }
};
int make_grid(const gls_octree &t, int L, LevelGrid &g) {
  g.dim = t.dim;
  g.L = L;
  g.pmask = t.pmask;
  g.N = (int64_t)t.n << L;
  int64_t tot = 1;
  for (int d = 0; d < t.dim; ++d) tot *= g.N;
  if (tot > ((int64_t)1 << 28)) return gls_io_set_error(GLS_EINVAL, "octree: finest grid too large");
  g.lev.assign((size_t)tot, -1);
  for (const Leaf &c : t.leaves) {
    const int64_t s = (int64_t)1 << (L - c.level);
    int64_t nb = 1;
    for (int d = 0; d < t.dim; ++d) nb *= s;
    for (int64_t b = 0; b < nb; ++b) {
      int64_t r = b, id = 0, st = 1;
      for (int d = 0; d < t.dim; ++d) {
        id += (c.x[d] * s + r % s) * st;
        r /= s;
        st *= g.N;
      }
      g.lev[(size_t)id] = (int8_t)c.level;
    }
  }
  return GLS_OK;
}
// highest leaf level in the one-cell shell around leaf c (cells sharing a vertex with c)
int shell_max(const LevelGrid &g, const Leaf &c) {
  const int64_t s = (int64_t)1 << (g.L - c.level);
  int64_t lo[3] = {0, 0, 0}, ext[3] = {1, 1, 1};
  for (int d = 0; d < g.dim; ++d) {
    lo[d] = c.x[d] * s - 1;
    ext[d] = s + 2;
  }
  int m = -1;
  int64_t nb = 1;
  for (int d = 0; d < g.dim; ++d) nb *= ext[d];
  for (int64_t b = 0; b < nb; ++b) {
    int64_t p[3] = {0, 0, 0}, r = b;
    bool inside = true;
    for (int d = 0; d < g.dim; ++d) {
      p[d] = lo[d] + r % ext[d];
      r /= ext[d];
      inside = inside && p[d] > lo[d] && p[d] < lo[d] + ext[d] - 1;
    }
    if (inside) continue;
    m = std::max(m, g.at(p));
  }
  return m;
}

std::vector<Leaf> children(const gls_octree &t, const Leaf &c) {
  std::vector<Leaf> out;
  for (int ch = 0; ch < (1 << t.dim); ++ch) {
    Leaf k{c.level + 1, {0, 0, 0}};
    for (int d = 0; d < t.dim; ++d) k.x[d] = 2 * c.x[d] + ((ch >> d) & 1);
    out.push_back(k);
  }
  return out;
}

// 2:1 balance over vertices: refine every leaf that shares a vertex with a leaf two levels finer
int balance(gls_octree &t) {
  for (int it = 0; it < 64; ++it) {
    const int L = t.max_level();
    LevelGrid g;
    if (int rc = make_grid(t, L, g); rc != GLS_OK) return rc;
    std::vector<Leaf> next;
    bool changed = false;
    for (const Leaf &c : t.leaves) {
      if (shell_max(g, c) >= c.level + 2) {
        for (const Leaf &k : children(t, c)) next.push_back(k);
        changed = true;
      } else {
        next.push_back(c);
      }
    }
    t.leaves.swap(next);
    if (!changed) break;
  }
  return GLS_OK;
}

double lagrange(int k, int a, double xi) {  // degree-k Lagrange basis a on the nodes b/k
  double v = 1.0;
  for (int b = 0; b <= k; ++b)
    if (b != a) v *= (xi - (double)b / k) / ((double)(a - b) / k);
  return v;
}

struct MeshImpl {
  gls_refined_mesh pub{};
  std::vector<int32_t> cell_vnodes, cell_pnodes, cell_level;
  std::vector<double> cell_x0, cell_h, vnode_x, pnode_x;
  std::vector<int64_t> vh_node, vh_off, vh_master, ph_node, ph_off, ph_master;
  std::vector<double> vh_w, ph_w;
  // for transfers: the tree geometry
  int n = 1, L = 0, pmask = 0;
  double lo = 0, hi = 1;
};

// FE_Q(kk) nodes on the finest node lattice (spacing h_L / kk), hanging lines with chains closed
int build_space(const gls_octree &t, int L, int kk, double lo, double hf, std::vector<int32_t> &cell_nodes,
                std::vector<double> &node_x, std::vector<int64_t> &hnode, std::vector<int64_t> &hoff,
                std::vector<double> &hw, std::vector<int64_t> &hmaster) {
  const int dim = t.dim;
  const int64_t np1 = (int64_t)kk * ((int64_t)t.n << L) + 1;
  int64_t npts = 1;
  for (int d = 0; d < dim; ++d) npts *= np1;
  if (npts > ((int64_t)1 << 31)) return gls_io_set_error(GLS_EINVAL, "octree mesh lattice too large");
  auto lat = [&](const int64_t *p) {  // periodic directions: the max face is the min face
    int64_t id = 0, st = 1;
    for (int d = 0; d < dim; ++d) {
      id += (((t.pmask >> d) & 1) ? p[d] % (np1 - 1) : p[d]) * st;
      st *= np1;
    }
    return id;
  };
  const int K1 = kk + 1;
  int npc = 1;
  for (int d = 0; d < dim; ++d) npc *= K1;
  // lattice point of local node a of leaf c: kk * origin + a * s, s = finest cells per leaf edge
  auto cell_point = [&](const Leaf &c, int a, int64_t *p) {
    const int64_t s = (int64_t)1 << (L - c.level);
    int r = a;
    for (int d = 0; d < dim; ++d) {
      p[d] = (int64_t)kk * c.x[d] * s + (int64_t)(r % K1) * s;
      r /= K1;
    }
  };
  std::unordered_map<int64_t, int32_t> id;
  id.reserve((size_t)t.leaves.size() * npc);
  for (const Leaf &c : t.leaves)
    for (int a = 0; a < npc; ++a) {
      int64_t p[3];
      cell_point(c, a, p);
      id.emplace(lat(p), 0);
    }
  std::vector<int64_t> used;
  used.reserve(id.size());
  for (auto &kv : id) used.push_back(kv.first);
  std::sort(used.begin(), used.end());  // lexicographic lattice order (x fastest)
  node_x.clear();
  for (size_t i = 0; i < used.size(); ++i) {
    id[used[i]] = (int32_t)i;
    int64_t r = used[i];
    for (int d = 0; d < dim; ++d) {
      node_x.push_back(lo + (double)(r % np1) * hf / kk);
      r /= np1;
    }
  }
  cell_nodes.resize(t.leaves.size() * (size_t)npc);
  for (size_t ci = 0; ci < t.leaves.size(); ++ci)
    for (int a = 0; a < npc; ++a) {
      int64_t p[3];
      cell_point(t.leaves[ci], a, p);
      cell_nodes[ci * npc + a] = id[lat(p)];
    }
  // raw lines: a used lattice point on the closed box of a leaf that is not one of its nodes is
  // hanging on that leaf's Qk interpolant (only a finer neighbour uses it)
  std::map<int32_t, std::vector<std::pair<int32_t, double>>> line;
  for (const Leaf &c : t.leaves) {
    if (c.level == L) continue;
    const int64_t s = (int64_t)1 << (L - c.level), span = (int64_t)kk * s;
    int64_t nbox = 1;
    for (int d = 0; d < dim; ++d) nbox *= span + 1;
    for (int64_t b = 0; b < nbox; ++b) {
      int64_t off[3] = {0, 0, 0}, p[3] = {0, 0, 0}, r = b;
      bool on_boundary = false, is_node = true;
      for (int d = 0; d < dim; ++d) {
        off[d] = r % (span + 1);
        r /= span + 1;
        on_boundary = on_boundary || off[d] == 0 || off[d] == span;
        is_node = is_node && off[d] % s == 0;
        p[d] = (int64_t)kk * c.x[d] * s + off[d];
      }
      if (!on_boundary || is_node) continue;
      auto it = id.find(lat(p));
      if (it == id.end() || line.count(it->second)) continue;
      std::vector<std::pair<int32_t, double>> ln;
      for (int a = 0; a < npc; ++a) {
        double w = 1.0;
        int rr = a;
        int64_t q[3] = {0, 0, 0};
        for (int d = 0; d < dim; ++d) {
          const int ad = rr % K1;
          rr /= K1;
          w *= lagrange(kk, ad, (double)off[d] / span);
          q[d] = (int64_t)kk * c.x[d] * s + (int64_t)ad * s;
        }
        if (std::fabs(w) < 1e-13) continue;
        ln.push_back({id[lat(q)], w});
      }
      line[it->second] = ln;
    }
  }
  // close the chains (AffineConstraints::close): substitute hanging masters by their lines
  for (int pass = 0; pass < 32; ++pass) {
    bool changed = false;
    for (auto &kv : line) {
      std::map<int32_t, double> acc;
      bool sub = false;
      for (auto &mw : kv.second) {
        auto it = line.find(mw.first);
        if (it == line.end()) {
          acc[mw.first] += mw.second;
        } else {
          sub = true;
          for (auto &m2 : it->second) acc[m2.first] += mw.second * m2.second;
        }
      }
      if (sub) {
        kv.second.clear();
        for (auto &a : acc)
          if (std::fabs(a.second) > 1e-14) kv.second.push_back(a);
        changed = true;
      }
    }
    if (!changed) break;
    if (pass == 31) return gls_io_set_error(GLS_EINVAL, "octree: hanging-node chains do not close");
  }
  hnode.clear();
  hoff.assign(1, 0);
  hw.clear();
  hmaster.clear();
  for (auto &kv : line) {
    hnode.push_back(kv.first);
    for (auto &mw : kv.second) {
      hmaster.push_back(mw.first);
      hw.push_back(mw.second);
    }
    hoff.push_back((int64_t)hmaster.size());
  }
  return GLS_OK;
}

// Triangulation::prepare_coarsening_and_refinement (deal.II 9.2 source/grid/tria.cc, third party, not
// vendored: restated from its published algorithm) with MeshSmoothing smoothing_on_refinement |
// smoothing_on_coarsening, as the reference constructs its triangulation (navier_stokes_base.cc:55-60)
// and calls it after the Kelly marking (:682). Cells are the tree's nodes (leaves = active cells,
// their ancestors = refined cells); "all cells" are visited level by level in Morton order, the
// active cells in reverse (finest level first), as deal.II's cell iterators run for a tree refined
// from one coarse cell. Isotropic refinement only.
struct Smoother {
  const gls_octree &t;
  int dim, LM;
  std::vector<char> ref, crs;                  // per-leaf refine / coarsen flags
  std::unordered_map<uint64_t, int32_t> node;  // (level, x) -> leaf index, or -1 for a refined cell
  std::vector<Leaf> all;                       // every cell, level-wise Morton order
  std::vector<size_t> active_rev;              // leaves, reverse of deal.II's active order
  std::unordered_map<uint64_t, char> user;     // refined cells to be coarsened (fix_coarsen_flags)

  static uint64_t key(int level, const int64_t *x) {
    return ((uint64_t)level << 58) | ((uint64_t)x[0] << 38) | ((uint64_t)x[1] << 19) | (uint64_t)x[2];
  }
  int64_t extent(int level) const { return (int64_t)t.n << level; }
  Smoother(const gls_octree &tree, const int32_t *r, const int32_t *c) : t(tree), dim(tree.dim) {
    LM = tree.max_level();
    const size_t nc = tree.leaves.size();
    ref.resize(nc);
    crs.resize(nc);
    for (size_t i = 0; i < nc; ++i) {
      ref[i] = r[i] != 0;
      crs[i] = c[i] != 0;
      const Leaf &l = tree.leaves[i];
      node[key(l.level, l.x)] = (int32_t)i;
      all.push_back(l);
    }
    for (size_t i = 0; i < nc; ++i) {
      Leaf a = tree.leaves[i];
      while (a.level > 0) {
        a.level -= 1;
        for (int d = 0; d < 3; ++d) a.x[d] /= 2;
        if (node.count(key(a.level, a.x))) break;
        node[key(a.level, a.x)] = -1;
        all.push_back(a);
      }
    }
    std::sort(all.begin(), all.end(), [&](const Leaf &a, const Leaf &b) {
      if (a.level != b.level) return a.level < b.level;
      return morton_key(t, a, LM) < morton_key(t, b, LM);
    });
    for (size_t j = all.size(); j-- > 0;) {
      const int32_t v = node[key(all[j].level, all[j].x)];
      if (v >= 0) active_rev.push_back((size_t)v);
    }
  }
  int32_t find(int level, const int64_t *x) const {  // -2: no such cell
    auto it = node.find(key(level, x));
    return it == node.end() ? -2 : it->second;
  }
  bool is_active(const Leaf &c) const { return find(c.level, c.x) >= 0; }
  // cell->neighbor(f): the cell of the same level across face f (active or refined), else the
  // coarser active cell; returns 0 at the boundary, 1 same level, 2 coarser
  int neighbor(const Leaf &c, int f, Leaf &nb) const {
    const int d = f / 2;
    nb = c;
    nb.x[d] += (f & 1) ? 1 : -1;
    if (nb.x[d] < 0 || nb.x[d] >= extent(c.level)) {
      if (!((t.pmask >> d) & 1)) return 0;
      nb.x[d] = (nb.x[d] + extent(c.level)) % extent(c.level);  // periodic neighbour
    }
    if (find(nb.level, nb.x) != -2) return 1;
    nb.level -= 1;
    for (int e = 0; e < 3; ++e) nb.x[e] /= 2;
    return 2;
  }
  std::vector<Leaf> kids(const Leaf &c) const { return children(t, c); }
  size_t leaf(const Leaf &c) const { return (size_t)find(c.level, c.x); }
  // cell_will_be_coarsened: every child active and flagged; otherwise the children's flags are cleared
  bool will_be_coarsened(const Leaf &c) {
    if (is_active(c)) return false;
    int n = 0;
    const std::vector<Leaf> ch = kids(c);
    for (const Leaf &k : ch) {
      const int32_t v = find(k.level, k.x);
      if (v >= 0 && crs[(size_t)v]) ++n;
    }
    if (n == (int)ch.size()) return true;
    for (const Leaf &k : ch) {
      const int32_t v = find(k.level, k.x);
      if (v >= 0) crs[(size_t)v] = 0;
    }
    return false;
  }
  // face_will_be_refined_by_neighbor (isotropic): a refined neighbour that stays refined, or an
  // active one flagged for refinement, of the same level
  bool face_refined_by_neighbor(const Leaf &c, int f) {
    Leaf nb;
    if (neighbor(c, f, nb) != 1) return false;
    const int32_t v = find(nb.level, nb.x);
    if (v < 0) return !will_be_coarsened(nb);
    return ref[(size_t)v] != 0;
  }
  uint64_t vkey(const Leaf &c, int corner) const {  // vertex on the lattice of level LM + 1
    int64_t v[3] = {0, 0, 0};
    for (int d = 0; d < dim; ++d) {
      v[d] = (c.x[d] + ((corner >> d) & 1)) << (LM + 1 - c.level);
      if ((t.pmask >> d) & 1) v[d] %= extent(LM + 1);  // periodic: the max vertex is the min vertex
    }
    return ((uint64_t)v[0] << 42) | ((uint64_t)v[1] << 21) | (uint64_t)v[2];
  }
  // limit_level_difference_at_vertices (step 3, repeated in fix_coarsen_flags): the highest future
  // level at each vertex (a cell flagged for coarsening tentatively counts one level down), then in
  // reverse order a cell below it loses its coarsen flag, and is refined when two levels below
  void limit_vertex_levels() {
    std::unordered_map<uint64_t, int> vl;
    const int nv = 1 << dim;
    for (size_t i = 0; i < t.leaves.size(); ++i) {
      const Leaf &c = t.leaves[i];
      const int lev = ref[i] ? c.level + 1 : crs[i] ? c.level - 1 : c.level;
      for (int v = 0; v < nv; ++v) {
        auto it = vl.find(vkey(c, v));
        if (it == vl.end()) vl[vkey(c, v)] = std::max(0, lev);
        else it->second = std::max(it->second, lev);
      }
    }
    for (size_t i : active_rev) {
      if (ref[i]) continue;
      const Leaf &c = t.leaves[i];
      for (int v = 0; v < nv; ++v) {
        const int lv = vl[vkey(c, v)];
        if (lv < c.level + 1) continue;
        crs[i] = 0;
        if (lv > c.level + 1) {
          ref[i] = 1;
          for (int w = 0; w < nv; ++w) vl[vkey(c, w)] = std::max(vl[vkey(c, w)], c.level + 1);
        }
      }
    }
  }
  // coarsening_allowed: no child on a face of p may have a same-level neighbour that is refined and
  // stays so, or is flagged for refinement (the 3D line rule is implied by the vertex rule)
  bool coarsening_allowed(const Leaf &p) const {
    for (int f = 0; f < 2 * dim; ++f) {
      Leaf nb;
      if (neighbor(p, f, nb) == 0) continue;
      const int d = f / 2;
      for (const Leaf &ch : kids(p)) {
        if (((ch.x[d] & 1) != 0) != ((f & 1) != 0)) continue;  // child not on face f
        Leaf cn;
        if (neighbor(ch, f, cn) != 1) continue;
        const int32_t v = find(cn.level, cn.x);
        if (v < 0 && !user.count(key(cn.level, cn.x))) return false;
        if (v >= 0 && ref[(size_t)v]) return false;
      }
    }
    return true;
  }
  // fix_coarsen_flags: coarsen flags survive only on complete families whose coarsening is allowed
  void fix_coarsen_flags() {
    for (int it = 0; it < 1000; ++it) {
      const std::vector<char> before = crs;
      limit_vertex_levels();
      for (size_t i = 0; i < t.leaves.size(); ++i)
        if (t.leaves[i].level == 0) crs[i] = 0;
      user.clear();
      for (const Leaf &c : all) {
        if (is_active(c)) continue;
        int n = 0;
        const std::vector<Leaf> ch = kids(c);
        for (const Leaf &k : ch) {
          const int32_t v = find(k.level, k.x);
          if (v >= 0 && crs[(size_t)v]) {
            ++n;
            crs[(size_t)v] = 0;
          }
        }
        if (n == (int)ch.size()) user[key(c.level, c.x)] = 1;
      }
      for (size_t j = all.size(); j-- > 0;) {
        const Leaf &c = all[j];
        if (!user.count(key(c.level, c.x)) || !coarsening_allowed(c)) continue;
        for (const Leaf &k : kids(c)) crs[leaf(k)] = 1;
      }
      user.clear();
      if (crs == before) break;
    }
  }
  int run() {
    const int nf = 2 * dim;
    int loops = 0;
    while (loops < 1000) {
      ++loops;
      const std::vector<char> r0 = ref, c0 = crs;
      // step 1: do_not_produce_unrefined_islands — keep a family whose neighbours (all, or all but
      // one of an interior cell's) will be refined
      for (const Leaf &c : all) {
        if (is_active(c) || !will_be_coarsened(c)) continue;
        int n_nb = 0, cnt = 0;
        for (int f = 0; f < nf; ++f) {
          Leaf nb;
          if (neighbor(c, f, nb) == 0) continue;
          ++n_nb;
          if (face_refined_by_neighbor(c, f)) ++cnt;
        }
        if (cnt == n_nb || (cnt == n_nb - 1 && n_nb == nf))
          for (const Leaf &k : kids(c)) crs[leaf(k)] = 0;
      }
      // step 2: eliminate_refined_inner_islands | eliminate_refined_boundary_islands — a cell
      // refined (or flagged) whose neighbours will all be unrefined is coarsened (or unflagged)
      for (const Leaf &c : all) {
        const int32_t v = find(c.level, c.x);
        if (v >= 0 && !ref[(size_t)v]) continue;
        bool all_active = true;
        if (v < 0)
          for (const Leaf &k : kids(c)) all_active = all_active && is_active(k);
        if (!all_active) continue;
        int total = 0, unrefined = 0;
        for (int f = 0; f < nf; ++f) {
          Leaf nb;
          if (neighbor(c, f, nb) == 0) continue;
          ++total;
          if (!face_refined_by_neighbor(c, f)) ++unrefined;
        }
        if (unrefined != total || total == 0) continue;
        if (v < 0) {
          for (const Leaf &k : kids(c)) {
            ref[leaf(k)] = 0;
            crs[leaf(k)] = 1;
          }
        } else {
          ref[(size_t)v] = 0;
        }
      }
      // step 3
      limit_vertex_levels();
      // step 4: eliminate_unrefined_islands — refine a cell with more refined than unrefined
      // interior neighbours
      for (size_t i : active_rev) {
        if (ref[i]) continue;
        const Leaf &c = t.leaves[i];
        int refined = 0, unrefined = 0;
        for (int f = 0; f < nf; ++f) {
          Leaf nb;
          if (neighbor(c, f, nb) == 0) continue;
          if (face_refined_by_neighbor(c, f)) ++refined;
          else ++unrefined;
        }
        if (unrefined < refined) {
          crs[i] = 0;
          ref[i] = 1;
        }
      }
      // step 6: no double refinement at a face — the coarser neighbour of a cell to be refined is refined
      for (size_t i : active_rev) {
        if (!ref[i]) continue;
        const Leaf &c = t.leaves[i];
        for (int f = 0; f < nf; ++f) {
          Leaf nb;
          if (neighbor(c, f, nb) != 2) continue;
          const size_t j = leaf(nb);
          crs[j] = 0;
          ref[j] = 1;
        }
      }
      // step 8
      fix_coarsen_flags();
      if (ref == r0 && crs == c0) break;
    }
    return loops;
  }
};

}  // namespace

extern "C" {

int gls_octree_create(int dim, int n, gls_octree **out) {
  if (!out || (dim != 2 && dim != 3) || n < 1) return gls_io_set_error(GLS_EINVAL, "gls_octree_create: dim 2/3, n >= 1");
  auto t = std::make_unique<gls_octree>();
  t->dim = dim;
  t->n = n;
  for (int64_t c = 0, nc = dim == 3 ? (int64_t)n * n * n : (int64_t)n * n; c < nc; ++c) {
    Leaf l{0, {c % n, (c / n) % n, dim == 3 ? c / ((int64_t)n * n) : 0}};
    t->leaves.push_back(l);
  }
  sort_leaves(*t);
  *out = t.release();
  return GLS_OK;
}
void gls_octree_destroy(gls_octree *t) { delete t; }

int gls_octree_set_periodic(gls_octree *t, int mask) {
  if (!t || mask < 0 || mask >= (1 << t->dim)) return gls_io_set_error(GLS_EINVAL, "gls_octree_set_periodic: bad mask");
  t->pmask = mask;
  return GLS_OK;
}

int gls_octree_info(const gls_octree *t, int64_t *n_cells, int *max_level) {
  if (!t) return gls_io_set_error(GLS_EINVAL, "null octree");
  if (n_cells) *n_cells = (int64_t)t->leaves.size();
  if (max_level) *max_level = t->max_level();
  return GLS_OK;
}

int gls_octree_cells(const gls_octree *t, int32_t *level, double *x0, double *h, double lo, double hi) {
  if (!t) return gls_io_set_error(GLS_EINVAL, "null octree");
  for (size_t i = 0; i < t->leaves.size(); ++i) {
    const Leaf &c = t->leaves[i];
    const double hc = (hi - lo) / ((double)t->n * (double)((int64_t)1 << c.level));
    if (level) level[i] = c.level;
    for (int d = 0; d < t->dim; ++d) {
      if (x0) x0[i * t->dim + d] = lo + c.x[d] * hc;
      if (h) h[i * t->dim + d] = hc;
    }
  }
  return GLS_OK;
}

// execute_coarsening_and_refinement: flagged leaves below max_level are refined, complete sibling
// groups whose members are all flagged for coarsening (and none for refinement) above min_level are
// coarsened unless that breaks the vertex 2:1 balance, then the balance is restored by refinement
int gls_octree_adapt(gls_octree *t, const int32_t *refine, const int32_t *coarsen, int max_level, int min_level) {
  if (!t) return gls_io_set_error(GLS_EINVAL, "null octree");
  const size_t nc = t->leaves.size();
  std::vector<Leaf> next;
  std::map<std::vector<int64_t>, std::vector<size_t>> groups;  // parent key -> member leaves
  std::vector<char> coarse_ok(nc, 0);
  for (size_t i = 0; i < nc; ++i) {
    const Leaf &c = t->leaves[i];
    if (coarsen && coarsen[i] && !(refine && refine[i]) && c.level > min_level) {
      std::vector<int64_t> key{c.level - 1, c.x[0] / 2, c.x[1] / 2, c.x[2] / 2};
      groups[key].push_back(i);
    }
  }
  // coarsening candidates: complete groups that keep the balance with the refined neighbours
  int L = t->max_level() + 1;
  std::vector<Leaf> refined;
  for (size_t i = 0; i < nc; ++i) {
    const Leaf &c = t->leaves[i];
    if (refine && refine[i] && c.level < max_level)
      for (const Leaf &k : children(*t, c)) refined.push_back(k);
    else
      refined.push_back(c);
  }
  gls_octree tmp = *t;
  tmp.leaves = refined;
  if (int rc = balance(tmp); rc != GLS_OK) return rc;
  L = std::max(L, tmp.max_level());
  LevelGrid g;
  if (int rc = make_grid(tmp, tmp.max_level(), g); rc != GLS_OK) return rc;
  std::map<std::vector<int64_t>, char> drop;  // parents that replace their children
  std::map<std::vector<int64_t>, char> is_leaf;
  for (const Leaf &c : tmp.leaves) is_leaf[{c.level, c.x[0], c.x[1], c.x[2]}] = 1;
  for (auto &kv : groups) {
    if ((int)kv.second.size() != (1 << t->dim)) continue;
    Leaf p{(int)kv.first[0], {kv.first[1], kv.first[2], kv.first[3]}};
    // every child is still a leaf after the refinement / balance pass, and no leaf sharing a
    // vertex with the parent is two levels finer than the parent
    bool ok = true;
    for (const Leaf &ch : children(*t, p)) ok = ok && is_leaf.count({ch.level, ch.x[0], ch.x[1], ch.x[2]});
    if (!ok || shell_max(g, p) >= p.level + 2) continue;
    drop[kv.first] = 1;
  }
  next.clear();
  std::map<std::vector<int64_t>, char> emitted;
  for (const Leaf &c : tmp.leaves) {
    if (c.level > 0) {
      std::vector<int64_t> key{c.level - 1, c.x[0] / 2, c.x[1] / 2, c.x[2] / 2};
      if (drop.count(key)) {
        if (!emitted.count(key)) {
          emitted[key] = 1;
          next.push_back(Leaf{c.level - 1, {key[1], key[2], key[3]}});
        }
        continue;
      }
    }
    next.push_back(c);
  }
  t->leaves.swap(next);
  if (int rc = balance(*t); rc != GLS_OK) return rc;
  sort_leaves(*t);
  return GLS_OK;
}

int gls_octree_prepare(const gls_octree *t, int32_t *refine, int32_t *coarsen) {
  if (!t || (!t->leaves.empty() && (!refine || !coarsen))) return gls_io_set_error(GLS_EINVAL, "gls_octree_prepare: bad arguments");
  if ((t->n << (t->max_level() + 1)) >= ((int64_t)1 << 19)) return gls_io_set_error(GLS_EINVAL, "gls_octree_prepare: tree too deep");
  Smoother sm(*t, refine, coarsen);
  const int loops = sm.run();
  for (size_t i = 0; i < t->leaves.size(); ++i) {
    refine[i] = sm.ref[i];
    coarsen[i] = sm.crs[i];
  }
  return loops;
}

int gls_octree_mesh(const gls_octree *t, int k, int kp, double lo, double hi, gls_refined_mesh **out) {
  if (!t || !out || k < 1 || k > 2 || kp < 1 || kp > k || !(hi > lo))
    return gls_io_set_error(GLS_EINVAL, "gls_octree_mesh: 1 <= kp <= k <= 2");
  const int L = t->max_level(), dim = t->dim;
  auto M = std::make_unique<MeshImpl>();
  const double hf = (hi - lo) / ((double)t->n * (double)((int64_t)1 << L));
  int rc = build_space(*t, L, k, lo, hf, M->cell_vnodes, M->vnode_x, M->vh_node, M->vh_off, M->vh_w, M->vh_master);
  if (rc != GLS_OK) return rc;
  rc = build_space(*t, L, kp, lo, hf, M->cell_pnodes, M->pnode_x, M->ph_node, M->ph_off, M->ph_w, M->ph_master);
  if (rc != GLS_OK) return rc;
  for (const Leaf &c : t->leaves) {
    const double hc = hf * (double)((int64_t)1 << (L - c.level));
    for (int d = 0; d < dim; ++d) {
      M->cell_x0.push_back(lo + (double)c.x[d] * hc);
      M->cell_h.push_back(hc);
    }
    M->cell_level.push_back(c.level);
  }
  M->n = t->n;
  M->L = L;
  M->pmask = t->pmask;
  M->lo = lo;
  M->hi = hi;
  gls_refined_mesh &p = M->pub;
  p.dim = dim;
  p.k = k;
  p.kp = kp;
  p.n_cells = (int64_t)t->leaves.size();
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
int gls_octree_mesh_destroy(gls_refined_mesh *m) {
  if (m) delete static_cast<MeshImpl *>(m->impl_);
  return GLS_OK;
}

// SolutionTransfer between two meshes of the same hyper_cube (refinement and coarsening): every
// node of the new mesh takes the old FE field's value at its position (the old cell containing
// it, its Qk interpolant). Lagrange nodes of a coarsened parent coincide with its children's
// nodes, so coarsening is exact injection, as deal.II's restriction of FE_Q is. Host vectors in
// the [velocity node-major | pressure] layout.
int gls_octree_transfer(const gls_refined_mesh *om, const gls_refined_mesh *nm, const double *ov, double *nv) {
  if (!om || !nm || !ov || !nv || om->dim != nm->dim || om->k != nm->k || om->kp != nm->kp)
    return gls_io_set_error(GLS_EINVAL, "gls_octree_transfer: incompatible meshes");
  const int dim = om->dim;
  const MeshImpl *O = static_cast<const MeshImpl *>(om->impl_);
  // locate old cells through a grid of the old finest cells
  const int64_t N = (int64_t)O->n << O->L;
  int64_t tot = 1;
  for (int d = 0; d < dim; ++d) tot *= N;
  if (tot > ((int64_t)1 << 28)) return gls_io_set_error(GLS_EINVAL, "gls_octree_transfer: grid too large");
  std::vector<int32_t> owner((size_t)tot, -1);
  const double hf = (O->hi - O->lo) / (double)N;
  for (int64_t c = 0; c < om->n_cells; ++c) {
    int64_t o[3] = {0, 0, 0}, s = (int64_t)std::llround(om->cell_h[c * dim] / hf);
    for (int d = 0; d < dim; ++d) o[d] = (int64_t)std::llround((om->cell_x0[c * dim + d] - O->lo) / hf);
    int64_t nb = 1;
    for (int d = 0; d < dim; ++d) nb *= s;
    for (int64_t b = 0; b < nb; ++b) {
      int64_t r = b, id = 0, st = 1;
      for (int d = 0; d < dim; ++d) {
        id += (o[d] + r % s) * st;
        r /= s;
        st *= N;
      }
      owner[(size_t)id] = (int32_t)c;
    }
  }
  auto eval = [&](const double *x, int comp) {
    const bool vel = comp < dim;
    const int kk = vel ? om->k : om->kp, K1 = kk + 1;
    int64_t q[3] = {0, 0, 0};
    for (int d = 0; d < dim; ++d) {
      int64_t v = (int64_t)std::floor((x[d] - O->lo) / hf);
      q[d] = std::min(std::max(v, (int64_t)0), N - 1);
    }
    int64_t id = 0, st = 1;
    for (int d = 0; d < dim; ++d) {
      id += q[d] * st;
      st *= N;
    }
    const int32_t c = owner[(size_t)id];
    double xi[3] = {0, 0, 0};
    for (int d = 0; d < dim; ++d) xi[d] = (x[d] - om->cell_x0[c * dim + d]) / om->cell_h[c * dim + d];
    const int npc = dim == 3 ? K1 * K1 * K1 : K1 * K1;
    const int32_t *cn = vel ? om->cell_vnodes + (int64_t)c * npc : om->cell_pnodes + (int64_t)c * npc;
    double s = 0;
    for (int a = 0; a < npc; ++a) {
      double w = 1.0;
      int r = a;
      for (int d = 0; d < dim; ++d) {
        w *= lagrange(kk, r % K1, xi[d]);
        r /= K1;
      }
      s += w * (vel ? ov[(int64_t)cn[a] * dim + comp] : ov[(int64_t)dim * om->n_vnodes + cn[a]]);
    }
    return s;
  };
  for (int64_t v = 0; v < nm->n_vnodes; ++v)
    for (int c = 0; c < dim; ++c) nv[v * dim + c] = eval(nm->vnode_x + v * dim, c);
  for (int64_t p = 0; p < nm->n_pnodes; ++p) nv[(int64_t)dim * nm->n_vnodes + p] = eval(nm->pnode_x + p * dim, dim);
  return GLS_OK;
}

// Interior faces of an octree mesh for KellyErrorEstimator, one entry per pair of cells sharing a
// piece of face: cell a's face at xi_d = 1 against cell b's face at xi_d = 0. On a non-conforming
// face the piece is the fine cell's whole face, a subface of the coarse one (deal.II integrates the
// jump over the subfaces of a refined neighbour, internal::integrate_over_irregular_face). rect_a /
// rect_b: [n][2 tangential dims][lo, hi] of the piece in each cell's reference coordinates.
// Call with null arrays to get the count.
int gls_octree_faces(const gls_refined_mesh *m, int64_t *n_faces, int32_t *fa, int32_t *fb, int32_t *fdir,
                     double *rect_a, double *rect_b) {
  if (!m || !n_faces) return gls_io_set_error(GLS_EINVAL, "gls_octree_faces: null argument");
  const MeshImpl *M = static_cast<const MeshImpl *>(m->impl_);
  const int dim = m->dim;
  const double hf = (M->hi - M->lo) / ((double)M->n * (double)((int64_t)1 << M->L));
  // integer finest-lattice boxes
  std::vector<std::array<int64_t, 6>> box((size_t)m->n_cells);
  for (int64_t c = 0; c < m->n_cells; ++c)
    for (int d = 0; d < 3; ++d) {
      const int64_t lo = d < dim ? (int64_t)std::llround((m->cell_x0[c * dim + d] - M->lo) / hf) : 0;
      const int64_t s = d < dim ? (int64_t)std::llround(m->cell_h[c * dim + d] / hf) : 1;
      box[(size_t)c][d] = lo;
      box[(size_t)c][3 + d] = lo + s;
    }
  // cells by (normal dir, low-face coordinate)
  std::map<std::pair<int, int64_t>, std::vector<int32_t>> low;
  for (int64_t c = 0; c < m->n_cells; ++c)
    for (int d = 0; d < dim; ++d) low[{d, box[(size_t)c][d]}].push_back((int32_t)c);
  int64_t cnt = 0;
  const int64_t NL = (int64_t)M->n << M->L;
  for (int64_t a = 0; a < m->n_cells; ++a)
    for (int d = 0; d < dim; ++d) {
      int64_t hi = box[(size_t)a][3 + d];
      if (((M->pmask >> d) & 1) && hi == NL) hi = 0;  // periodic face pair: a at the max, b at the min face
      auto it = low.find({d, hi});
      if (it == low.end()) continue;
      for (int32_t b : it->second) {
        int64_t olo[3], ohi[3];
        bool overlap = true;
        for (int e = 0; e < dim; ++e) {
          if (e == d) continue;
          olo[e] = std::max(box[(size_t)a][e], box[(size_t)b][e]);
          ohi[e] = std::min(box[(size_t)a][3 + e], box[(size_t)b][3 + e]);
          overlap = overlap && ohi[e] > olo[e];
        }
        if (!overlap) continue;
        if (fa) {
          fa[cnt] = (int32_t)a;
          fb[cnt] = b;
          fdir[cnt] = d;
          int t = 0;
          for (int e = 0; e < dim; ++e) {
            if (e == d) continue;
            const double sa = (double)(box[(size_t)a][3 + e] - box[(size_t)a][e]);
            const double sb = (double)(box[(size_t)b][3 + e] - box[(size_t)b][e]);
            rect_a[cnt * 4 + 2 * t] = (double)(olo[e] - box[(size_t)a][e]) / sa;
            rect_a[cnt * 4 + 2 * t + 1] = (double)(ohi[e] - box[(size_t)a][e]) / sa;
            rect_b[cnt * 4 + 2 * t] = (double)(olo[e] - box[(size_t)b][e]) / sb;
            rect_b[cnt * 4 + 2 * t + 1] = (double)(ohi[e] - box[(size_t)b][e]) / sb;
            ++t;
          }
          for (; t < 2; ++t) {
            rect_a[cnt * 4 + 2 * t] = rect_b[cnt * 4 + 2 * t] = 0.0;
            rect_a[cnt * 4 + 2 * t + 1] = rect_b[cnt * 4 + 2 * t + 1] = 1.0;
          }
        }
        ++cnt;
      }
    }
  *n_faces = cnt;
  return GLS_OK;
}

// Level meshes of a multigrid on the refinement hierarchy (global coarsening): the forest with every leaf
// finer than `level` replaced by its ancestor on `level`. Truncation keeps the vertex 2:1 balance (two
// truncated leaves that touch have ancestors-or-selves that touched, whose levels differed by <= 1).
int gls_octree_coarsen_to(const gls_octree *t, int level, gls_octree **out) {
  if (!t || !out || level < 0) return gls_io_set_error(GLS_EINVAL, "gls_octree_coarsen_to: bad arguments");
  auto r = std::make_unique<gls_octree>(*t);
  r->leaves.clear();
  std::map<std::array<int64_t, 4>, char> seen;
  for (const Leaf &c : t->leaves) {
    Leaf a = c;
    if (a.level > level) {
      for (int d = 0; d < t->dim; ++d) a.x[d] >>= (a.level - level);
      a.level = level;
    }
    if (seen.emplace(std::array<int64_t, 4>{a.level, a.x[0], a.x[1], a.x[2]}, 1).second) r->leaves.push_back(a);
  }
  sort_leaves(*r);
  *out = r.release();
  return GLS_OK;
}

// Grid transfer between two nested octree meshes of the same cube (coarse = a coarsening of fine, e.g.
// gls_octree_coarsen_to): the prolongation P as a DoF-level CSR over the fine DoFs ([velocity node-major |
// pressure]), fine DoF i = sum_j P_ij coarse DoF j -- the coarse FE field (its hanging nodes replaced by
// their lines, so a conforming field) evaluated at the fine node: the Qk interpolant of the coarse cell
// holding it, in exact lattice arithmetic. Rows of fine hanging DoFs are empty (their values follow from
// the fine lines); columns are coarse masters only. inject[j] = the fine DoF at coarse DoF j's position
// (the state injection of the coarse levels). Call with off == NULL for nnz only. Non-periodic meshes.
int gls_octree_mg_transfer(const gls_refined_mesh *fm, const gls_refined_mesh *cm, int64_t *nnz, int64_t *off,
                           int32_t *col, double *w, int64_t *inject) {
  if (!fm || !cm || !nnz || fm->dim != cm->dim || fm->k != cm->k || fm->kp != cm->kp)
    return gls_io_set_error(GLS_EINVAL, "gls_octree_mg_transfer: incompatible meshes");
  const MeshImpl *F = static_cast<const MeshImpl *>(fm->impl_), *Cm = static_cast<const MeshImpl *>(cm->impl_);
  // nested: the coarse mesh's finest cells are unions of the fine mesh's finest cells (the two forests may
  // have different level-0 grids, e.g. a uniform level below an adapted forest's base)
  const int64_t Nf = (int64_t)F->n << F->L, Nc = (int64_t)Cm->n << Cm->L;  // finest cells per direction
  if (F->lo != Cm->lo || F->hi != Cm->hi || F->pmask || Cm->pmask || Nf % Nc != 0)
    return gls_io_set_error(GLS_EINVAL, "gls_octree_mg_transfer: not nested meshes of one cube (or periodic)");
  const int dim = fm->dim;
  int64_t tot = 1;
  for (int d = 0; d < dim; ++d) tot *= Nc;
  if (tot > ((int64_t)1 << 28)) return gls_io_set_error(GLS_EINVAL, "gls_octree_mg_transfer: grid too large");
  const double hff = (F->hi - F->lo) / ((double)F->n * (double)((int64_t)1 << F->L));  // fine-finest cell
  std::vector<int64_t> rows_v, rows_p;                                                  // per space
  std::vector<int32_t> cols_acc;
  std::vector<double> w_acc;
  std::vector<int64_t> row_off{0};
  const int64_t nvf = fm->n_vnodes, nvc = cm->n_vnodes;
  std::vector<int64_t> inj((size_t)(dim * nvc + cm->n_pnodes), -1);
  for (int sp = 0; sp < 2; ++sp) {
    const bool vel = sp == 0;
    const int kk = vel ? fm->k : fm->kp, K1 = kk + 1;
    int npc = 1;
    for (int d = 0; d < dim; ++d) npc *= K1;
    const double u = hff / kk;                                    // fine lattice spacing of this space
    const int64_t sc = (int64_t)kk * (Nf / Nc);                    // coarse-finest cell in lattice units
    auto lattice = [&](const double *x, int64_t *p) {
      for (int d = 0; d < dim; ++d) p[d] = (int64_t)std::llround((x[d] - F->lo) / u);
    };
    // coarse cells: integer boxes, owner grid at the coarse-finest resolution
    std::vector<int32_t> owner((size_t)tot, -1);
    std::vector<std::array<int64_t, 4>> cbox((size_t)cm->n_cells);  // origin[3], size
    for (int64_t c = 0; c < cm->n_cells; ++c) {
      int64_t o[3] = {0, 0, 0};
      lattice(cm->cell_x0 + c * dim, o);
      const int64_t S = (int64_t)std::llround(cm->cell_h[c * dim] / u);
      cbox[(size_t)c] = {o[0], o[1], o[2], S};
      const int64_t s = S / sc;
      int64_t nb = 1;
      for (int d = 0; d < dim; ++d) nb *= s;
      for (int64_t b = 0; b < nb; ++b) {
        int64_t r = b, id = 0, st = 1;
        for (int d = 0; d < dim; ++d) {
          id += (o[d] / sc + r % s) * st;
          r /= s;
          st *= Nc;
        }
        owner[(size_t)id] = (int32_t)c;
      }
    }
    // hanging lines (node level) of both meshes
    const int64_t nh_c = vel ? cm->n_vhang : cm->n_phang, nh_f = vel ? fm->n_vhang : fm->n_phang;
    const int64_t *hc_node = vel ? cm->vhang_node : cm->phang_node, *hc_off = vel ? cm->vhang_off : cm->phang_off;
    const int64_t *hc_mas = vel ? cm->vhang_master : cm->phang_master;
    const double *hc_w = vel ? cm->vhang_w : cm->phang_w;
    const int64_t *hf_node = vel ? fm->vhang_node : fm->phang_node;
    std::unordered_map<int64_t, int64_t> cline;  // coarse hanging node -> line index
    for (int64_t i = 0; i < nh_c; ++i) cline[hc_node[i]] = i;
    const int64_t nnf = vel ? nvf : fm->n_pnodes, nnc = vel ? nvc : cm->n_pnodes;
    std::vector<char> fhang((size_t)nnf, 0);
    for (int64_t i = 0; i < nh_f; ++i) fhang[(size_t)hf_node[i]] = 1;
    const double *fx = vel ? fm->vnode_x : fm->pnode_x, *cx = vel ? cm->vnode_x : cm->pnode_x;
    const int32_t *cnodes = vel ? cm->cell_vnodes : cm->cell_pnodes;
    // fine lattice position -> fine node (injection)
    std::unordered_map<int64_t, int64_t> fpos;
    fpos.reserve((size_t)nnf);
    const int64_t span = kk * ((int64_t)F->n << F->L) + 1;
    auto key = [&](const int64_t *p) {
      int64_t k = 0, st = 1;
      for (int d = 0; d < dim; ++d) {
        k += p[d] * st;
        st *= span;
      }
      return k;
    };
    for (int64_t v = 0; v < nnf; ++v) {
      int64_t p[3] = {0, 0, 0};
      lattice(fx + v * dim, p);
      fpos[key(p)] = v;
    }
    for (int64_t j = 0; j < nnc; ++j) {
      int64_t p[3] = {0, 0, 0};
      lattice(cx + j * dim, p);
      auto it = fpos.find(key(p));
      if (it == fpos.end()) return gls_io_set_error(GLS_EINVAL, "gls_octree_mg_transfer: coarse node %lld not a fine node",
                                                    (long long)j);
      if (vel)
        for (int c = 0; c < dim; ++c) inj[(size_t)(j * dim + c)] = it->second * dim + c;
      else
        inj[(size_t)(dim * nvc + j)] = dim * nvf + it->second;
    }
    std::vector<std::pair<int32_t, double>> acc;
    for (int64_t v = 0; v < nnf; ++v) {
      acc.clear();
      if (!fhang[(size_t)v]) {
        int64_t p[3] = {0, 0, 0}, id = 0, st = 1;
        lattice(fx + v * dim, p);
        for (int d = 0; d < dim; ++d) {
          id += std::min(p[d] / sc, Nc - 1) * st;
          st *= Nc;
        }
        const int32_t c = owner[(size_t)id];
        if (c < 0) return gls_io_set_error(GLS_EINVAL, "gls_octree_mg_transfer: fine node outside the coarse mesh");
        const auto &B = cbox[(size_t)c];
        double xi[3] = {0, 0, 0};
        for (int d = 0; d < dim; ++d) xi[d] = (double)(p[d] - B[d]) / (double)B[3];
        for (int a = 0; a < npc; ++a) {
          double wa = 1.0;
          int r = a;
          for (int d = 0; d < dim; ++d) {
            wa *= lagrange(kk, r % K1, xi[d]);
            r /= K1;
          }
          if (std::fabs(wa) < 1e-14) continue;
          const int32_t cn = cnodes[(size_t)c * npc + a];
          auto it = cline.find(cn);
          if (it == cline.end()) {
            acc.push_back({cn, wa});
          } else {
            for (int64_t q = hc_off[it->second]; q < hc_off[it->second + 1]; ++q)
              acc.push_back({(int32_t)hc_mas[q], wa * hc_w[q]});
          }
        }
        std::sort(acc.begin(), acc.end(), [](const std::pair<int32_t, double> &x, const std::pair<int32_t, double> &y) {
          return x.first < y.first;
        });
        size_t m = 0;  // merge duplicate masters (fixed order: ascending node, then the order of the terms)
        for (size_t i = 0; i < acc.size(); ++i) {
          if (m > 0 && acc[m - 1].first == acc[i].first) acc[m - 1].second += acc[i].second;
          else acc[m++] = acc[i];
        }
        acc.resize(m);
        acc.erase(std::remove_if(acc.begin(), acc.end(), [](const std::pair<int32_t, double> &e) {
                    return std::fabs(e.second) < 1e-14;
                  }),
                  acc.end());
      }
      const int nrow = vel ? dim : 1;
      for (int c = 0; c < nrow; ++c) {
        for (auto &e : acc) {
          cols_acc.push_back(vel ? (int32_t)(e.first * dim + c) : (int32_t)(dim * nvc + e.first));
          w_acc.push_back(e.second);
        }
        row_off.push_back((int64_t)cols_acc.size());
      }
    }
  }
  *nnz = (int64_t)cols_acc.size();
  if (off) {
    if (!col || !w) return gls_io_set_error(GLS_EINVAL, "gls_octree_mg_transfer: col / w missing");
    std::memcpy(off, row_off.data(), sizeof(int64_t) * row_off.size());
    std::memcpy(col, cols_acc.data(), sizeof(int32_t) * cols_acc.size());
    std::memcpy(w, w_acc.data(), sizeof(double) * w_acc.size());
  }
  if (inject) std::memcpy(inject, inj.data(), sizeof(int64_t) * inj.size());
  return GLS_OK;
}

}  // extern "C"
