// gls_umesh.cpp — unstructured quadrilateral / hexahedral meshes with manifolds (host C++17).
//
// What the reference gets from deal.II for its non-box meshes:
//   * GridGenerator::generate_from_name_and_arguments (source/core/grids.cc:30-36): hyper_cube,
//     hyper_rectangle, subdivided_hyper_rectangle, hyper_shell (2D), cylinder (3D), and the
//     builder-defined cylinder_shell (the 3D Taylor-Couette geometry of BASELINE configs[3]);
//   * GridIn::read_msh (grids.cc:21-28): gmsh ASCII 2.2 / 4.0 / 4.1, physical tag (or the entity tag
//     when an entity has none) = boundary id of boundary elements;
//   * manifolds (source/core/manifolds.cc:226-247): SphericalManifold attached to boundary ids,
//     the generators' own spherical / cylindrical manifolds;
//   * Triangulation::refine_global (grids.cc:70-77) with deal.II 9.2's placement of new vertices:
//     line midpoints on the line's manifold, quad / hex centres from the transfinite-interpolation
//     (TFI) weights of their surrounding points on the object's manifold; children inherit manifold
//     and boundary ids;
//   * MappingQ(k, qmapping_all) support points (gls_navier_stokes.cc:245-246): Qk mapping on every
//     cell, or only on cells with a boundary line; the other cells are Q1, embedded exactly in the
//     same (k+1)^dim Lagrange support-point layout (Q1 is a subspace of Qk);
//   * FE_Q(k) / FE_Q(kp) node numbering for k <= 2 (one node per vertex, line, face, cell
//     interior), periodic node identification (make_periodicity_constraints as node identity).
// Cells are kept parent-major under refinement (children of cell c are 2^dim*c + child, child
// bits = lexicographic position), so a solution transfer needs no extra map.
#include <algorithm>
#include <array>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <functional>
#include <map>
#include <set>
#include <sstream>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/gls_native.h"

int gls_io_set_error(int code, const char *fmt, ...);  // gls_api.cpp

namespace {

using V3 = std::array<double, 3>;
enum { MF_FLAT = 0, MF_SPHERICAL = 1, MF_CYLINDRICAL = 2 };

struct ManifoldDesc {
  int type = MF_FLAT;
  V3 center{0, 0, 0};  // spherical centre / point on the cylinder axis
  V3 axis{0, 0, 1};    // cylinder axis (unit)
};

// sorted vertex ids of a line (2) or quad face (4); unused slots -1
struct EKey {
  int64_t v[4];
  bool operator<(const EKey &o) const {
    for (int i = 0; i < 4; ++i)
      if (v[i] != o.v[i]) return v[i] < o.v[i];
    return false;
  }
  bool operator==(const EKey &o) const { return std::memcmp(v, o.v, sizeof(v)) == 0; }
};
EKey mkey(std::initializer_list<int64_t> ids) {
  EKey k{{-1, -1, -1, -1}};
  int n = 0;
  for (int64_t i : ids) k.v[n++] = i;
  std::sort(k.v, k.v + n);
  return k;
}

V3 add(const V3 &a, const V3 &b) { return {a[0] + b[0], a[1] + b[1], a[2] + b[2]}; }
V3 sub(const V3 &a, const V3 &b) { return {a[0] - b[0], a[1] - b[1], a[2] - b[2]}; }
V3 scl(const V3 &a, double s) { return {a[0] * s, a[1] * s, a[2] * s}; }
double dot3(const V3 &a, const V3 &b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
double nrm(const V3 &a) { return std::sqrt(dot3(a, a)); }
V3 cross(const V3 &a, const V3 &b) {
  return {a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]};
}

struct UMesh {
  int dim = 2;
  std::vector<V3> X;
  std::vector<std::array<int64_t, 8>> cells;  // deal.II lexicographic vertex order (x fastest)
  std::vector<int> cell_mf;                   // manifold id per cell (-1 flat)
  std::map<EKey, int> bface;                  // boundary faces -> boundary id
  std::map<EKey, int> line_mf, face_mf;       // manifold ids of lines (and 3D quads)
  std::map<int, ManifoldDesc> mf;
  // refinement hierarchy (the triangulation's cells on every level): cells / cell_mf above are the
  // active cells, tree[active[i]] their hierarchy records. Records are never removed (coarsened
  // children stay as dead records), so hierarchy ids are stable across adaptations.
  struct HCell {
    std::array<int64_t, 8> v;
    int mf, level;
    int64_t parent;  // -1 on level 0
    int pos;         // child position in the parent (bit d: upper half in local direction d)
    int64_t child0;  // first of the 2^dim consecutive children, -1 when active
  };
  std::vector<HCell> tree;
  std::vector<int64_t> roots, active;
  std::map<EKey, int64_t> line_mid, face_mid;  // refined lines / quads -> their midpoint vertex
  // periodic boundary pairs (id a, id b, direction) of the triangulation (add_periodicity, grids.cc:41-58):
  // the mesh smoothing and the vertex 2:1 balance see across them
  std::vector<std::array<int, 3>> periodic;

  int nvc() const { return dim == 2 ? 4 : 8; }
  int mf_of(const std::map<EKey, int> &m, const EKey &k) const {
    auto it = m.find(k);
    return it == m.end() ? -1 : it->second;
  }
};

// ---- manifolds: new point from surrounding points and weights (deal.II 9.2 semantics)
V3 slerp_unit(const V3 &a, const V3 &b, double t) {  // geodesic between unit vectors
  const double c = std::max(-1.0, std::min(1.0, dot3(a, b)));
  const double th = std::acos(c);
  if (th < 1e-14) return a;
  const double s = std::sin(th);
  return add(scl(a, std::sin((1 - t) * th) / s), scl(b, std::sin(t * th) / s));
}

V3 new_point(const UMesh &m, int mfid, const std::vector<V3> &p, const std::vector<double> &w) {
  auto it = mfid < 0 ? m.mf.end() : m.mf.find(mfid);
  const int type = it == m.mf.end() ? MF_FLAT : it->second.type;
  V3 lin{0, 0, 0};
  for (size_t i = 0; i < p.size(); ++i) lin = add(lin, scl(p[i], w[i]));
  if (type == MF_FLAT) return lin;
  const ManifoldDesc &md = it->second;
  if (type == MF_SPHERICAL) {
    // SphericalManifold::get_new_points: radius = sum w_i |p_i - c|; direction: the geodesic
    // (slerp) for two points, else the normalised weighted sum of the unit directions (which is
    // deal.II's spherical mean for the symmetric stencils used here)
    double rho = 0;
    std::vector<V3> d(p.size());
    for (size_t i = 0; i < p.size(); ++i) {
      const V3 r = sub(p[i], md.center);
      const double n = nrm(r);
      rho += w[i] * n;
      d[i] = n > 0 ? scl(r, 1.0 / n) : V3{0, 0, 0};
    }
    V3 dir;
    if (p.size() == 2) {
      dir = slerp_unit(d[0], d[1], w[1]);
    } else {
      dir = {0, 0, 0};
      for (size_t i = 0; i < p.size(); ++i) dir = add(dir, scl(d[i], w[i]));
      const double n = nrm(dir);
      if (n == 0) return md.center;
      dir = scl(dir, 1.0 / n);
    }
    if (m.dim == 2) dir[2] = 0;
    return add(md.center, scl(dir, rho));
  }
  // CylindricalManifold::get_new_point: a weighted average lying on the axis stays there; else the
  // ChartManifold average in (r, phi, z) with phi periodic (FlatManifold periodicity rule)
  const V3 a = md.axis;
  double avg_len = 0;
  for (size_t i = 0; i < p.size(); ++i) avg_len += w[i] * dot3(p[i], p[i]);
  const V3 mid = sub(lin, md.center);
  const double lam = dot3(mid, a);
  const V3 off = sub(mid, scl(a, lam));
  if (dot3(off, off) < 1e-10 * std::fabs(avg_len)) return add(md.center, scl(a, lam));
  V3 e1 = std::fabs(a[0]) < 0.9 ? cross(a, V3{1, 0, 0}) : cross(a, V3{0, 1, 0});
  e1 = scl(e1, 1.0 / nrm(e1));
  const V3 e2 = cross(a, e1);
  std::vector<V3> ch(p.size());
  double minphi = 2 * M_PI;
  for (size_t i = 0; i < p.size(); ++i) {
    const V3 r = sub(p[i], md.center);
    const double z = dot3(r, a);
    const V3 rad = sub(r, scl(a, z));
    ch[i] = {nrm(rad), std::atan2(dot3(rad, e2), dot3(rad, e1)), z};
    minphi = std::min(minphi, ch[i][1]);
  }
  V3 c{0, 0, 0};
  for (size_t i = 0; i < p.size(); ++i) {
    V3 q = ch[i];
    if (q[1] - minphi > M_PI) q[1] -= 2 * M_PI;
    c = add(c, scl(q, w[i]));
  }
  return add(md.center, add(scl(a, c[2]), scl(add(scl(e1, std::cos(c[1])), scl(e2, std::sin(c[1]))), c[0])));
}

// ---- local topology (lexicographic vertex index v = x + 2y + 4z)
// lines: vertex pairs differing in one bit; 3D faces: the 4 vertices with bit d == s
std::vector<std::array<int, 2>> local_lines(int dim) {
  std::vector<std::array<int, 2>> L;
  const int nv = 1 << dim;
  for (int d = 0; d < dim; ++d)
    for (int v = 0; v < nv; ++v)
      if (!((v >> d) & 1)) L.push_back({v, v | (1 << d)});
  return L;
}
std::array<int, 4> face_verts(int dim, int d, int s) {
  std::array<int, 4> f{-1, -1, -1, -1};
  int n = 0;
  for (int v = 0; v < (1 << dim); ++v)
    if (((v >> d) & 1) == s) f[n++] = v;
  return f;
}
EKey face_key(const UMesh &m, size_t c, int d, int s) {
  const auto fv = face_verts(m.dim, d, s);
  const auto &cv = m.cells[c];
  return m.dim == 2 ? mkey({cv[fv[0]], cv[fv[1]]}) : mkey({cv[fv[0]], cv[fv[1]], cv[fv[2]], cv[fv[3]]});
}

// boundary faces = faces of exactly one cell; ids from `idfun` (face centre -> id) or 0
template <class F>
void mark_boundary(UMesh &m, F idfun) {
  std::map<EKey, int> cnt;
  for (size_t c = 0; c < m.cells.size(); ++c)
    for (int d = 0; d < m.dim; ++d)
      for (int s = 0; s < 2; ++s) ++cnt[face_key(m, c, d, s)];
  m.bface.clear();
  for (auto &kv : cnt)
    if (kv.second == 1) {
      V3 ctr{0, 0, 0};
      const int n = m.dim == 2 ? 2 : 4;
      for (int i = 0; i < n; ++i) ctr = add(ctr, scl(m.X[(size_t)kv.first.v[i]], 1.0 / n));
      m.bface[kv.first] = idfun(ctr);
    }
}

// signed Jacobian determinant of the multilinear map at the cell centre
double center_det(const UMesh &m, const std::array<int64_t, 8> &cv) {
  double J[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
  const int nv = m.nvc();
  for (int v = 0; v < nv; ++v)
    for (int a = 0; a < m.dim; ++a) {
      double g = ((v >> a) & 1) ? 1.0 : -1.0;
      for (int b = 0; b < m.dim; ++b)
        if (b != a) g *= 0.5;
      for (int i = 0; i < m.dim; ++i) J[i][a] += g * m.X[(size_t)cv[v]][i];
    }
  if (m.dim == 2) return J[0][0] * J[1][1] - J[0][1] * J[1][0];
  return J[0][0] * (J[1][1] * J[2][2] - J[1][2] * J[2][1]) - J[0][1] * (J[1][0] * J[2][2] - J[1][2] * J[2][0]) +
         J[0][2] * (J[1][0] * J[2][1] - J[1][1] * J[2][0]);
}
// deal.II keeps every cell positively oriented (GridReordering / invert_all_cells_of_negative_grid):
// mirror the local x direction of inverted cells (the Qk space and Gauss rules are invariant)
void orient(UMesh &m) {
  for (auto &cv : m.cells)
    if (center_det(m, cv) < 0)
      for (int v = 0; v < m.nvc(); v += 2) std::swap(cv[v], cv[v + 1]);
}

// ---- refinement (Triangulation::refine_global / execute_coarsening_and_refinement, deal.II 9.2
// vertex placement)
EKey face_key_v(int dim, const std::array<int64_t, 8> &cv, int d, int s) {
  const auto fv = face_verts(dim, d, s);
  return dim == 2 ? mkey({cv[fv[0]], cv[fv[1]]}) : mkey({cv[fv[0]], cv[fv[1]], cv[fv[2]], cv[fv[3]]});
}

// the level-0 records of the hierarchy (once, after the coarse mesh is complete)
void init_tree(UMesh &m) {
  if (!m.tree.empty()) return;
  for (size_t c = 0; c < m.cells.size(); ++c) {
    m.tree.push_back({m.cells[c], m.cell_mf[c], 0, -1, 0, -1});
    m.roots.push_back((int64_t)c);
  }
  m.active = m.roots;
}

// active cells in depth-first order (children in lexicographic position order inside their parent):
// after a global refinement, the children of active cell c are 2^dim c + child
void sync_active(UMesh &m) {
  m.active.clear();
  std::vector<int64_t> st;
  for (auto r = m.roots.rbegin(); r != m.roots.rend(); ++r) st.push_back(*r);
  const int nch = 1 << m.dim;
  while (!st.empty()) {
    const int64_t id = st.back();
    st.pop_back();
    const auto &h = m.tree[(size_t)id];
    if (h.child0 < 0) {
      m.active.push_back(id);
      continue;
    }
    for (int ch = nch - 1; ch >= 0; --ch) st.push_back(h.child0 + ch);
  }
  m.cells.resize(m.active.size());
  m.cell_mf.resize(m.active.size());
  for (size_t i = 0; i < m.active.size(); ++i) {
    m.cells[i] = m.tree[(size_t)m.active[i]].v;
    m.cell_mf[i] = m.tree[(size_t)m.active[i]].mf;
  }
}

// split hierarchy cell `id` into 2^dim children: line midpoints on the line's manifold, quad / hex
// centres from the TFI weights; children inherit manifold and boundary ids of the parent object
// they lie in. Midpoints are shared through m.line_mid / m.face_mid across cells and adaptations.
void refine_cell(UMesh &m, int64_t id) {
  const int dim = m.dim, nv = m.nvc(), nch = 1 << dim;
  const auto lines = local_lines(dim);
  const std::array<int64_t, 8> cv = m.tree[(size_t)id].v;
  const int cellmf = m.tree[(size_t)id].mf;
  // lattice of 3^dim points: index (i, j, l) in {0,1,2}
  int64_t lat[27];
  auto L = [&](int i, int j, int l) -> int64_t & { return lat[i + 3 * (j + 3 * l)]; };
  for (int v = 0; v < nv; ++v) L(2 * (v & 1), 2 * ((v >> 1) & 1), 2 * ((v >> 2) & 1)) = cv[v];
  // line midpoints
  std::vector<V3> lmid(lines.size());
  for (size_t li = 0; li < lines.size(); ++li) {
    const int a = lines[li][0], b = lines[li][1];
    const EKey k = mkey({cv[a], cv[b]});
    auto it = m.line_mid.find(k);
    int64_t vid;
    if (it == m.line_mid.end()) {
      const V3 p = new_point(m, m.mf_of(m.line_mf, k), {m.X[(size_t)cv[a]], m.X[(size_t)cv[b]]}, {0.5, 0.5});
      vid = (int64_t)m.X.size();
      m.X.push_back(p);
      m.line_mid[k] = vid;
    } else {
      vid = it->second;
    }
    lmid[li] = m.X[(size_t)vid];
    int q[3];  // lattice: coordinate 1 along the line's direction
    for (int d = 0; d < 3; ++d) q[d] = ((a >> d) & 1) == ((b >> d) & 1) ? 2 * ((a >> d) & 1) : 1;
    L(q[0], q[1], dim > 2 ? q[2] : 0) = vid;
  }
  auto quad_center = [&](int mfid, const std::array<int, 4> &fv) {  // TFI: vertices -1/4, lines +1/2
    std::vector<V3> p;
    std::vector<double> w;
    for (int i = 0; i < 4; ++i) {
      p.push_back(m.X[(size_t)cv[fv[i]]]);
      w.push_back(-0.25);
    }
    for (size_t li = 0; li < lines.size(); ++li) {
      const int a = lines[li][0], b = lines[li][1];
      if (std::find(fv.begin(), fv.end(), a) != fv.end() && std::find(fv.begin(), fv.end(), b) != fv.end()) {
        p.push_back(lmid[li]);
        w.push_back(0.5);
      }
    }
    return new_point(m, mfid, p, w);
  };
  if (dim == 3) {
    std::vector<V3> fmid;
    for (int d = 0; d < 3; ++d)
      for (int s = 0; s < 2; ++s) {
        const EKey k = face_key_v(3, cv, d, s);
        auto it = m.face_mid.find(k);
        int64_t vid;
        if (it == m.face_mid.end()) {
          const V3 p = quad_center(m.mf_of(m.face_mf, k), face_verts(3, d, s));
          vid = (int64_t)m.X.size();
          m.X.push_back(p);
          m.face_mid[k] = vid;
        } else {
          vid = it->second;
        }
        fmid.push_back(m.X[(size_t)vid]);
        int q[3] = {1, 1, 1};
        q[d] = 2 * s;
        L(q[0], q[1], q[2]) = vid;
      }
    // hex centre: TFI weights vertices +1/8, lines -1/4, faces +1/2
    std::vector<V3> p;
    std::vector<double> w;
    for (int v = 0; v < 8; ++v) { p.push_back(m.X[(size_t)cv[v]]); w.push_back(0.125); }
    for (auto &x : lmid) { p.push_back(x); w.push_back(-0.25); }
    for (auto &x : fmid) { p.push_back(x); w.push_back(0.5); }
    L(1, 1, 1) = (int64_t)m.X.size();
    m.X.push_back(new_point(m, cellmf, p, w));
  } else {
    L(1, 1, 0) = (int64_t)m.X.size();
    m.X.push_back(quad_center(cellmf, {0, 1, 2, 3}));
  }
  // children (lexicographic child position)
  const int64_t child0 = (int64_t)m.tree.size();
  for (int ch = 0; ch < nch; ++ch) {
    const int cx = ch & 1, cy = (ch >> 1) & 1, cz = (ch >> 2) & 1;
    std::array<int64_t, 8> nc{};
    for (int v = 0; v < nv; ++v) nc[v] = L(cx + (v & 1), cy + ((v >> 1) & 1), dim == 3 ? cz + ((v >> 2) & 1) : 0);
    m.tree.push_back({nc, cellmf, m.tree[(size_t)id].level + 1, id, ch, -1});
    // manifold / boundary ids of the child's lines and faces: inherited from the parent object
    // they lie in (parent line, parent face, or the parent cell's interior)
    for (auto &ln : lines) {
      int pa[3], pb[3];
      for (int d = 0; d < 3; ++d) {
        pa[d] = (d == 0 ? cx : d == 1 ? cy : cz) + ((ln[0] >> d) & 1);
        pb[d] = (d == 0 ? cx : d == 1 ? cy : cz) + ((ln[1] >> d) & 1);
      }
      int dir = 0;
      for (int d = 0; d < dim; ++d)
        if (pa[d] != pb[d]) dir = d;
      int nend = 0, ends[3], endd[3];
      for (int d = 0; d < dim; ++d)
        if (d != dir && (pa[d] == 0 || pa[d] == 2)) { ends[nend] = pa[d]; endd[nend++] = d; }
      int mfv;
      if (nend == dim - 1) {  // on a parent line
        int va = 0, vb = 0;
        for (int d = 0; d < dim; ++d)
          if (d != dir) { va |= (pa[d] / 2) << d; vb |= (pa[d] / 2) << d; }
        vb |= 1 << dir;
        mfv = m.mf_of(m.line_mf, mkey({cv[va], cv[vb]}));
      } else if (dim == 3 && nend == 1) {  // inside a parent face
        mfv = m.mf_of(m.face_mf, face_key_v(3, cv, endd[0], ends[0] / 2));
      } else {
        mfv = cellmf;
      }
      if (mfv >= 0) m.line_mf[mkey({nc[ln[0]], nc[ln[1]]})] = mfv;
    }
    for (int d = 0; d < dim; ++d)
      for (int s = 0; s < 2; ++s) {
        const int pc = (d == 0 ? cx : d == 1 ? cy : cz) + s;  // parent-lattice coordinate of the face
        const EKey k = face_key_v(dim, nc, d, s);
        if (pc == 0 || pc == 2) {
          const EKey pk = face_key_v(dim, cv, d, pc / 2);
          auto b = m.bface.find(pk);
          if (b != m.bface.end()) m.bface[k] = b->second;
          if (dim == 3) {
            const int f = m.mf_of(m.face_mf, pk);
            if (f >= 0) m.face_mf[k] = f;
          }
        } else if (dim == 3 && cellmf >= 0) {
          m.face_mf[k] = cellmf;
        }
      }
  }
  m.tree[(size_t)id].child0 = child0;
}

// refine_global(1): every active cell. Object maps keep the entries of the parent objects (keys are
// vertex sets, so an object of any level keeps its own boundary / manifold id).
int refine_once(UMesh &m) {
  init_tree(m);
  const std::vector<int64_t> act = m.active;
  for (int64_t id : act) refine_cell(m, id);
  sync_active(m);
  return GLS_OK;
}

// ---- local adaptation of the hierarchy (the reference's p::d::Triangulation with
// smoothing_on_refinement | smoothing_on_coarsening, navier_stokes_base.cc:55-60, 592-780)

// ---- periodicity under local refinement (add_periodicity, grids.cc:41-58; make_periodicity_constraints,
// gls_navier_stokes.cc:128-134, 162-168): per pair (id a, id b, direction d) the vertices of the boundary
// faces with id b are matched onto those of id a by the translation along d (every other coordinate
// equal). A vertex without a partner lies on a face finer than the one across the periodic boundary.
// `rep` joins matched vertices into classes (smallest id) for the level rules of the smoothing / balance.
struct PeriodicVerts {
  std::vector<std::array<int, 3>> pairs;
  std::vector<std::map<int64_t, int64_t>> b2a, a2b;  // per pair
  std::vector<int64_t> rep;
  bool on() const { return !pairs.empty(); }
  int64_t cls(int64_t v) const { return rep.empty() ? v : rep[(size_t)v]; }
};
double periodic_tol(const std::vector<V3> &X) {
  double scale = 0;
  for (auto &x : X) scale = std::max(scale, std::fabs(x[0]) + std::fabs(x[1]) + std::fabs(x[2]));
  return 1e-8 * std::max(scale, 1e-300);
}
PeriodicVerts periodic_vertices(const UMesh &m, const std::vector<std::array<int, 3>> &pairs) {
  PeriodicVerts P;
  if (pairs.empty()) return P;
  P.pairs = pairs;
  const double tol = periodic_tol(m.X);
  P.rep.resize(m.X.size());
  for (size_t i = 0; i < P.rep.size(); ++i) P.rep[i] = (int64_t)i;
  std::function<int64_t(int64_t)> root = [&](int64_t v) {
    while (P.rep[(size_t)v] != v) v = P.rep[(size_t)v] = P.rep[(size_t)P.rep[(size_t)v]];
    return v;
  };
  for (const auto &pr : pairs) {
    std::set<int64_t> A, B;
    for (const auto &kv : m.bface) {
      if (kv.second != pr[0] && kv.second != pr[1]) continue;
      for (int i = 0; i < 4; ++i)
        if (kv.first.v[i] >= 0) (kv.second == pr[0] ? A : B).insert(kv.first.v[i]);
    }
    const int o1 = (pr[2] + 1) % 3, o2 = (pr[2] + 2) % 3;
    auto cellk = [&](const V3 &x) {
      return std::array<long long, 2>{std::llround(x[o1] / (100 * tol)), std::llround(x[o2] / (100 * tol))};
    };
    std::map<std::array<long long, 2>, std::vector<int64_t>> grid;
    for (int64_t i : A) grid[cellk(m.X[(size_t)i])].push_back(i);
    std::map<int64_t, int64_t> b2a, a2b;
    for (int64_t j : B) {
      const auto ck = cellk(m.X[(size_t)j]);
      int64_t match = -1;
      for (long long dx = -1; dx <= 1 && match < 0; ++dx)
        for (long long dy = -1; dy <= 1 && match < 0; ++dy) {
          auto g = grid.find({ck[0] + dx, ck[1] + dy});
          if (g == grid.end()) continue;
          for (int64_t i : g->second)
            if (i != j && std::fabs(m.X[(size_t)i][o1] - m.X[(size_t)j][o1]) < tol &&
                std::fabs(m.X[(size_t)i][o2] - m.X[(size_t)j][o2]) < tol) {
              match = i;
              break;
            }
        }
      if (match < 0) continue;
      b2a[j] = match;
      a2b[match] = j;
      const int64_t ra = root(match), rb = root(j);
      if (ra != rb) P.rep[(size_t)std::max(ra, rb)] = std::min(ra, rb);
    }
    P.b2a.push_back(std::move(b2a));
    P.a2b.push_back(std::move(a2b));
  }
  for (size_t i = 0; i < P.rep.size(); ++i) P.rep[i] = root((int64_t)i);
  return P;
}
// the face across the periodic boundary with the same vertices (translated); false when `key` is not a
// periodic boundary face or its translate is not a face of vertices that exist
bool periodic_partner(const UMesh &m, const PeriodicVerts &P, const EKey &key, EKey &out) {
  if (!P.on()) return false;
  auto b = m.bface.find(key);
  if (b == m.bface.end()) return false;
  for (size_t p = 0; p < P.pairs.size(); ++p) {
    const bool onA = b->second == P.pairs[p][0], onB = b->second == P.pairs[p][1];
    if (!onA && !onB) continue;
    const auto &mp = onA ? P.a2b[p] : P.b2a[p];
    EKey k{{-1, -1, -1, -1}};
    int n = 0;
    bool ok = true;
    for (int i = 0; i < 4 && ok; ++i) {
      if (key.v[i] < 0) continue;
      auto it = mp.find(key.v[i]);
      if (it == mp.end()) ok = false;
      else k.v[n++] = it->second;
    }
    if (!ok) continue;
    std::sort(k.v, k.v + n);
    out = k;
    return true;
  }
  return false;
}

// highest active level at every vertex (periodic partners share it)
std::vector<int> vertex_levels(const UMesh &m) {
  std::vector<int> vl(m.X.size(), -1);
  for (int64_t id : m.active) {
    const auto &h = m.tree[(size_t)id];
    for (int v = 0; v < m.nvc(); ++v) vl[(size_t)h.v[v]] = std::max(vl[(size_t)h.v[v]], h.level);
  }
  if (!m.periodic.empty()) {
    const PeriodicVerts P = periodic_vertices(m, m.periodic);
    for (size_t v = 0; v < vl.size(); ++v) vl[(size_t)P.cls((int64_t)v)] = std::max(vl[(size_t)P.cls((int64_t)v)], vl[v]);
    for (size_t v = 0; v < vl.size(); ++v) vl[v] = vl[(size_t)P.cls((int64_t)v)];
  }
  return vl;
}

// 2:1 balance over vertices (p4est corner balance): refine every active cell that shares a vertex
// with an active cell two or more levels finer, until none does
void balance(UMesh &m) {
  for (int it = 0; it < 64; ++it) {
    const std::vector<int> vl = vertex_levels(m);
    std::vector<int64_t> todo;
    for (int64_t id : m.active) {
      const auto &h = m.tree[(size_t)id];
      for (int v = 0; v < m.nvc(); ++v)
        if (vl[(size_t)h.v[v]] >= h.level + 2) { todo.push_back(id); break; }
    }
    if (todo.empty()) return;
    for (int64_t id : todo) refine_cell(m, id);
    sync_active(m);
  }
}

// the vertices on the closed boundary of hierarchy cell `id` at its children's resolution: corners,
// line midpoints and (3D) face centres that exist
std::vector<int64_t> boundary_half_lattice(const UMesh &m, int64_t id) {
  const auto &h = m.tree[(size_t)id];
  std::vector<int64_t> out(h.v.begin(), h.v.begin() + m.nvc());
  for (auto &ln : local_lines(m.dim)) {
    auto it = m.line_mid.find(mkey({h.v[ln[0]], h.v[ln[1]]}));
    if (it != m.line_mid.end()) out.push_back(it->second);
  }
  if (m.dim == 3)
    for (int d = 0; d < 3; ++d)
      for (int s = 0; s < 2; ++s) {
        auto it = m.face_mid.find(face_key_v(3, h.v, d, s));
        if (it != m.face_mid.end()) out.push_back(it->second);
      }
  return out;
}

// execute_coarsening_and_refinement: flagged active cells are refined, complete sibling families
// whose members are all flagged for coarsening (none for refinement) are coarsened unless a cell
// two levels finer than the parent touches its boundary after the refinement and balance pass;
// then the vertex balance is restored by refinement
int adapt(UMesh &m, const int32_t *ref, const int32_t *crs) {
  init_tree(m);
  const size_t na = m.active.size();
  const int nch = 1 << m.dim;
  std::map<int64_t, int> fam;  // parent -> flagged children
  for (size_t i = 0; i < na; ++i) {
    const auto &h = m.tree[(size_t)m.active[i]];
    if (crs && crs[i] && !(ref && ref[i]) && h.parent >= 0) ++fam[h.parent];
  }
  const std::vector<int64_t> act = m.active;
  for (size_t i = 0; i < na; ++i)
    if (ref && ref[i]) refine_cell(m, act[i]);
  sync_active(m);
  balance(m);
  const std::vector<int> vl = vertex_levels(m);
  std::vector<int64_t> drop;
  for (auto &kv : fam) {
    if (kv.second != nch) continue;
    const auto &p = m.tree[(size_t)kv.first];
    bool ok = true;
    for (int ch = 0; ch < nch && ok; ++ch) ok = m.tree[(size_t)(p.child0 + ch)].child0 < 0;
    for (int64_t v : boundary_half_lattice(m, kv.first)) ok = ok && vl[(size_t)v] <= p.level + 1;
    if (ok) drop.push_back(kv.first);
  }
  for (int64_t id : drop) m.tree[(size_t)id].child0 = -1;
  sync_active(m);
  balance(m);
  return GLS_OK;
}

// Triangulation::prepare_coarsening_and_refinement (deal.II 9.2 source/grid/tria.cc, third party,
// not vendored: restated from its published algorithm) with the reference's MeshSmoothing
// smoothing_on_refinement | smoothing_on_coarsening (navier_stokes_base.cc:55-60, called at :682),
// on the unstructured hierarchy. The same steps as gls_octree_prepare (gls_octree.cpp), with
// neighbours found through shared face vertex sets instead of a lattice: cells on each level in
// hierarchy order (coarse cells, then children of the previous level's refined cells), active cells
// visited in reverse; isotropic refinement only.
struct USmoother {
  const UMesh &m;
  int dim;
  std::vector<char> ref, crs;                   // per active cell
  std::unordered_map<int64_t, int64_t> leaf;    // hierarchy id -> active index
  std::vector<int64_t> all;                     // live cells, level by level
  std::vector<int64_t> active_rev;              // active indices, reverse level order
  std::map<EKey, std::vector<int64_t>> faces;   // face vertex set -> live cells having that face
  std::unordered_map<int64_t, char> user;       // refined cells to be coarsened (fix_coarsen_flags)
  PeriodicVerts pv;                             // faces across periodic boundaries are neighbours

  USmoother(const UMesh &mesh, const int32_t *r, const int32_t *c)
      : m(mesh), dim(mesh.dim), pv(periodic_vertices(mesh, mesh.periodic)) {
    const size_t na = m.active.size();
    ref.resize(na);
    crs.resize(na);
    for (size_t i = 0; i < na; ++i) {
      ref[i] = r[i] != 0;
      crs[i] = c[i] != 0;
      leaf[m.active[i]] = (int64_t)i;
    }
    std::vector<int64_t> lev = m.roots;
    while (!lev.empty()) {
      std::vector<int64_t> next;
      for (int64_t id : lev) {
        all.push_back(id);
        const auto &h = m.tree[(size_t)id];
        for (int d = 0; d < dim; ++d)
          for (int s = 0; s < 2; ++s) faces[face_key_v(dim, h.v, d, s)].push_back(id);
        if (h.child0 >= 0)
          for (int ch = 0; ch < (1 << dim); ++ch) next.push_back(h.child0 + ch);
      }
      lev.swap(next);
    }
    for (size_t j = all.size(); j-- > 0;) {
      auto it = leaf.find(all[j]);
      if (it != leaf.end()) active_rev.push_back(it->second);
    }
  }
  bool is_active(int64_t id) const { return m.tree[(size_t)id].child0 < 0; }
  int64_t kid(int64_t id, int ch) const { return m.tree[(size_t)id].child0 + ch; }
  int nkids() const { return 1 << dim; }
  // cell->neighbor(f): the live cell of the same level across face f (active or refined), else the
  // coarser active cell; returns 0 at the boundary, 1 same level, 2 coarser
  int neighbor(int64_t id, int f, int64_t &nb) const {
    const auto &h = m.tree[(size_t)id];
    const int d = f / 2, s = f & 1;
    const EKey key = face_key_v(dim, h.v, d, s);
    auto it = faces.find(key);
    if (it != faces.end())
      for (int64_t o : it->second)
        if (o != id) { nb = o; return 1; }
    EKey pk;  // across a periodic boundary: the live cell of this level on the translated face
    if (periodic_partner(m, pv, key, pk)) {
      auto jt = faces.find(pk);
      if (jt != faces.end() && !jt->second.empty()) { nb = jt->second[0]; return 1; }
    }
    if (h.parent < 0 || ((h.pos >> d) & 1) != s) return 0;  // boundary (a child's inner face is shared)
    int64_t pn;
    if (neighbor(h.parent, f, pn) != 1) return 0;
    nb = pn;
    return 2;
  }
  bool will_be_coarsened(int64_t id) {
    if (is_active(id)) return false;
    int n = 0;
    for (int ch = 0; ch < nkids(); ++ch) {
      auto it = leaf.find(kid(id, ch));
      if (it != leaf.end() && crs[(size_t)it->second]) ++n;
    }
    if (n == nkids()) return true;
    for (int ch = 0; ch < nkids(); ++ch) {
      auto it = leaf.find(kid(id, ch));
      if (it != leaf.end()) crs[(size_t)it->second] = 0;
    }
    return false;
  }
  bool face_refined_by_neighbor(int64_t id, int f) {
    int64_t nb;
    if (neighbor(id, f, nb) != 1) return false;
    if (!is_active(nb)) return !will_be_coarsened(nb);
    return ref[(size_t)leaf.at(nb)] != 0;
  }
  void limit_vertex_levels() {
    std::unordered_map<int64_t, int> vl;
    const int nv = m.nvc();
    for (size_t i = 0; i < m.active.size(); ++i) {
      const auto &h = m.tree[(size_t)m.active[i]];
      const int lev = ref[i] ? h.level + 1 : crs[i] ? h.level - 1 : h.level;
      for (int v = 0; v < nv; ++v) {
        auto it = vl.find(pv.cls(h.v[v]));
        if (it == vl.end()) vl[pv.cls(h.v[v])] = std::max(0, lev);
        else it->second = std::max(it->second, lev);
      }
    }
    for (int64_t i : active_rev) {
      if (ref[(size_t)i]) continue;
      const auto &h = m.tree[(size_t)m.active[(size_t)i]];
      for (int v = 0; v < nv; ++v) {
        const int lv = vl[pv.cls(h.v[v])];
        if (lv < h.level + 1) continue;
        crs[(size_t)i] = 0;
        if (lv > h.level + 1) {
          ref[(size_t)i] = 1;
          for (int w = 0; w < nv; ++w) vl[pv.cls(h.v[w])] = std::max(vl[pv.cls(h.v[w])], h.level + 1);
        }
      }
    }
  }
  bool coarsening_allowed(int64_t p) const {
    for (int f = 0; f < 2 * dim; ++f) {
      int64_t nb;
      if (neighbor(p, f, nb) == 0) continue;
      const int d = f / 2;
      for (int ch = 0; ch < nkids(); ++ch) {
        if (((ch >> d) & 1) != (f & 1)) continue;  // child not on face f
        int64_t cn;
        if (neighbor(kid(p, ch), f, cn) != 1) continue;
        if (!is_active(cn) && !user.count(cn)) return false;
        if (is_active(cn) && ref[(size_t)leaf.at(cn)]) return false;
      }
    }
    return true;
  }
  void fix_coarsen_flags() {
    for (int it = 0; it < 1000; ++it) {
      const std::vector<char> before = crs;
      limit_vertex_levels();
      for (size_t i = 0; i < m.active.size(); ++i)
        if (m.tree[(size_t)m.active[i]].level == 0) crs[i] = 0;
      user.clear();
      for (int64_t c : all) {
        if (is_active(c)) continue;
        int n = 0;
        for (int ch = 0; ch < nkids(); ++ch) {
          auto lt = leaf.find(kid(c, ch));
          if (lt != leaf.end() && crs[(size_t)lt->second]) {
            ++n;
            crs[(size_t)lt->second] = 0;
          }
        }
        if (n == nkids()) user[c] = 1;
      }
      for (size_t j = all.size(); j-- > 0;) {
        const int64_t c = all[j];
        if (!user.count(c) || !coarsening_allowed(c)) continue;
        for (int ch = 0; ch < nkids(); ++ch) crs[(size_t)leaf.at(kid(c, ch))] = 1;
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
      // step 1: do_not_produce_unrefined_islands
      for (int64_t c : all) {
        if (is_active(c) || !will_be_coarsened(c)) continue;
        int n_nb = 0, cnt = 0;
        for (int f = 0; f < nf; ++f) {
          int64_t nb;
          if (neighbor(c, f, nb) == 0) continue;
          ++n_nb;
          if (face_refined_by_neighbor(c, f)) ++cnt;
        }
        if (cnt == n_nb || (cnt == n_nb - 1 && n_nb == nf))
          for (int ch = 0; ch < nkids(); ++ch) crs[(size_t)leaf.at(kid(c, ch))] = 0;
      }
      // step 2: eliminate_refined_inner_islands | eliminate_refined_boundary_islands
      for (int64_t c : all) {
        const bool act = is_active(c);
        if (act && !ref[(size_t)leaf.at(c)]) continue;
        bool all_active = true;
        if (!act)
          for (int ch = 0; ch < nkids(); ++ch) all_active = all_active && is_active(kid(c, ch));
        if (!all_active) continue;
        int total = 0, unrefined = 0;
        for (int f = 0; f < nf; ++f) {
          int64_t nb;
          if (neighbor(c, f, nb) == 0) continue;
          ++total;
          if (!face_refined_by_neighbor(c, f)) ++unrefined;
        }
        if (unrefined != total || total == 0) continue;
        if (!act) {
          for (int ch = 0; ch < nkids(); ++ch) {
            const size_t k = (size_t)leaf.at(kid(c, ch));
            ref[k] = 0;
            crs[k] = 1;
          }
        } else {
          ref[(size_t)leaf.at(c)] = 0;
        }
      }
      // step 3
      limit_vertex_levels();
      // step 4: eliminate_unrefined_islands
      for (int64_t i : active_rev) {
        if (ref[(size_t)i]) continue;
        const int64_t c = m.active[(size_t)i];
        int refined = 0, unrefined = 0;
        for (int f = 0; f < nf; ++f) {
          int64_t nb;
          if (neighbor(c, f, nb) == 0) continue;
          if (face_refined_by_neighbor(c, f)) ++refined;
          else ++unrefined;
        }
        if (unrefined < refined) {
          crs[(size_t)i] = 0;
          ref[(size_t)i] = 1;
        }
      }
      // step 6: no double refinement at a face
      for (int64_t i : active_rev) {
        if (!ref[(size_t)i]) continue;
        const int64_t c = m.active[(size_t)i];
        for (int f = 0; f < nf; ++f) {
          int64_t nb;
          if (neighbor(c, f, nb) != 2) continue;
          const size_t j = (size_t)leaf.at(nb);
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

// ---- generators (GridGenerator::*, deal.II 9.2 geometry and boundary ids)
std::vector<std::string> split(const std::string &s, char sep) {
  std::vector<std::string> out;
  std::string cur;
  for (char ch : s) {
    if (ch == sep) { out.push_back(cur); cur.clear(); }
    else cur += ch;
  }
  out.push_back(cur);
  for (auto &x : out) {
    size_t a = x.find_first_not_of(" \t"), b = x.find_last_not_of(" \t");
    x = a == std::string::npos ? std::string() : x.substr(a, b - a + 1);
  }
  return out;
}
bool parse_bool(const std::string &s) { return s == "true" || s == "1" || s == "yes"; }
std::vector<double> parse_point(const std::string &s) {
  std::vector<double> p;
  for (auto &t : split(s, ',')) p.push_back(std::stod(t));
  return p;
}

void box_grid(UMesh &m, const int rep[3], const double p1[3], const double p2[3], bool colorize) {
  const int dim = m.dim;
  const int n0 = rep[0] + 1, n1 = rep[1] + 1, n2 = dim == 3 ? rep[2] + 1 : 1;
  for (int k = 0; k < n2; ++k)
    for (int j = 0; j < n1; ++j)
      for (int i = 0; i < n0; ++i)
        m.X.push_back({p1[0] + (p2[0] - p1[0]) * i / rep[0], p1[1] + (p2[1] - p1[1]) * j / rep[1],
                       dim == 3 ? p1[2] + (p2[2] - p1[2]) * k / rep[2] : 0.0});
  for (int k = 0; k < (dim == 3 ? rep[2] : 1); ++k)
    for (int j = 0; j < rep[1]; ++j)
      for (int i = 0; i < rep[0]; ++i) {
        std::array<int64_t, 8> cv{};
        for (int v = 0; v < m.nvc(); ++v)
          cv[v] = (i + (v & 1)) + (int64_t)n0 * ((j + ((v >> 1) & 1)) + (int64_t)n1 * (k + ((v >> 2) & 1)));
        m.cells.push_back(cv);
        m.cell_mf.push_back(-1);
      }
  const double lo[3] = {std::min(p1[0], p2[0]), std::min(p1[1], p2[1]), std::min(p1[2], p2[2])};
  const double hi[3] = {std::max(p1[0], p2[0]), std::max(p1[1], p2[1]), std::max(p1[2], p2[2])};
  mark_boundary(m, [&](const V3 &x) {
    if (!colorize) return 0;
    for (int d = 0; d < dim; ++d) {
      const double tol = 1e-10 * (hi[d] - lo[d]);
      if (std::fabs(x[d] - lo[d]) < tol) return 2 * d;
      if (std::fabs(x[d] - hi[d]) < tol) return 2 * d + 1;
    }
    return 0;
  });
}

int generate(UMesh &m, const std::string &type, const std::string &args) {
  const int dim = m.dim;
  const auto a = split(args, ':');
  try {
    if (type == "hyper_cube") {  // lo : hi : colorize
      const double lo = a.size() > 0 && !a[0].empty() ? std::stod(a[0]) : 0.0;
      const double hi = a.size() > 1 ? std::stod(a[1]) : 1.0;
      const bool col = a.size() > 2 && parse_bool(a[2]);
      const int rep[3] = {1, 1, 1};
      const double p1[3] = {lo, lo, lo}, p2[3] = {hi, hi, hi};
      box_grid(m, rep, p1, p2, col);
    } else if (type == "hyper_rectangle" || type == "subdivided_hyper_rectangle") {
      size_t o = 0;
      int rep[3] = {1, 1, 1};
      if (type == "subdivided_hyper_rectangle") {
        auto r = split(a.at(o++), ',');
        for (int d = 0; d < dim; ++d) rep[d] = std::stoi(r.at((size_t)d));
      }
      const auto q1 = parse_point(a.at(o)), q2 = parse_point(a.at(o + 1));
      const bool col = a.size() > o + 2 && parse_bool(a[o + 2]);
      double p1[3] = {0, 0, 0}, p2[3] = {0, 0, 0};
      for (int d = 0; d < dim; ++d) { p1[d] = q1.at((size_t)d); p2[d] = q2.at((size_t)d); }
      box_grid(m, rep, p1, p2, col);
    } else if (type == "hyper_shell") {  // centre : inner : outer : n_cells : colorize (2D)
      if (dim != 2) return gls_io_set_error(GLS_EINVAL, "hyper_shell: 2D only here (3D: cylinder_shell)");
      const auto c = parse_point(a.at(0));
      const double ri = std::stod(a.at(1)), ro = std::stod(a.at(2));
      int N = a.size() > 3 ? std::stoi(a[3]) : 0;
      const bool col = a.size() > 4 && parse_bool(a[4]);
      if (!(ri > 0 && ri < ro)) return gls_io_set_error(GLS_EINVAL, "hyper_shell: radii");
      if (N == 0) N = (int)std::ceil((2 * M_PI * (ro + ri) / 2) / (ro - ri));
      for (int i = 0; i < N; ++i) m.X.push_back({c[0] + ro * std::cos(2 * M_PI * i / N), c[1] + ro * std::sin(2 * M_PI * i / N), 0});
      for (int i = 0; i < N; ++i) m.X.push_back({c[0] + ri * std::cos(2 * M_PI * i / N), c[1] + ri * std::sin(2 * M_PI * i / N), 0});
      for (int i = 0; i < N; ++i) {  // vertices: outer i, outer i+1, inner i, inner i+1
        m.cells.push_back({i, (i + 1) % N, N + i, N + (i + 1) % N, 0, 0, 0, 0});
        m.cell_mf.push_back(0);
      }
      const double mid = 0.5 * (ri + ro);
      const V3 cc{c[0], c[1], 0};
      mark_boundary(m, [&](const V3 &x) { return col ? (nrm(sub(x, cc)) < mid ? 0 : 1) : 0; });
      // tria.set_all_manifold_ids(0); set_manifold(0, SphericalManifold<2>(center))
      for (size_t ci = 0; ci < m.cells.size(); ++ci)
        for (auto &ln : local_lines(2)) m.line_mf[mkey({m.cells[ci][ln[0]], m.cells[ci][ln[1]]})] = 0;
      ManifoldDesc md;
      md.type = MF_SPHERICAL;
      md.center = cc;
      m.mf[0] = md;
    } else if (type == "cylinder") {  // radius : half_length (3D, axis x)
      if (dim != 3) return gls_io_set_error(GLS_EINVAL, "cylinder: 3D only");
      const double r = a.size() > 0 && !a[0].empty() ? std::stod(a[0]) : 1.0;
      const double hl = a.size() > 1 ? std::stod(a[1]) : 1.0;
      const double d = r / std::sqrt(2.0), s = d / (1 + std::sqrt(2.0));
      // cross-section (y, z): outer corners (+-d, +-d) on the circle, inner square +-s; 3 layers in x
      const double yz[8][2] = {{-d, -d}, {d, -d}, {-s, -s}, {s, -s}, {-s, s}, {s, s}, {-d, d}, {d, d}};
      for (int l = 0; l < 3; ++l)
        for (int i = 0; i < 8; ++i) m.X.push_back({-hl + hl * l, yz[i][0], yz[i][1]});
      // 5 cross-section quads (lexicographic (u, v) corners), extruded along x (local z = x)
      const int q[5][4] = {{0, 1, 2, 3}, {0, 2, 6, 4}, {2, 3, 4, 5}, {3, 1, 5, 7}, {4, 5, 6, 7}};
      for (int l = 0; l < 2; ++l)
        for (auto &qq : q) {
          std::array<int64_t, 8> cv{};
          for (int v = 0; v < 4; ++v) { cv[v] = 8 * l + qq[v]; cv[v + 4] = 8 * (l + 1) + qq[v]; }
          m.cells.push_back(cv);
          m.cell_mf.push_back(-1);
        }
      orient(m);
      mark_boundary(m, [&](const V3 &x) { return x[0] > hl - 1e-5 ? 2 : (x[0] < -hl + 1e-5 ? 1 : 0); });
      // set_all_manifold_ids_on_boundary(0) + CylindricalManifold (axis x); the caps and the cap
      // lines touching the inner square are flat again
      for (auto &bf : m.bface)
        if (bf.second == 0) m.face_mf[bf.first] = 0;
      for (size_t ci = 0; ci < m.cells.size(); ++ci) {
        const auto &cv = m.cells[ci];
        for (int dd = 0; dd < 3; ++dd)
          for (int ss = 0; ss < 2; ++ss) {
            const EKey fk = face_key(m, ci, dd, ss);
            auto b = m.bface.find(fk);
            if (b == m.bface.end()) continue;
            const auto fvv = face_verts(3, dd, ss);
            for (auto &ln : local_lines(3)) {
              if (std::find(fvv.begin(), fvv.end(), ln[0]) == fvv.end() || std::find(fvv.begin(), fvv.end(), ln[1]) == fvv.end())
                continue;
              const EKey lk = mkey({cv[ln[0]], cv[ln[1]]});
              const V3 &p0 = m.X[(size_t)cv[ln[0]]], &p1 = m.X[(size_t)cv[ln[1]]];
              const bool inner = std::fabs(std::fabs(p0[1]) - s) < 1e-12 || std::fabs(std::fabs(p0[2]) - s) < 1e-12 ||
                                 std::fabs(std::fabs(p1[1]) - s) < 1e-12 || std::fabs(std::fabs(p1[2]) - s) < 1e-12;
              if (b->second == 0) {
                if (!m.line_mf.count(lk)) m.line_mf[lk] = 0;
              } else if (inner) {
                m.line_mf[lk] = -2;  // flat (cap lines at the inner square), wins over the hull
              }
            }
          }
      }
      for (auto it = m.line_mf.begin(); it != m.line_mf.end();)
        it = it->second == -2 ? m.line_mf.erase(it) : std::next(it);
      ManifoldDesc md;
      md.type = MF_CYLINDRICAL;
      md.axis = {1, 0, 0};
      m.mf[0] = md;
    } else if (type == "cylinder_shell") {  // length : inner : outer : n_radial : n_axial (3D, axis z)
      if (dim != 3) return gls_io_set_error(GLS_EINVAL, "cylinder_shell: 3D only");
      const double len = std::stod(a.at(0)), ri = std::stod(a.at(1)), ro = std::stod(a.at(2));
      int nr = a.size() > 3 ? std::stoi(a[3]) : 0, nz = a.size() > 4 ? std::stoi(a[4]) : 0;
      if (!(ri > 0 && ri < ro && len > 0)) return gls_io_set_error(GLS_EINVAL, "cylinder_shell: arguments");
      if (nr == 0) nr = (int)std::ceil((2 * M_PI * (ro + ri) / 2) / (ro - ri));
      if (nz == 0) nz = (int)std::ceil(len / (2 * M_PI * (ro + ri) / 2 / nr));
      for (int l = 0; l <= nz; ++l)
        for (int ring = 0; ring < 2; ++ring)
          for (int i = 0; i < nr; ++i) {
            const double rr = ring == 0 ? ro : ri;
            m.X.push_back({rr * std::cos(2 * M_PI * i / nr), rr * std::sin(2 * M_PI * i / nr), len * l / nz});
          }
      for (int l = 0; l < nz; ++l)
        for (int i = 0; i < nr; ++i) {
          const int64_t b0 = (int64_t)l * 2 * nr, b1 = b0 + 2 * nr;
          m.cells.push_back({b0 + i, b0 + (i + 1) % nr, b0 + nr + i, b0 + nr + (i + 1) % nr,
                             b1 + i, b1 + (i + 1) % nr, b1 + nr + i, b1 + nr + (i + 1) % nr});
          m.cell_mf.push_back(0);
        }
      orient(m);
      const double mid = 0.5 * (ri + ro);
      // builder-defined colouring: inner 0, outer 1, z = 0 -> 2, z = length -> 3
      mark_boundary(m, [&](const V3 &x) {
        if (x[2] < 1e-10 * len) return 2;
        if (x[2] > len * (1 - 1e-10)) return 3;
        return std::hypot(x[0], x[1]) < mid ? 0 : 1;
      });
      // set_all_manifold_ids(0) + CylindricalManifold<3>(2)
      for (size_t ci = 0; ci < m.cells.size(); ++ci) {
        for (auto &ln : local_lines(3)) m.line_mf[mkey({m.cells[ci][ln[0]], m.cells[ci][ln[1]]})] = 0;
        for (int dd = 0; dd < 3; ++dd)
          for (int ss = 0; ss < 2; ++ss) m.face_mf[face_key(m, ci, dd, ss)] = 0;
      }
      ManifoldDesc md;
      md.type = MF_CYLINDRICAL;
      md.axis = {0, 0, 1};
      m.mf[0] = md;
    } else {
      return gls_io_set_error(GLS_EINVAL, "grid type '%s' is not supported", type.c_str());
    }
  } catch (const std::exception &e) {
    return gls_io_set_error(GLS_EINVAL, "grid arguments '%s' for %s: %s", args.c_str(), type.c_str(), e.what());
  }
  return GLS_OK;
}

// ---- gmsh ASCII reader (GridIn::read_msh, formats 2.2 / 4.0 / 4.1)
int read_gmsh(UMesh &m, const std::string &path) {
  std::ifstream in(path);
  if (!in) return gls_io_set_error(GLS_EIO, "cannot open mesh file '%s'", path.c_str());
  std::string tok;
  double version = 0;
  std::unordered_map<int64_t, int64_t> node_id;  // gmsh node tag -> vertex index
  std::map<std::pair<int, int>, int> tagmap;     // (entity dim, entity tag) -> physical (or entity) tag
  struct Elem { int type; int tag; std::vector<int64_t> nodes; };
  std::vector<Elem> elems;
  while (in >> tok) {
    if (tok == "$MeshFormat") {
      int ft, ds;
      in >> version >> ft >> ds;
      if (ft != 0) return gls_io_set_error(GLS_EIO, "%s: binary gmsh files are not supported", path.c_str());
    } else if (tok == "$Entities") {
      int64_t np, nc, ns, nv;
      in >> np >> nc >> ns >> nv;
      const int64_t cnt[4] = {np, nc, ns, nv};
      for (int ed = 0; ed < 4; ++ed)
        for (int64_t i = 0; i < cnt[ed]; ++i) {
          int tag;
          double x;
          in >> tag;
          const int nco = (ed == 0 && version >= 4.1) ? 3 : 6;
          for (int j = 0; j < nco; ++j) in >> x;
          int nphys;
          in >> nphys;
          int phys = tag;
          for (int j = 0; j < nphys; ++j) {
            int pt;
            in >> pt;
            if (j == 0) phys = pt;
          }
          tagmap[{ed, tag}] = phys;
          if (ed > 0) {
            int64_t nb, t;
            in >> nb;
            for (int64_t j = 0; j < nb; ++j) in >> t;
          }
        }
    } else if (tok == "$Nodes") {
      if (version < 4) {
        int64_t n;
        in >> n;
        for (int64_t i = 0; i < n; ++i) {
          int64_t id;
          V3 x;
          in >> id >> x[0] >> x[1] >> x[2];
          node_id[id] = (int64_t)m.X.size();
          m.X.push_back(x);
        }
      } else {
        int64_t nb, n, a, b;
        in >> nb >> n;
        if (version >= 4.1) in >> a >> b;
        for (int64_t blk = 0; blk < nb; ++blk) {
          int64_t e1, e2, par, nn;
          in >> e1 >> e2 >> par >> nn;
          if (par) return gls_io_set_error(GLS_EIO, "%s: parametric gmsh nodes are not supported", path.c_str());
          if (version >= 4.1) {
            std::vector<int64_t> tags((size_t)nn);
            for (auto &t : tags) in >> t;
            for (int64_t i = 0; i < nn; ++i) {
              V3 x;
              in >> x[0] >> x[1] >> x[2];
              node_id[tags[(size_t)i]] = (int64_t)m.X.size();
              m.X.push_back(x);
            }
          } else {
            for (int64_t i = 0; i < nn; ++i) {
              int64_t id;
              V3 x;
              in >> id >> x[0] >> x[1] >> x[2];
              node_id[id] = (int64_t)m.X.size();
              m.X.push_back(x);
            }
          }
        }
      }
    } else if (tok == "$Elements") {
      auto nodes_of = [](int type) { return type == 1 ? 2 : type == 3 ? 4 : type == 5 ? 8 : type == 15 ? 1 : type == 2 ? 3 : type == 4 ? 4 : -1; };
      if (version < 4) {
        int64_t n;
        in >> n;
        for (int64_t i = 0; i < n; ++i) {
          int64_t id;
          int type, ntags;
          in >> id >> type >> ntags;
          int phys = 0;
          for (int j = 0; j < ntags; ++j) {
            int t;
            in >> t;
            if (j == 0) phys = t;
          }
          const int nn = nodes_of(type);
          if (nn < 0) return gls_io_set_error(GLS_EIO, "%s: gmsh element type %d is not supported", path.c_str(), type);
          Elem e{type, phys, std::vector<int64_t>((size_t)nn)};
          for (auto &x : e.nodes) in >> x;
          elems.push_back(std::move(e));
        }
      } else {
        int64_t nb, n, a, b;
        in >> nb >> n;
        if (version >= 4.1) in >> a >> b;
        for (int64_t blk = 0; blk < nb; ++blk) {
          int ed, et, type;
          int64_t ne;
          if (version >= 4.1) in >> ed >> et >> type >> ne;
          else in >> et >> ed >> type >> ne;
          auto tm = tagmap.find({ed, et});
          const int phys = tm == tagmap.end() ? et : tm->second;
          const int nn = nodes_of(type);
          if (nn < 0) return gls_io_set_error(GLS_EIO, "%s: gmsh element type %d is not supported", path.c_str(), type);
          for (int64_t i = 0; i < ne; ++i) {
            int64_t id;
            in >> id;
            Elem e{type, phys, std::vector<int64_t>((size_t)nn)};
            for (auto &x : e.nodes) in >> x;
            elems.push_back(std::move(e));
          }
        }
      }
    }
  }
  if (m.X.empty()) return gls_io_set_error(GLS_EIO, "%s: no nodes", path.c_str());
  const int cell_type = m.dim == 2 ? 3 : 5, face_type = m.dim == 2 ? 1 : 3;
  std::vector<std::pair<EKey, int>> bf;
  for (auto &e : elems) {
    std::vector<int64_t> v;
    for (auto t : e.nodes) {
      auto it = node_id.find(t);
      if (it == node_id.end()) return gls_io_set_error(GLS_EIO, "%s: element node %lld undefined", path.c_str(), (long long)t);
      v.push_back(it->second);
    }
    if (e.type == cell_type) {
      std::array<int64_t, 8> cv{};
      if (m.dim == 2) cv = {v[0], v[1], v[3], v[2], 0, 0, 0, 0};  // gmsh counter-clockwise -> lexicographic
      else cv = {v[0], v[1], v[3], v[2], v[4], v[5], v[7], v[6]};
      m.cells.push_back(cv);
      m.cell_mf.push_back(-1);
    } else if (e.type == face_type) {
      bf.push_back({m.dim == 2 ? mkey({v[0], v[1]}) : mkey({v[0], v[1], v[2], v[3]}), e.tag});
    } else if (e.type == 2 || e.type == 4 || (m.dim == 3 && e.type != 1 && e.type != 15)) {
      return gls_io_set_error(GLS_EIO, "%s: simplex elements are not supported (quads / hexes only)", path.c_str());
    }
  }
  if (m.cells.empty()) return gls_io_set_error(GLS_EIO, "%s: no %s elements", path.c_str(), m.dim == 2 ? "quad" : "hex");
  // drop unused nodes (gmsh files may carry geometry points)
  std::vector<int64_t> used(m.X.size(), -1);
  std::vector<V3> X2;
  for (auto &cv : m.cells)
    for (int v = 0; v < m.nvc(); ++v)
      if (used[(size_t)cv[v]] < 0) { used[(size_t)cv[v]] = (int64_t)X2.size(); X2.push_back(m.X[(size_t)cv[v]]); }
  for (auto &cv : m.cells)
    for (int v = 0; v < m.nvc(); ++v) cv[v] = used[(size_t)cv[v]];
  m.X.swap(X2);
  orient(m);
  mark_boundary(m, [](const V3 &) { return 0; });
  for (auto &p : bf) {
    EKey k = p.first;
    bool ok = true;
    for (int i = 0; i < (m.dim == 2 ? 2 : 4); ++i) {
      if (used[(size_t)k.v[i]] < 0) ok = false;
      else k.v[i] = used[(size_t)k.v[i]];
    }
    if (!ok) continue;
    std::sort(k.v, k.v + (m.dim == 2 ? 2 : 4));
    auto it = m.bface.find(k);
    if (it != m.bface.end()) it->second = p.second;
  }
  return GLS_OK;
}

// ---- FE space (FE_Q(k) x dim + FE_Q(kp)) on the mesh, k <= 2
struct FESpaceImpl {
  gls_fe_space pub{};
  std::vector<int32_t> cell_vnodes, cell_pnodes, cell_mapping, cell_level;
  std::vector<double> vnode_x, pnode_x, cell_support, cell_measure;
  std::vector<uint32_t> vnode_bid, pnode_bid;
  // hanging lines (node level, chains closed): node = sum_j w_j master_j
  std::vector<int64_t> vh_node, vh_off, vh_master, ph_node, ph_off, ph_master;
  std::vector<double> vh_w, ph_w;
  // hierarchy snapshot for SolutionTransfer: hierarchy id of every active cell, and per record its
  // parent, child position and first child
  std::vector<int64_t> hid, t_parent, t_child0;
  std::vector<int> t_pos;
  std::vector<std::array<int64_t, 8>> cell_verts, t_verts;  // vertex ids of the active cells / all records
  std::vector<V3> verts;
  std::map<EKey, int64_t> line_mid, face_mid;
  std::vector<int> face_bid;  // [n_cells][2 dim] boundary id of each cell face, -1 interior
  std::vector<std::array<int, 3>> periodic;  // the space's periodic pairs (id a, id b, direction)
};

using HangLines = std::map<int64_t, std::vector<std::pair<int64_t, double>>>;
double lag1(int k, int a, double x);
int close_lines(HangLines &out);
bool periodic_face_params(int dim, int dir, const V3 (&C)[2][2], const V3 &x, double tol, double uv[2]);

// DoFTools::make_hanging_node_constraints (gls_navier_stokes.cc:84, 143) for FE_Q(kk) on the
// hierarchy: every line (3D: and quad) of an active cell that is refined in the active mesh (its
// midpoint vertex is a node) carries the nodes of the refined object (midpoint vertex, child lines,
// child quads); each is constrained to the active cell's Qk interpolant on that object, evaluated
// at the node's reference position (2kk+1 positions per direction on the refined object). `ids`
// maps object keys (vertex {-3, v}, line / quad = sorted vertex ids) to node ids; cn = the active
// cells' node lists. Chains are closed afterwards (AffineConstraints::close).
int hanging_lines(const UMesh &m, int kk, const std::map<EKey, int64_t> &ids, const std::vector<int32_t> &cn,
                  HangLines &out) {
  const int dim = m.dim, kk1 = kk + 1, nn = dim == 2 ? kk1 * kk1 : kk1 * kk1 * kk1, P = 2 * kk;
  auto vnode = [&](int64_t v) -> int64_t {
    auto it = ids.find(EKey{{-3, v, -1, -1}});
    return it == ids.end() ? -1 : it->second;
  };
  auto onode = [&](const EKey &k) -> int64_t {
    auto it = ids.find(k);
    return it == ids.end() ? -1 : it->second;
  };
  auto mid = [&](const std::map<EKey, int64_t> &mp, const EKey &k) -> int64_t {
    auto it = mp.find(k);
    return it == mp.end() ? -1 : it->second;
  };
  auto local = [&](const int *ia) {
    return ia[0] + kk1 * (ia[1] + (dim == 3 ? kk1 * ia[2] : 0));
  };
  for (size_t c = 0; c < m.cells.size(); ++c) {
    const auto &cv = m.cells[c];
    // lines
    for (auto &ln : local_lines(dim)) {
      const int la = ln[0], lb = ln[1];
      int dir = 0;
      for (int d = 0; d < dim; ++d)
        if (((la ^ lb) >> d) & 1) dir = d;
      const int64_t mv = mid(m.line_mid, mkey({cv[la], cv[lb]}));
      if (mv < 0 || vnode(mv) < 0) continue;
      const int64_t V[3] = {cv[la], mv, cv[lb]};
      int64_t kn[4];
      for (int j = 0; j <= kk; ++j) {
        int ia[3] = {0, 0, 0};
        for (int d = 0; d < dim; ++d) ia[d] = d == dir ? j : kk * ((la >> d) & 1);
        kn[j] = cn[c * nn + (size_t)local(ia)];
      }
      for (int p = 0; p <= P; ++p) {
        const int64_t fn = p % kk == 0 ? vnode(V[p / kk]) : onode(mkey({V[p / kk], V[p / kk + 1]}));
        if (fn < 0 || out.count(fn)) continue;
        bool own = false;
        for (int j = 0; j <= kk; ++j) own = own || kn[j] == fn;
        if (own) continue;
        std::vector<std::pair<int64_t, double>> line;
        for (int j = 0; j <= kk; ++j) {
          const double w = lag1(kk, j, (double)p / P);
          if (std::fabs(w) > 1e-13) line.push_back({kn[j], w});
        }
        out[fn] = line;
      }
    }
    if (dim != 3) continue;
    // quads
    for (int d = 0; d < 3; ++d)
      for (int s = 0; s < 2; ++s) {
        const int64_t fv = mid(m.face_mid, face_key_v(3, cv, d, s));
        if (fv < 0 || vnode(fv) < 0) continue;
        int t[2], nt = 0;
        for (int e = 0; e < 3; ++e)
          if (e != d) t[nt++] = e;
        int64_t C[2][2];
        for (int iu = 0; iu < 2; ++iu)
          for (int iv = 0; iv < 2; ++iv) C[iu][iv] = cv[(s << d) | (iu << t[0]) | (iv << t[1])];
        int64_t V[3][3];
        V[1][1] = fv;
        bool ok = true;
        for (int i = 0; i < 2; ++i) {
          V[2 * i][0] = C[i][0];
          V[2 * i][2] = C[i][1];
          V[0][2 * i] = C[0][i];
          V[2][2 * i] = C[1][i];
          V[1][2 * i] = mid(m.line_mid, mkey({C[0][i], C[1][i]}));
          V[2 * i][1] = mid(m.line_mid, mkey({C[i][0], C[i][1]}));
          ok = ok && V[1][2 * i] >= 0 && V[2 * i][1] >= 0;
        }
        if (!ok) return gls_io_set_error(GLS_EINVAL, "hanging nodes: refined quad without refined lines");
        std::vector<int64_t> kn;
        for (int jv = 0; jv <= kk; ++jv)
          for (int ju = 0; ju <= kk; ++ju) {
            int ia[3];
            ia[d] = s * kk;
            ia[t[0]] = ju;
            ia[t[1]] = jv;
            kn.push_back(cn[c * nn + (size_t)local(ia)]);
          }
        for (int pv = 0; pv <= P; ++pv)
          for (int pu = 0; pu <= P; ++pu) {
            const int eu = pu / kk, ev = pv / kk;
            const bool ou = pu % kk != 0, ov = pv % kk != 0;
            int64_t fn;
            if (!ou && !ov) fn = vnode(V[eu][ev]);
            else if (ou && !ov) fn = onode(mkey({V[eu][ev], V[eu + 1][ev]}));
            else if (!ou && ov) fn = onode(mkey({V[eu][ev], V[eu][ev + 1]}));
            else fn = onode(mkey({V[eu][ev], V[eu + 1][ev], V[eu][ev + 1], V[eu + 1][ev + 1]}));
            if (fn < 0 || out.count(fn)) continue;
            bool own = false;
            for (int64_t x : kn) own = own || x == fn;
            if (own) continue;
            std::vector<std::pair<int64_t, double>> line;
            for (int jv = 0; jv <= kk; ++jv)
              for (int ju = 0; ju <= kk; ++ju) {
                const double w = lag1(kk, ju, (double)pu / P) * lag1(kk, jv, (double)pv / P);
                if (std::fabs(w) > 1e-13) line.push_back({kn[(size_t)(ju + kk1 * jv)], w});
              }
            out[fn] = line;
          }
      }
  }
  return close_lines(out);
}

// AffineConstraints::close: substitute constrained masters by their lines until none is left
int close_lines(HangLines &out) {
  for (int pass = 0; pass < 32; ++pass) {
    bool changed = false;
    for (auto &kv : out) {
      std::map<int64_t, double> acc;
      bool sub = false;
      for (auto &mw : kv.second) {
        auto it = out.find(mw.first);
        if (it == out.end()) {
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
    if (!changed) return GLS_OK;
  }
  return gls_io_set_error(GLS_EINVAL, "hanging-node chains do not close");
}

double lag1(int k, int a, double x) {  // Lagrange basis a of degree k on equidistant nodes (k <= 2)
  double v = 1.0;
  for (int b = 0; b <= k; ++b)
    if (b != a) v *= (x - (double)b / k) / ((double)(a - b) / k);
  return v;
}

// (u, v) on a straight periodic face with corners C[iu][iv] (2D: a line, v = 0) of the point x, in the
// coordinates across the periodic direction `dir` (x and the face may sit on either side of the
// boundary); false when x is off the face. Snapped to multiples of 1/16 (the positions of nodes of
// finer faces of the hierarchy) when within 1e-10.
bool periodic_face_params(int dim, int dir, const V3 (&C)[2][2], const V3 &x, double tol, double uv[2]) {
  auto pr = [&](V3 a) {
    a[dir] = 0.0;
    return a;
  };
  const V3 c00 = pr(C[0][0]), c10 = pr(C[1][0]), xx = pr(x);
  double u = 0.5, v = 0.0;
  if (dim == 2) {
    const V3 t = sub(c10, c00);
    const double tt = dot3(t, t);
    if (tt <= 0) return false;
    u = dot3(sub(xx, c00), t) / tt;
    if (nrm(sub(add(c00, scl(t, u)), xx)) > tol) return false;
  } else {
    const V3 c01 = pr(C[0][1]), c11 = pr(C[1][1]);
    const int o1 = (dir + 1) % 3, o2 = (dir + 2) % 3;
    v = 0.5;
    for (int it = 0; it < 40; ++it) {
      V3 F = sub(add(add(scl(c00, (1 - u) * (1 - v)), scl(c10, u * (1 - v))), add(scl(c01, (1 - u) * v), scl(c11, u * v))), xx);
      const V3 Fu = add(scl(sub(c10, c00), 1 - v), scl(sub(c11, c01), v));
      const V3 Fv = add(scl(sub(c01, c00), 1 - u), scl(sub(c11, c10), u));
      const double det = Fu[o1] * Fv[o2] - Fu[o2] * Fv[o1];
      if (std::fabs(det) < 1e-300) return false;
      const double du = -(F[o1] * Fv[o2] - F[o2] * Fv[o1]) / det, dv = -(Fu[o1] * F[o2] - Fu[o2] * F[o1]) / det;
      u += du;
      v += dv;
      if (std::fabs(du) + std::fabs(dv) < 1e-15) break;
    }
    const V3 F = sub(add(add(scl(c00, (1 - u) * (1 - v)), scl(c10, u * (1 - v))), add(scl(c01, (1 - u) * v), scl(c11, u * v))), xx);
    if (nrm(F) > tol) return false;
  }
  const double e = 1e-9;
  if (u < -e || u > 1 + e || v < -e || v > 1 + e) return false;
  for (double *w : {&u, &v}) {
    const double r = std::round(*w * 16.0) / 16.0;
    if (std::fabs(r - *w) < 1e-10) *w = r;
  }
  uv[0] = u;
  uv[1] = v;
  return true;
}

// deal.II cell->measure(): exact area / volume of the bilinear / trilinear cell (2-point Gauss of
// det J, exact for these polynomial degrees)
double cell_measure(const UMesh &m, const std::array<int64_t, 8> &cv) {
  const double g = 0.5 / std::sqrt(3.0), xs[2] = {0.5 - g, 0.5 + g};
  double vol = 0;
  const int dim = m.dim, nv = m.nvc();
  for (int q = 0; q < (1 << dim); ++q) {
    const double xi[3] = {xs[q & 1], xs[(q >> 1) & 1], xs[(q >> 2) & 1]};
    double J[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
    for (int v = 0; v < nv; ++v)
      for (int a = 0; a < dim; ++a) {
        double gr = ((v >> a) & 1) ? 1.0 : -1.0;
        for (int b = 0; b < dim; ++b)
          if (b != a) gr *= ((v >> b) & 1) ? xi[b] : 1 - xi[b];
        for (int i = 0; i < dim; ++i) J[i][a] += gr * m.X[(size_t)cv[v]][i];
      }
    const double det = dim == 2 ? J[0][0] * J[1][1] - J[0][1] * J[1][0]
                                : J[0][0] * (J[1][1] * J[2][2] - J[1][2] * J[2][1]) -
                                      J[0][1] * (J[1][0] * J[2][2] - J[1][2] * J[2][0]) +
                                      J[0][2] * (J[1][0] * J[2][1] - J[1][1] * J[2][0]);
    vol += det / (1 << dim);
  }
  return vol;
}

// MappingQGeneric(2) support points of one cell: vertices, line points on the lines' manifolds,
// quad points from the TFI weights (vertices -1/4, lines +1/2) on the face's (2D: the cell's)
// manifold, the hex centre from (vertices +1/8, lines -1/4, faces +1/2) on the cell's manifold
void q2_support(const UMesh &m, size_t c, std::vector<V3> &S) {
  const int dim = m.dim, n1 = 3, ns = dim == 2 ? 9 : 27;
  const auto &cv = m.cells[c];
  S.assign((size_t)ns, V3{0, 0, 0});
  auto idx = [&](int i, int j, int l) { return (size_t)(i + n1 * (j + n1 * l)); };
  for (int v = 0; v < m.nvc(); ++v) S[idx(2 * (v & 1), 2 * ((v >> 1) & 1), 2 * ((v >> 2) & 1))] = m.X[(size_t)cv[v]];
  const auto lines = local_lines(dim);
  std::vector<V3> lmid(lines.size());
  for (size_t li = 0; li < lines.size(); ++li) {
    const int a = lines[li][0], b = lines[li][1];
    const EKey k = mkey({cv[a], cv[b]});
    lmid[li] = new_point(m, m.mf_of(m.line_mf, k), {m.X[(size_t)cv[a]], m.X[(size_t)cv[b]]}, {0.5, 0.5});
    int q[3];
    for (int d = 0; d < 3; ++d) q[d] = ((a >> d) & 1) == ((b >> d) & 1) ? 2 * ((a >> d) & 1) : 1;
    S[idx(q[0], dim > 1 ? q[1] : 0, dim > 2 ? q[2] : 0)] = lmid[li];
  }
  auto quad = [&](int mfid, const std::array<int, 4> &fv) {
    std::vector<V3> p;
    std::vector<double> w;
    for (int i = 0; i < 4; ++i) { p.push_back(m.X[(size_t)cv[fv[i]]]); w.push_back(-0.25); }
    for (size_t li = 0; li < lines.size(); ++li)
      if (std::find(fv.begin(), fv.end(), lines[li][0]) != fv.end() && std::find(fv.begin(), fv.end(), lines[li][1]) != fv.end()) {
        p.push_back(lmid[li]);
        w.push_back(0.5);
      }
    return new_point(m, mfid, p, w);
  };
  if (dim == 2) {
    S[idx(1, 1, 0)] = quad(m.cell_mf[c], {0, 1, 2, 3});
    return;
  }
  std::vector<V3> fmid;
  for (int d = 0; d < 3; ++d)
    for (int s = 0; s < 2; ++s) {
      const V3 p = quad(m.mf_of(m.face_mf, face_key(m, c, d, s)), face_verts(3, d, s));
      fmid.push_back(p);
      int q[3] = {1, 1, 1};
      q[d] = 2 * s;
      S[idx(q[0], q[1], q[2])] = p;
    }
  std::vector<V3> p;
  std::vector<double> w;
  for (int v = 0; v < 8; ++v) { p.push_back(m.X[(size_t)cv[v]]); w.push_back(0.125); }
  for (auto &x : lmid) { p.push_back(x); w.push_back(-0.25); }
  for (auto &x : fmid) { p.push_back(x); w.push_back(0.5); }
  S[idx(1, 1, 1)] = new_point(m, m.cell_mf[c], p, w);
}

int build_fe_space(const UMesh &m, int k, int kp, int qall, int nper, const int32_t *per, FESpaceImpl &F) {
  const int dim = m.dim;
  if (k < 1 || k > 2 || kp < 1 || kp > k) return gls_io_set_error(GLS_EINVAL, "unstructured meshes: 1 <= kp <= k <= 2");
  const int64_t nc = (int64_t)m.cells.size();
  const int k1 = k + 1, nl = dim == 2 ? k1 * k1 : k1 * k1 * k1;
  // boundary lines (MappingQ uses the Qk mapping on cells with a boundary line)
  std::map<EKey, char> bline;
  for (size_t c = 0; c < m.cells.size(); ++c)
    for (int d = 0; d < dim; ++d)
      for (int s = 0; s < 2; ++s) {
        if (!m.bface.count(face_key(m, c, d, s))) continue;
        const auto fv = face_verts(dim, d, s);
        const int nf = dim == 2 ? 2 : 4;
        for (auto &ln : local_lines(dim))
          if (std::find(fv.begin(), fv.begin() + nf, ln[0]) != fv.begin() + nf &&
              std::find(fv.begin(), fv.begin() + nf, ln[1]) != fv.begin() + nf)
            bline[mkey({m.cells[c][ln[0]], m.cells[c][ln[1]]})] = 1;
      }
  F.cell_support.assign((size_t)(nc * nl * dim), 0.0);
  F.cell_mapping.assign((size_t)nc, 1);
  F.cell_measure.assign((size_t)nc, 0.0);
  std::vector<V3> S;
  double volume = 0;
  for (int64_t c = 0; c < nc; ++c) {
    const auto &cv = m.cells[(size_t)c];
    F.cell_measure[(size_t)c] = cell_measure(m, cv);
    volume += F.cell_measure[(size_t)c];
    bool hb = false;
    for (auto &ln : local_lines(dim))
      if (bline.count(mkey({cv[ln[0]], cv[ln[1]]}))) hb = true;
    const bool qk = k == 2 && (qall || hb);
    F.cell_mapping[(size_t)c] = qk ? k : 1;
    if (qk) {
      q2_support(m, (size_t)c, S);
    } else {  // multilinear map sampled at the Qk support points (exact embedding)
      S.assign((size_t)nl, V3{0, 0, 0});
      for (int a = 0; a < nl; ++a) {
        const int ia[3] = {a % k1, (a / k1) % k1, a / (k1 * k1)};
        for (int v = 0; v < m.nvc(); ++v) {
          double wv = 1.0;
          for (int d = 0; d < dim; ++d) {
            const double x = (double)ia[d] / k;
            wv *= ((v >> d) & 1) ? x : 1 - x;
          }
          S[(size_t)a] = add(S[(size_t)a], scl(m.X[(size_t)cv[v]], wv));
        }
      }
    }
    for (int a = 0; a < nl; ++a)
      for (int d = 0; d < dim; ++d) F.cell_support[((size_t)c * nl + a) * dim + d] = S[(size_t)a][d];
  }
  // node numbering: one node per vertex / line / face / cell interior touched by the lattice
  auto number = [&](int kk, std::vector<int32_t> &cn, std::vector<double> &nx, std::vector<uint32_t> &nb,
                    std::vector<int64_t> &hnode, std::vector<int64_t> &hoff, std::vector<int64_t> &hmaster,
                    std::vector<double> &hw) -> int {
    const int kk1 = kk + 1, nn = dim == 2 ? kk1 * kk1 : kk1 * kk1 * kk1;
    std::map<EKey, int64_t> ids;  // entity key (with a type tag in v[3] for vertices/cells) -> node
    cn.assign((size_t)(nc * nn), -1);
    std::vector<V3> pos;
    std::vector<int> posdeg;
    for (int64_t c = 0; c < nc; ++c) {
      const auto &cv = m.cells[(size_t)c];
      for (int a = 0; a < nn; ++a) {
        const int ia[3] = {a % kk1, (a / kk1) % kk1, dim == 3 ? a / (kk1 * kk1) : 0};
        std::vector<int64_t> verts;
        // vertices of the entity: every corner reachable by moving interior coordinates to 0 / kk
        int nint = 0;
        for (int d = 0; d < dim; ++d)
          if (ia[d] != 0 && ia[d] != kk) ++nint;
        for (int v = 0; v < m.nvc(); ++v) {
          bool on = true;
          for (int d = 0; d < dim; ++d) {
            const int b = (v >> d) & 1;
            if ((ia[d] == 0 && b != 0) || (ia[d] == kk && b != 1)) on = false;
          }
          if (on) verts.push_back(cv[v]);
        }
        std::sort(verts.begin(), verts.end());
        EKey key{{-1, -1, -1, -1}};
        if (nint == dim) key = EKey{{-2, c, -1, -1}};  // cell interior
        else if (verts.size() == 1) key = EKey{{-3, verts[0], -1, -1}};
        else for (size_t i = 0; i < verts.size() && i < 4; ++i) key.v[i] = verts[i];
        auto it = ids.find(key);
        int64_t id;
        if (it == ids.end()) {
          id = (int64_t)pos.size();
          ids[key] = id;
          pos.push_back(V3{0, 0, 0});
          posdeg.push_back(0);
        } else {
          id = it->second;
        }
        cn[(size_t)(c * nn + a)] = (int32_t)id;
        // position from this cell's mapping (cells with the higher mapping degree win)
        const int md = F.cell_mapping[(size_t)c];
        if (md >= posdeg[(size_t)id]) {
          V3 x{0, 0, 0};
          for (int b = 0; b < nl; ++b) {
            const int ib[3] = {b % k1, (b / k1) % k1, b / (k1 * k1)};
            double wv = 1.0;
            for (int d = 0; d < dim; ++d) wv *= lag1(k, ib[d], (double)ia[d] / kk);
            if (wv == 0.0) continue;
            for (int d = 0; d < dim; ++d) x[d] += wv * F.cell_support[((size_t)c * nl + b) * dim + d];
          }
          pos[(size_t)id] = x;
          posdeg[(size_t)id] = md;
        }
      }
    }
    HangLines hang;
    if (int rc = hanging_lines(m, kk, ids, cn, hang); rc != GLS_OK) return rc;
    // boundary id bits
    std::vector<uint32_t> bits(pos.size(), 0u);
    for (int64_t c = 0; c < nc; ++c)
      for (int d = 0; d < dim; ++d)
        for (int s = 0; s < 2; ++s) {
          auto b = m.bface.find(face_key(m, (size_t)c, d, s));
          if (b == m.bface.end() || b->second < 0 || b->second > 31) continue;
          for (int a = 0; a < nn; ++a) {
            const int ia[3] = {a % kk1, (a / kk1) % kk1, dim == 3 ? a / (kk1 * kk1) : 0};
            if (ia[d] == s * kk) bits[(size_t)cn[(size_t)(c * nn + a)]] |= 1u << b->second;
          }
        }
    // periodic identification (make_periodicity_constraints): nodes on faces of id b map onto the
    // translated nodes of id a. Under local refinement a node without a partner lies on a face finer than
    // the one across the boundary; it is constrained to that coarser face's Q_kk interpolant at its
    // position (deal.II constrains the finer side's DoFs to the coarser side's), like a hanging node.
    std::vector<int64_t> rep(pos.size());
    for (size_t i = 0; i < rep.size(); ++i) rep[i] = (int64_t)i;
    HangLines phang;  // pre-identification node ids
    const double tol = periodic_tol(pos);
    for (int p = 0; p < nper; ++p) {
      const int ida = per[3 * p], idb = per[3 * p + 1], dir = per[3 * p + 2];
      std::vector<int64_t> A, B;
      for (size_t i = 0; i < pos.size(); ++i) {
        if ((bits[i] >> ida) & 1) A.push_back((int64_t)i);
        if ((bits[i] >> idb) & 1) B.push_back((int64_t)i);
      }
      std::map<std::array<long long, 2>, std::vector<int64_t>> grid;
      const int o1 = (dir + 1) % 3, o2 = (dir + 2) % 3;
      auto cellk = [&](const V3 &x) { return std::array<long long, 2>{std::llround(x[o1] / (100 * tol)), std::llround(x[o2] / (100 * tol))}; };
      for (auto i : A) grid[cellk(pos[(size_t)i])].push_back(i);
      std::set<int64_t> hitA;
      std::vector<int64_t> loneB;
      for (auto j : B) {
        int64_t match = -1;
        const auto ck = cellk(pos[(size_t)j]);
        for (long long dx = -1; dx <= 1 && match < 0; ++dx)
          for (long long dy = -1; dy <= 1 && match < 0; ++dy) {
            auto g = grid.find({ck[0] + dx, ck[1] + dy});
            if (g == grid.end()) continue;
            for (auto i : g->second)
              if (std::fabs(pos[(size_t)i][o1] - pos[(size_t)j][o1]) < tol &&
                  std::fabs(pos[(size_t)i][o2] - pos[(size_t)j][o2]) < tol) { match = i; break; }
          }
        if (match < 0) {
          loneB.push_back(j);
          continue;
        }
        rep[(size_t)j] = match;
        hitA.insert(match);
      }
      std::vector<int64_t> loneA;
      for (auto i : A)
        if (!hitA.count(i)) loneA.push_back(i);
      if (loneA.empty() && loneB.empty()) continue;
      // the active cells' faces on a side: corners (lexicographic in the two tangential directions) + nodes
      struct PFace {
        V3 C[2][2];
        std::vector<int64_t> kn;
      };
      auto side_faces = [&](int bid) {
        std::vector<PFace> out;
        for (int64_t c = 0; c < nc; ++c)
          for (int d = 0; d < dim; ++d)
            for (int s2 = 0; s2 < 2; ++s2) {
              auto bf = m.bface.find(face_key(m, (size_t)c, d, s2));
              if (bf == m.bface.end() || bf->second != bid) continue;
              int t[2] = {0, 0}, nt = 0;
              for (int e = 0; e < dim; ++e)
                if (e != d) t[nt++] = e;
              PFace f;
              const auto &cv = m.cells[(size_t)c];
              for (int iu = 0; iu < 2; ++iu)
                for (int iv = 0; iv < 2; ++iv)
                  f.C[iu][iv] = m.X[(size_t)cv[(size_t)((s2 << d) | (iu << t[0]) | (dim == 3 ? iv << t[1] : 0))]];
              for (int jv = 0; jv <= (dim == 3 ? kk : 0); ++jv)
                for (int ju = 0; ju <= kk; ++ju) {
                  int ia[3] = {0, 0, 0};
                  ia[d] = s2 * kk;
                  ia[t[0]] = ju;
                  if (dim == 3) ia[t[1]] = jv;
                  f.kn.push_back(cn[(size_t)(c * nn + ia[0] + kk1 * (ia[1] + (dim == 3 ? kk1 * ia[2] : 0)))]);
                }
              out.push_back(std::move(f));
            }
        return out;
      };
      auto constrain = [&](const std::vector<int64_t> &lone, const std::vector<PFace> &across, int ida_, int idb_) -> int {
        for (int64_t j : lone) {
          if (hang.count(j) || phang.count(j)) continue;  // already a hanging node of its own side
          bool done = false;
          for (const auto &f : across) {
            double uv[2];
            if (!periodic_face_params(dim, dir, f.C, pos[(size_t)j], tol, uv)) continue;
            std::vector<std::pair<int64_t, double>> line;
            for (int jv = 0; jv <= (dim == 3 ? kk : 0); ++jv)
              for (int ju = 0; ju <= kk; ++ju) {
                const double w = lag1(kk, ju, uv[0]) * (dim == 3 ? lag1(kk, jv, uv[1]) : 1.0);
                if (std::fabs(w) > 1e-13) line.push_back({f.kn[(size_t)(ju + kk1 * jv)], w});
              }
            phang[j] = line;
            done = true;
            break;
          }
          if (!done)
            return gls_io_set_error(GLS_EINVAL, "periodic boundaries %d / %d: node without a partner face", ida_, idb_);
        }
        return GLS_OK;
      };
      if (!loneB.empty()) {
        if (int rc = constrain(loneB, side_faces(ida), ida, idb); rc != GLS_OK) return rc;
      }
      if (!loneA.empty()) {
        if (int rc = constrain(loneA, side_faces(idb), ida, idb); rc != GLS_OK) return rc;
      }
    }
    for (size_t i = 0; i < rep.size(); ++i)  // chains (corner nodes of several periodic pairs)
      while (rep[(size_t)rep[i]] != rep[i]) rep[i] = rep[(size_t)rep[i]];
    std::vector<int64_t> compact(pos.size(), -1);
    int64_t n = 0;
    for (size_t i = 0; i < pos.size(); ++i)
      if (rep[i] == (int64_t)i) compact[i] = n++;
    nx.assign((size_t)(n * dim), 0.0);
    nb.assign((size_t)n, 0u);
    for (size_t i = 0; i < pos.size(); ++i) {
      const int64_t t = compact[(size_t)rep[i]];
      if (rep[i] == (int64_t)i)
        for (int d = 0; d < dim; ++d) nx[(size_t)(t * dim + d)] = pos[i][d];
      nb[(size_t)t] |= bits[i];
    }
    for (auto &x : cn) x = (int32_t)compact[(size_t)rep[(size_t)x]];
    // constraint lines in the identified numbering: the hanging lines of each side, then the periodic
    // lines of unpartnered nodes (a node keeps its first line), chains closed together
    HangLines all;
    auto put = [&](const HangLines &H) {
      for (auto &kv : H) {
        const int64_t nd = compact[(size_t)rep[(size_t)kv.first]];
        if (all.count(nd)) continue;
        std::map<int64_t, double> acc;
        for (auto &mw : kv.second) acc[compact[(size_t)rep[(size_t)mw.first]]] += mw.second;
        std::vector<std::pair<int64_t, double>> line;
        for (auto &a : acc)
          if (std::fabs(a.second) > 1e-14 && a.first != nd) line.push_back(a);
        all[nd] = line;
      }
    };
    put(hang);
    put(phang);
    if (!phang.empty())
      if (int rc = close_lines(all); rc != GLS_OK) return rc;
    hnode.clear();
    hoff.assign(1, 0);
    hmaster.clear();
    hw.clear();
    for (auto &kv : all) {
      hnode.push_back(kv.first);
      for (auto &mw : kv.second) {
        hmaster.push_back(mw.first);
        hw.push_back(mw.second);
      }
      hoff.push_back((int64_t)hmaster.size());
    }
    if (n > INT32_MAX) return gls_io_set_error(GLS_EINVAL, "too many nodes for int32 ids");
    return GLS_OK;
  };
  int rc = number(k, F.cell_vnodes, F.vnode_x, F.vnode_bid, F.vh_node, F.vh_off, F.vh_master, F.vh_w);
  if (rc) return rc;
  if (kp == k) {
    F.cell_pnodes = F.cell_vnodes;
    F.pnode_x = F.vnode_x;
    F.pnode_bid = F.vnode_bid;
    F.ph_node = F.vh_node;
    F.ph_off = F.vh_off;
    F.ph_master = F.vh_master;
    F.ph_w = F.vh_w;
  } else {
    rc = number(kp, F.cell_pnodes, F.pnode_x, F.pnode_bid, F.ph_node, F.ph_off, F.ph_master, F.ph_w);
    if (rc) return rc;
  }
  // hierarchy snapshot (levels, ids, topology for transfers and Kelly faces)
  F.cell_level.resize((size_t)nc);
  F.hid.resize((size_t)nc);
  for (int64_t c = 0; c < nc; ++c) {
    const int64_t h = m.tree.empty() ? c : m.active[(size_t)c];
    F.hid[(size_t)c] = h;
    F.cell_level[(size_t)c] = m.tree.empty() ? 0 : m.tree[(size_t)h].level;
  }
  for (const auto &h : m.tree) {
    F.t_parent.push_back(h.parent);
    F.t_child0.push_back(h.child0);
    F.t_pos.push_back(h.pos);
  }
  F.cell_verts = m.cells;
  for (const auto &h : m.tree) F.t_verts.push_back(h.v);
  F.face_bid.assign((size_t)(nc * 2 * dim), -1);
  for (int64_t c = 0; c < nc; ++c)
    for (int f = 0; f < 2 * dim; ++f) {
      auto b = m.bface.find(face_key_v(dim, m.cells[(size_t)c], f / 2, f & 1));
      if (b != m.bface.end()) F.face_bid[(size_t)(c * 2 * dim + f)] = b->second;
    }
  F.verts = m.X;
  F.periodic.clear();
  for (int p = 0; p < nper; ++p) F.periodic.push_back({per[3 * p], per[3 * p + 1], per[3 * p + 2]});
  F.line_mid = m.line_mid;
  F.face_mid = m.face_mid;
  auto &P = F.pub;
  P.dim = dim;
  P.k = k;
  P.kp = kp;
  P.n_cells = nc;
  P.n_vnodes = (int64_t)F.vnode_bid.size();
  P.n_pnodes = (int64_t)F.pnode_bid.size();
  P.cell_vnodes = F.cell_vnodes.data();
  P.cell_pnodes = F.cell_pnodes.data();
  P.vnode_x = F.vnode_x.data();
  P.pnode_x = F.pnode_x.data();
  P.vnode_bid = F.vnode_bid.data();
  P.pnode_bid = F.pnode_bid.data();
  P.cell_support = F.cell_support.data();
  P.cell_mapping = F.cell_mapping.data();
  P.cell_measure = F.cell_measure.data();
  P.volume = volume;
  P.cell_level = F.cell_level.data();
  P.n_vhang = (int64_t)F.vh_node.size();
  P.vhang_node = F.vh_node.data();
  P.vhang_off = F.vh_off.data();
  P.vhang_master = F.vh_master.data();
  P.vhang_w = F.vh_w.data();
  P.n_phang = (int64_t)F.ph_node.size();
  P.phang_node = F.ph_node.data();
  P.phang_off = F.ph_off.data();
  P.phang_master = F.ph_master.data();
  P.phang_w = F.ph_w.data();
  P.impl_ = &F;
  return GLS_OK;
}

}  // namespace

// ---- Kelly face-piece geometry helpers (gls_fe_space_kelly_faces)
namespace {
void gauss01(int n, double *x, double *w) {
  for (int i = 0; i < n; ++i) {
    double z = std::cos(M_PI * (i + 0.75) / (n + 0.5)), dp = 1.0;
    for (int it = 0; it < 100; ++it) {
      double p0 = 1.0, p1 = 0.0;
      for (int j = 1; j <= n; ++j) {
        const double p2 = p1;
        p1 = p0;
        p0 = ((2.0 * j - 1.0) * z * p1 - (j - 1.0) * p2) / j;
      }
      dp = n * (z * p0 - p1) / (z * z - 1.0);
      const double dz = p0 / dp;
      z -= dz;
      if (std::fabs(dz) < 1e-16) break;
    }
    x[n - 1 - i] = 0.5 * (1.0 + z);
    w[n - 1 - i] = 1.0 / ((1.0 - z * z) * dp * dp);
  }
}
void lagd1(int k, int a, double x, double &v, double &dv) {  // equidistant Lagrange basis and derivative
  v = 1.0;
  dv = 0.0;
  for (int b = 0; b <= k; ++b) {
    if (b == a) continue;
    const double inv = 1.0 / ((double)(a - b) / k);
    dv = dv * (x - (double)b / k) * inv + v * inv;
    v *= (x - (double)b / k) * inv;
  }
}
// J[i][a] = d x_i / d xi_a of the cell's MappingQ (support points at the FE_Q(k) lattice)
void jacobian(const gls_fe_space &S, int64_t c, const double *xi, double J[3][3]) {
  const int dim = S.dim, k = S.k, k1 = k + 1, nl = dim == 2 ? k1 * k1 : k1 * k1 * k1;
  double v[3][4], dv[3][4];
  for (int d = 0; d < dim; ++d)
    for (int a = 0; a <= k; ++a) lagd1(k, a, xi[d], v[d][a], dv[d][a]);
  for (int i = 0; i < 3; ++i)
    for (int a = 0; a < 3; ++a) J[i][a] = (i == a && i >= dim) ? 1.0 : 0.0;
  for (int b = 0; b < nl; ++b) {
    const int ib[3] = {b % k1, (b / k1) % k1, b / (k1 * k1)};
    const double *x = S.cell_support + ((size_t)c * nl + b) * dim;
    for (int a = 0; a < dim; ++a) {
      double t = dv[a][ib[a]];
      for (int o = 0; o < dim; ++o)
        if (o != a) t *= v[o][ib[o]];
      for (int i = 0; i < dim; ++i) J[i][a] += t * x[i];
    }
  }
}
// y = J^-1 r
void solve3(const double J[3][3], const double *r, double *y, int dim) {
  if (dim == 2) {
    const double det = J[0][0] * J[1][1] - J[0][1] * J[1][0];
    y[0] = (J[1][1] * r[0] - J[0][1] * r[1]) / det;
    y[1] = (-J[1][0] * r[0] + J[0][0] * r[1]) / det;
    return;
  }
  const double det = J[0][0] * (J[1][1] * J[2][2] - J[1][2] * J[2][1]) - J[0][1] * (J[1][0] * J[2][2] - J[1][2] * J[2][0]) +
                     J[0][2] * (J[1][0] * J[2][1] - J[1][1] * J[2][0]);
  double inv[3][3];
  inv[0][0] = (J[1][1] * J[2][2] - J[1][2] * J[2][1]) / det;
  inv[0][1] = (J[0][2] * J[2][1] - J[0][1] * J[2][2]) / det;
  inv[0][2] = (J[0][1] * J[1][2] - J[0][2] * J[1][1]) / det;
  inv[1][0] = (J[1][2] * J[2][0] - J[1][0] * J[2][2]) / det;
  inv[1][1] = (J[0][0] * J[2][2] - J[0][2] * J[2][0]) / det;
  inv[1][2] = (J[0][2] * J[1][0] - J[0][0] * J[1][2]) / det;
  inv[2][0] = (J[1][0] * J[2][1] - J[1][1] * J[2][0]) / det;
  inv[2][1] = (J[0][1] * J[2][0] - J[0][0] * J[2][1]) / det;
  inv[2][2] = (J[0][0] * J[1][1] - J[0][1] * J[1][0]) / det;
  for (int i = 0; i < 3; ++i) y[i] = inv[i][0] * r[0] + inv[i][1] * r[1] + inv[i][2] * r[2];
}
}  // namespace

struct gls_umesh {
  UMesh m;
};

extern "C" {

int gls_umesh_generate(int dim, const char *grid_type, const char *grid_arguments, gls_umesh **out) {
  if (!out || !grid_type || (dim != 2 && dim != 3)) return gls_io_set_error(GLS_EINVAL, "gls_umesh_generate: arguments");
  *out = nullptr;
  auto *g = new gls_umesh;
  g->m.dim = dim;
  const int rc = generate(g->m, grid_type, grid_arguments ? grid_arguments : "");
  if (rc) {
    delete g;
    return rc;
  }
  init_tree(g->m);
  *out = g;
  return GLS_OK;
}

int gls_umesh_read_gmsh(int dim, const char *path, gls_umesh **out) {
  if (!out || !path || (dim != 2 && dim != 3)) return gls_io_set_error(GLS_EINVAL, "gls_umesh_read_gmsh: arguments");
  *out = nullptr;
  auto *g = new gls_umesh;
  g->m.dim = dim;
  const int rc = read_gmsh(g->m, path);
  if (rc) {
    delete g;
    return rc;
  }
  init_tree(g->m);
  *out = g;
  return GLS_OK;
}

int gls_umesh_set_manifold(gls_umesh *g, int manifold_id, int type, const double *center, const double *axis) {
  if (!g || manifold_id < 0 || type < 0 || type > 2) return gls_io_set_error(GLS_EINVAL, "gls_umesh_set_manifold: arguments");
  ManifoldDesc md;
  md.type = type;
  if (center)
    for (int d = 0; d < 3; ++d) md.center[d] = d < g->m.dim ? center[d] : 0.0;
  if (axis && type == MF_CYLINDRICAL) {
    V3 a{axis[0], axis[1], axis[2]};
    const double n = nrm(a);
    if (n == 0) return gls_io_set_error(GLS_EINVAL, "gls_umesh_set_manifold: zero axis");
    md.axis = scl(a, 1.0 / n);
  }
  g->m.mf[manifold_id] = md;
  return GLS_OK;
}

// Triangulation::set_all_manifold_ids_on_boundary(boundary_id, manifold_id): the faces with that
// boundary id and (3D) their lines
int gls_umesh_boundary_manifold(gls_umesh *g, int boundary_id, int manifold_id) {
  if (!g) return gls_io_set_error(GLS_EINVAL, "null mesh");
  UMesh &m = g->m;
  for (size_t c = 0; c < m.cells.size(); ++c)
    for (int d = 0; d < m.dim; ++d)
      for (int s = 0; s < 2; ++s) {
        const EKey fk = face_key(m, c, d, s);
        auto b = m.bface.find(fk);
        if (b == m.bface.end() || b->second != boundary_id) continue;
        const auto fv = face_verts(m.dim, d, s);
        if (m.dim == 2) {
          m.line_mf[fk] = manifold_id;
        } else {
          m.face_mf[fk] = manifold_id;
          for (auto &ln : local_lines(3))
            if (std::find(fv.begin(), fv.end(), ln[0]) != fv.end() && std::find(fv.begin(), fv.end(), ln[1]) != fv.end())
              m.line_mf[mkey({m.cells[c][ln[0]], m.cells[c][ln[1]]})] = manifold_id;
        }
      }
  return GLS_OK;
}

int gls_umesh_refine_global(gls_umesh *g, int times) {
  if (!g || times < 0) return gls_io_set_error(GLS_EINVAL, "gls_umesh_refine_global: arguments");
  for (int t = 0; t < times; ++t) {
    const int rc = refine_once(g->m);
    if (rc) return rc;
  }
  return GLS_OK;
}

int gls_umesh_info(const gls_umesh *g, int64_t *n_cells, int64_t *n_vertices, double *volume) {
  if (!g) return gls_io_set_error(GLS_EINVAL, "null mesh");
  if (n_cells) *n_cells = (int64_t)g->m.cells.size();
  if (n_vertices) *n_vertices = (int64_t)g->m.X.size();
  if (volume) {
    double v = 0;
    for (auto &cv : g->m.cells) v += cell_measure(g->m, cv);
    *volume = v;
  }
  return GLS_OK;
}

void gls_umesh_destroy(gls_umesh *g) { delete g; }

int gls_umesh_fe_space(const gls_umesh *g, int k, int kp, int qmapping_all, int n_periodic, const int32_t *periodic,
                       gls_fe_space **out) {
  if (!g || !out || n_periodic < 0 || (n_periodic > 0 && !periodic)) return gls_io_set_error(GLS_EINVAL, "gls_umesh_fe_space: arguments");
  *out = nullptr;
  auto *F = new FESpaceImpl;
  const int rc = build_fe_space(g->m, k, kp, qmapping_all, n_periodic, periodic, *F);
  if (rc) {
    delete F;
    return rc;
  }
  *out = &F->pub;
  return GLS_OK;
}

int gls_fe_space_destroy(gls_fe_space *s) {
  if (s) delete static_cast<FESpaceImpl *>(s->impl_);
  return GLS_OK;
}

// SolutionTransfer::interpolate (navier_stokes_base.cc:689-780) between two FE spaces of the same
// triangulation (refinement, coarsening, any number of levels). Every new active cell is found in
// the old mesh through the hierarchy: unchanged (nodal copy), a descendant of an old active cell
// (the old cell's Qk / Qkp interpolant at the node's reference position in it, exact because Qk on
// children contains the parent's Qk), or an ancestor of old active cells (each node evaluated in the
// old descendant that contains its reference position: FE_Q restriction is interpolation).
int gls_fe_space_transfer(const gls_fe_space *co, const gls_fe_space *fi, const double *cvec, double *fvec) {
  if (!co || !fi || !cvec || !fvec || co->dim != fi->dim || co->k != fi->k || co->kp != fi->kp)
    return gls_io_set_error(GLS_EINVAL, "gls_fe_space_transfer: spaces of different dimension / degree");
  if (!co->impl_ || !fi->impl_) return gls_io_set_error(GLS_EINVAL, "gls_fe_space_transfer: spaces from gls_umesh_fe_space required");
  const FESpaceImpl &O = *static_cast<const FESpaceImpl *>(co->impl_);
  const FESpaceImpl &N = *static_cast<const FESpaceImpl *>(fi->impl_);
  if (O.t_parent.size() > N.t_parent.size())
    return gls_io_set_error(GLS_EINVAL, "gls_fe_space_transfer: the new space must come from the same (later) triangulation");
  const int dim = co->dim;
  std::unordered_map<int64_t, int64_t> old_of;  // hierarchy id -> old active cell
  for (int64_t c = 0; c < co->n_cells; ++c) old_of[O.hid[(size_t)c]] = c;
  const int64_t voc = (int64_t)dim * co->n_vnodes, vof = (int64_t)dim * fi->n_vnodes;
  for (int pass = 0; pass < 2; ++pass) {
    const int kk = pass == 0 ? co->k : co->kp, kk1 = kk + 1, nn = dim == 2 ? kk1 * kk1 : kk1 * kk1 * kk1;
    const int32_t *cc = pass == 0 ? co->cell_vnodes : co->cell_pnodes, *fc = pass == 0 ? fi->cell_vnodes : fi->cell_pnodes;
    const int ncomp = pass == 0 ? dim : 1;
    auto eval = [&](int64_t oc, const double *xi, double *val) {
      for (int e = 0; e < ncomp; ++e) val[e] = 0.0;
      for (int b = 0; b < nn; ++b) {
        const int ib[3] = {b % kk1, (b / kk1) % kk1, dim == 3 ? b / (kk1 * kk1) : 0};
        double w = 1.0;
        for (int d = 0; d < dim; ++d) w *= lag1(kk, ib[d], xi[d]);
        if (w == 0.0) continue;
        const int64_t node = cc[oc * nn + b];
        for (int e = 0; e < ncomp; ++e) val[e] += w * cvec[pass == 0 ? node * dim + e : voc + node];
      }
    };
    for (int64_t f = 0; f < fi->n_cells; ++f) {
      const int64_t h = N.hid[(size_t)f];
      // ancestor chain up to an old active cell (refinement or unchanged)
      int64_t anc = h;
      std::vector<int> path;
      while (anc >= 0 && !old_of.count(anc)) {
        path.push_back(N.t_pos[(size_t)anc]);
        anc = N.t_parent[(size_t)anc];
      }
      for (int a = 0; a < nn; ++a) {
        const int ia[3] = {a % kk1, (a / kk1) % kk1, dim == 3 ? a / (kk1 * kk1) : 0};
        double xi[3] = {0, 0, 0}, val[3] = {0, 0, 0};
        for (int d = 0; d < dim; ++d) xi[d] = (double)ia[d] / kk;
        int64_t oc;
        if (anc >= 0) {
          for (int pos : path)  // child -> parent reference coordinates
            for (int d = 0; d < dim; ++d) xi[d] = 0.5 * (xi[d] + ((pos >> d) & 1));
          oc = old_of[anc];
        } else {  // coarsened: descend the old hierarchy from the new cell
          int64_t c = h;
          int guard = 0;
          while (!old_of.count(c)) {
            if ((size_t)c >= O.t_child0.size() || O.t_child0[(size_t)c] < 0 || ++guard > 64)
              return gls_io_set_error(GLS_EINVAL, "gls_fe_space_transfer: cell %lld not found in the old mesh", (long long)h);
            int ch = 0;
            for (int d = 0; d < dim; ++d) {
              const int bit = xi[d] > 0.5 ? 1 : 0;
              ch |= bit << d;
              xi[d] = 2 * xi[d] - bit;
            }
            c = O.t_child0[(size_t)c] + ch;
          }
          oc = old_of[c];
        }
        eval(oc, xi, val);
        const int64_t fn = fc[f * nn + a];
        for (int e = 0; e < ncomp; ++e) fvec[pass == 0 ? fn * dim + e : vof + fn] = val[e];
      }
    }
  }
  return GLS_OK;
}

// Level meshes of a geometric multigrid on the triangulation's refinement hierarchy (global coarsening):
// a copy whose active cells are the current ones with every cell finer than `level` replaced by its
// ancestor on `level` (depth-first order kept; the 2:1 balance survives truncation). Its FE spaces
// (gls_umesh_fe_space) share the hierarchy ids of the original's, which gls_fe_space_mg_transfer uses.
int gls_umesh_coarsen_to(const gls_umesh *g, int level, gls_umesh **out) {
  if (!g || !out || level < 0) return gls_io_set_error(GLS_EINVAL, "gls_umesh_coarsen_to: arguments");
  auto *r = new gls_umesh(*g);
  UMesh &m = r->m;
  if (!m.tree.empty()) {
    std::vector<int64_t> act;
    std::unordered_map<int64_t, char> seen;
    for (int64_t h : g->m.active) {
      int64_t a = h;
      while (m.tree[(size_t)a].level > level && m.tree[(size_t)a].parent >= 0) a = m.tree[(size_t)a].parent;
      if (seen.emplace(a, 1).second) act.push_back(a);
    }
    m.active = act;
    m.cells.resize(act.size());
    m.cell_mf.resize(act.size());
    for (size_t i = 0; i < act.size(); ++i) {
      m.cells[i] = m.tree[(size_t)act[i]].v;
      m.cell_mf[i] = m.tree[(size_t)act[i]].mf;
    }
  }
  *out = r;
  return GLS_OK;
}

// Prolongation between the FE spaces of two levels of one hierarchy (coarse from gls_umesh_coarsen_to of
// the fine space's triangulation): fine DoF i = sum_j P_ij coarse DoF j = the coarse field (its hanging
// nodes replaced by their lines) at the fine node's reference position in its coarse ancestor cell --
// FE_Q's embedding (child -> parent reference coordinates), independent of the mapping, as
// SolutionTransfer interpolates (gls_fe_space_transfer). Rows of fine hanging DoFs are empty; columns are
// coarse masters. inject[j] = the fine DoF at coarse DoF j's node (descending the hierarchy to the fine
// cell holding it). off == NULL: nnz only.
// p-level pair (same active cells, the coarse space of lower degree, e.g. Q2-Q1 -> Q1-Q1 on the base mesh of a
// hierarchy): fine DoF i = the coarse degree's interpolant at the fine node's reference position in the same cell
// (FE_Q's embedding of the lower degree), hanging coarse nodes replaced by their lines; inject[j] = the fine DoF at
// coarse DoF j's node (the fine degree a multiple of the coarse one).
static int p_level_transfer(const gls_fe_space *fi, const gls_fe_space *co, int64_t *nnz, int64_t *off, int32_t *col,
                            double *w, int64_t *inject) {
  const int dim = fi->dim;
  const int64_t nvf = fi->n_vnodes, nvc = co->n_vnodes;
  const bool fsep = fi->kp != fi->k, csep = co->kp != co->k;
  std::vector<int64_t> inj((size_t)(dim * nvc + co->n_pnodes), -1);
  std::vector<int32_t> cols;
  std::vector<double> ws;
  std::vector<int64_t> roff{0};
  for (int pass = 0; pass < 2; ++pass) {
    const bool vel = pass == 0;
    const int kf = vel ? fi->k : fi->kp, kc = vel ? co->k : co->kp;
    if (kf % kc) return gls_io_set_error(GLS_EINVAL, "gls_fe_space_mg_transfer: degree %d is not a multiple of %d", kf, kc);
    const int kf1 = kf + 1, kc1 = kc + 1;
    const int nnf_c = dim == 2 ? kf1 * kf1 : kf1 * kf1 * kf1, nnc_c = dim == 2 ? kc1 * kc1 : kc1 * kc1 * kc1;
    // node arrays of the field: separate pressure nodes when the space has them, else the velocity nodes
    const int32_t *fcn = (vel || !fsep) ? fi->cell_vnodes : fi->cell_pnodes;
    const int32_t *ccn = (vel || !csep) ? co->cell_vnodes : co->cell_pnodes;
    const int fstride = (vel || !fsep) ? (dim == 2 ? (fi->k + 1) * (fi->k + 1) : (fi->k + 1) * (fi->k + 1) * (fi->k + 1)) : nnf_c;
    const int cstride = (vel || !csep) ? (dim == 2 ? (co->k + 1) * (co->k + 1) : (co->k + 1) * (co->k + 1) * (co->k + 1)) : nnc_c;
    const int64_t nnf = vel ? nvf : (fsep ? fi->n_pnodes : nvf);
    const int64_t nh_c = vel ? co->n_vhang : co->n_phang, nh_f = vel ? fi->n_vhang : fi->n_phang;
    const int64_t *hc_node = vel ? co->vhang_node : co->phang_node, *hc_off = vel ? co->vhang_off : co->phang_off;
    const int64_t *hc_mas = vel ? co->vhang_master : co->phang_master;
    const double *hc_w = vel ? co->vhang_w : co->phang_w;
    const int64_t *hf_node = vel ? fi->vhang_node : fi->phang_node;
    std::unordered_map<int64_t, int64_t> cline;
    for (int64_t i = 0; i < nh_c; ++i) cline[hc_node[i]] = i;
    std::vector<char> fh((size_t)nnf, 0), seen((size_t)nnf, 0);
    for (int64_t i = 0; i < nh_f; ++i) fh[(size_t)hf_node[i]] = 1;
    std::vector<std::vector<std::pair<int32_t, double>>> rows((size_t)nnf);
    // the fine field's local nodes: the degree-kf lattice of a node array with degree (vel || !fsep ? k : kp)
    const int kfa = (vel || !fsep) ? fi->k : fi->kp, kca = (vel || !csep) ? co->k : co->kp;
    if (kfa != kf || kca != kc) return gls_io_set_error(GLS_EINVAL, "gls_fe_space_mg_transfer: equal-order pressure degree");
    for (int64_t f = 0; f < fi->n_cells; ++f) {
      for (int a = 0; a < nnf_c; ++a) {
        const int64_t node = fcn[f * fstride + a];
        if (seen[(size_t)node] || fh[(size_t)node]) continue;
        seen[(size_t)node] = 1;
        const int ia[3] = {a % kf1, (a / kf1) % kf1, dim == 3 ? a / (kf1 * kf1) : 0};
        auto &acc = rows[(size_t)node];
        for (int b = 0; b < nnc_c; ++b) {
          const int ib[3] = {b % kc1, (b / kc1) % kc1, dim == 3 ? b / (kc1 * kc1) : 0};
          double wb = 1.0;
          for (int d = 0; d < dim; ++d) wb *= lag1(kc, ib[d], (double)ia[d] / kf);
          if (std::fabs(wb) < 1e-14) continue;
          const int64_t cn = ccn[f * cstride + b];
          auto it = cline.find(cn);
          if (it == cline.end()) acc.push_back({(int32_t)cn, wb});
          else
            for (int64_t q = hc_off[it->second]; q < hc_off[it->second + 1]; ++q) acc.push_back({(int32_t)hc_mas[q], wb * hc_w[q]});
        }
        std::sort(acc.begin(), acc.end(), [](const std::pair<int32_t, double> &x, const std::pair<int32_t, double> &y) {
          return x.first < y.first;
        });
        size_t m = 0;
        for (size_t i = 0; i < acc.size(); ++i) {
          if (m > 0 && acc[m - 1].first == acc[i].first) acc[m - 1].second += acc[i].second;
          else acc[m++] = acc[i];
        }
        acc.resize(m);
      }
      for (int b = 0; b < nnc_c; ++b) {  // injection: coarse node b sits on fine local node (kf / kc) * ib
        const int ib[3] = {b % kc1, (b / kc1) % kc1, dim == 3 ? b / (kc1 * kc1) : 0};
        int la = 0, st = 1;
        for (int d = 0; d < dim; ++d) {
          la += ib[d] * (kf / kc) * st;
          st *= kf1;
        }
        const int64_t cnode = ccn[f * cstride + b], fnode = fcn[f * fstride + la];
        if (vel)
          for (int e = 0; e < dim; ++e) inj[(size_t)(cnode * dim + e)] = fnode * dim + e;
        else
          inj[(size_t)(dim * nvc + cnode)] = dim * nvf + fnode;
      }
    }
    for (int64_t v = 0; v < nnf; ++v) {
      const int nrow = vel ? dim : 1;
      for (int c = 0; c < nrow; ++c) {
        for (auto &e : rows[(size_t)v]) {
          cols.push_back(vel ? (int32_t)(e.first * dim + c) : (int32_t)(dim * nvc + e.first));
          ws.push_back(e.second);
        }
        roff.push_back((int64_t)cols.size());
      }
    }
  }
  *nnz = (int64_t)cols.size();
  if (off) {
    if (!col || !w) return gls_io_set_error(GLS_EINVAL, "gls_fe_space_mg_transfer: col / w missing");
    std::memcpy(off, roff.data(), sizeof(int64_t) * roff.size());
    std::memcpy(col, cols.data(), sizeof(int32_t) * cols.size());
    std::memcpy(w, ws.data(), sizeof(double) * ws.size());
  }
  if (inject) std::memcpy(inject, inj.data(), sizeof(int64_t) * inj.size());
  return GLS_OK;
}

int gls_fe_space_mg_transfer(const gls_fe_space *fi, const gls_fe_space *co, int64_t *nnz, int64_t *off, int32_t *col,
                             double *w, int64_t *inject) {
  if (fi && co && nnz && fi->dim == co->dim && fi->impl_ && co->impl_ && (fi->k != co->k || fi->kp != co->kp)) {
    const FESpaceImpl &N = *static_cast<const FESpaceImpl *>(fi->impl_);
    const FESpaceImpl &O = *static_cast<const FESpaceImpl *>(co->impl_);
    if (fi->n_cells != co->n_cells || N.hid != O.hid || co->k > fi->k || co->kp > fi->kp)
      return gls_io_set_error(GLS_EINVAL, "gls_fe_space_mg_transfer: a p-level pair needs the same cells and a "
                                          "coarse space of lower degree");
    return p_level_transfer(fi, co, nnz, off, col, w, inject);
  }
  if (!fi || !co || !nnz || fi->dim != co->dim || fi->k != co->k || fi->kp != co->kp || !fi->impl_ || !co->impl_)
    return gls_io_set_error(GLS_EINVAL, "gls_fe_space_mg_transfer: spaces of different dimension / degree");
  const FESpaceImpl &N = *static_cast<const FESpaceImpl *>(fi->impl_);
  const FESpaceImpl &O = *static_cast<const FESpaceImpl *>(co->impl_);
  if (N.t_parent.size() != O.t_parent.size())
    return gls_io_set_error(GLS_EINVAL, "gls_fe_space_mg_transfer: the spaces are not levels of one hierarchy");
  const int dim = fi->dim;
  std::unordered_map<int64_t, int64_t> cof, fof;  // hierarchy id -> active cell
  for (int64_t c = 0; c < co->n_cells; ++c) cof[O.hid[(size_t)c]] = c;
  for (int64_t f = 0; f < fi->n_cells; ++f) fof[N.hid[(size_t)f]] = f;
  const int64_t nvf = fi->n_vnodes, nvc = co->n_vnodes;
  std::vector<int64_t> inj((size_t)(dim * nvc + co->n_pnodes), -1);
  std::vector<int32_t> cols;
  std::vector<double> ws;
  std::vector<int64_t> roff{0};
  for (int pass = 0; pass < 2; ++pass) {
    const bool vel = pass == 0;
    const int kk = vel ? fi->k : fi->kp, kk1 = kk + 1, nn = dim == 2 ? kk1 * kk1 : kk1 * kk1 * kk1;
    const int32_t *ccn = vel ? co->cell_vnodes : co->cell_pnodes, *fcn = vel ? fi->cell_vnodes : fi->cell_pnodes;
    const int64_t nnf = vel ? nvf : fi->n_pnodes, nnc = vel ? nvc : co->n_pnodes;
    const int64_t nh_c = vel ? co->n_vhang : co->n_phang, nh_f = vel ? fi->n_vhang : fi->n_phang;
    const int64_t *hc_node = vel ? co->vhang_node : co->phang_node, *hc_off = vel ? co->vhang_off : co->phang_off;
    const int64_t *hc_mas = vel ? co->vhang_master : co->phang_master;
    const double *hc_w = vel ? co->vhang_w : co->phang_w;
    const int64_t *hf_node = vel ? fi->vhang_node : fi->phang_node;
    std::unordered_map<int64_t, int64_t> cline;
    for (int64_t i = 0; i < nh_c; ++i) cline[hc_node[i]] = i;
    std::vector<char> fh((size_t)nnf, 0), seen((size_t)nnf, 0);
    for (int64_t i = 0; i < nh_f; ++i) fh[(size_t)hf_node[i]] = 1;
    std::vector<std::vector<std::pair<int32_t, double>>> rows((size_t)nnf);
    for (int64_t f = 0; f < fi->n_cells; ++f) {
      int64_t anc = N.hid[(size_t)f];
      std::vector<int> path;
      while (anc >= 0 && !cof.count(anc)) {
        path.push_back(N.t_pos[(size_t)anc]);
        anc = N.t_parent[(size_t)anc];
      }
      if (anc < 0) return gls_io_set_error(GLS_EINVAL, "gls_fe_space_mg_transfer: fine cell %lld has no coarse ancestor", (long long)f);
      const int64_t oc = cof[anc];
      for (int a = 0; a < nn; ++a) {
        const int64_t node = fcn[f * nn + a];
        if (seen[(size_t)node] || fh[(size_t)node]) continue;
        seen[(size_t)node] = 1;
        const int ia[3] = {a % kk1, (a / kk1) % kk1, dim == 3 ? a / (kk1 * kk1) : 0};
        double xi[3] = {0, 0, 0};
        for (int d = 0; d < dim; ++d) xi[d] = (double)ia[d] / kk;
        for (int pos : path)
          for (int d = 0; d < dim; ++d) xi[d] = 0.5 * (xi[d] + ((pos >> d) & 1));
        auto &acc = rows[(size_t)node];
        for (int b = 0; b < nn; ++b) {
          const int ib[3] = {b % kk1, (b / kk1) % kk1, dim == 3 ? b / (kk1 * kk1) : 0};
          double wb = 1.0;
          for (int d = 0; d < dim; ++d) wb *= lag1(kk, ib[d], xi[d]);
          if (std::fabs(wb) < 1e-14) continue;
          const int64_t cn = ccn[oc * nn + b];
          auto it = cline.find(cn);
          if (it == cline.end()) {
            acc.push_back({(int32_t)cn, wb});
          } else {
            for (int64_t q = hc_off[it->second]; q < hc_off[it->second + 1]; ++q) acc.push_back({(int32_t)hc_mas[q], wb * hc_w[q]});
          }
        }
        std::sort(acc.begin(), acc.end(), [](const std::pair<int32_t, double> &x, const std::pair<int32_t, double> &y) {
          return x.first < y.first;
        });
        size_t m = 0;
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
    }
    for (int64_t v = 0; v < nnf; ++v) {
      const int nrow = vel ? dim : 1;
      for (int c = 0; c < nrow; ++c) {
        for (auto &e : rows[(size_t)v]) {
          cols.push_back(vel ? (int32_t)(e.first * dim + c) : (int32_t)(dim * nvc + e.first));
          ws.push_back(e.second);
        }
        roff.push_back((int64_t)cols.size());
      }
    }
    // injection: each coarse node's position, descended to the fine active cell holding it
    std::vector<char> done((size_t)nnc, 0);
    for (int64_t oc = 0; oc < co->n_cells; ++oc)
      for (int b = 0; b < nn; ++b) {
        const int64_t cnode = ccn[oc * nn + b];
        if (done[(size_t)cnode]) continue;
        done[(size_t)cnode] = 1;
        double xi[3] = {0, 0, 0};
        const int ib[3] = {b % kk1, (b / kk1) % kk1, dim == 3 ? b / (kk1 * kk1) : 0};
        for (int d = 0; d < dim; ++d) xi[d] = (double)ib[d] / kk;
        int64_t c = O.hid[(size_t)oc];
        int guard = 0;
        while (!fof.count(c)) {
          if ((size_t)c >= N.t_child0.size() || N.t_child0[(size_t)c] < 0 || ++guard > 64)
            return gls_io_set_error(GLS_EINVAL, "gls_fe_space_mg_transfer: coarse cell %lld not refined into the fine mesh", (long long)oc);
          int ch = 0;
          for (int d = 0; d < dim; ++d) {
            const int bit = xi[d] > 0.5 ? 1 : 0;
            ch |= bit << d;
            xi[d] = 2 * xi[d] - bit;
          }
          c = N.t_child0[(size_t)c] + ch;
        }
        const int64_t f = fof[c];
        int la = 0, st = 1;
        for (int d = 0; d < dim; ++d) {
          const double q = xi[d] * kk;
          const int iq = (int)std::lround(q);
          if (std::fabs(q - iq) > 1e-9) return gls_io_set_error(GLS_EINVAL, "gls_fe_space_mg_transfer: coarse node not a fine node");
          la += iq * st;
          st *= kk1;
        }
        const int64_t fnode = fcn[f * nn + la];
        if (vel)
          for (int e = 0; e < dim; ++e) inj[(size_t)(cnode * dim + e)] = fnode * dim + e;
        else
          inj[(size_t)(dim * nvc + cnode)] = dim * nvf + fnode;
      }
  }
  *nnz = (int64_t)cols.size();
  if (off) {
    if (!col || !w) return gls_io_set_error(GLS_EINVAL, "gls_fe_space_mg_transfer: col / w missing");
    std::memcpy(off, roff.data(), sizeof(int64_t) * roff.size());
    std::memcpy(col, cols.data(), sizeof(int32_t) * cols.size());
    std::memcpy(w, ws.data(), sizeof(double) * ws.size());
  }
  if (inject) std::memcpy(inject, inj.data(), sizeof(int64_t) * inj.size());
  return GLS_OK;
}

// Face pieces of KellyErrorEstimator::estimate with a MappingQ (navier_stokes_base.cc:612-652;
// deal.II 9.2 error_estimator.cc, third party, restated): every interior face between two active
// cells of the same level is one piece; on a face between an active cell and a refined neighbour
// each child face is a piece (integrate_over_irregular_face), its geometry (normal, JxW) taken on the
// coarse cell's subface as deal.II's present cell does. QGauss<dim-1>(nq) on each piece; per point,
// both sides' reference coordinates xi, g = J^-1 n and JxW. cell_diam: cell->diameter() (the longest
// vertex diagonal). Null arrays: count only.
int gls_fe_space_kelly_faces(const gls_fe_space *sp, int nq, int64_t *n_pieces, int32_t *ca, int32_t *cb, double *xi,
                             double *g, double *jxw, double *cell_diam) {
  if (!sp || !sp->impl_ || !n_pieces || nq < 1 || nq > 8) return gls_io_set_error(GLS_EINVAL, "gls_fe_space_kelly_faces: arguments");
  const FESpaceImpl &F = *static_cast<const FESpaceImpl *>(sp->impl_);
  const int dim = sp->dim, nqf = dim == 3 ? nq * nq : nq;
  const int64_t nc = sp->n_cells;
  if (cell_diam)
    for (int64_t c = 0; c < nc; ++c) {
      const auto &cv = F.cell_verts[(size_t)c];
      const int nd = dim == 2 ? 2 : 4, top = (1 << dim) - 1;
      double dm = 0;
      for (int i = 0; i < nd; ++i) dm = std::max(dm, nrm(sub(F.verts[(size_t)cv[i]], F.verts[(size_t)cv[top - i]])));
      cell_diam[c] = dm;
    }
  std::map<EKey, std::vector<std::pair<int64_t, int>>> faces;  // active faces -> (cell, 2d + s)
  for (int64_t c = 0; c < nc; ++c)
    for (int f = 0; f < 2 * dim; ++f) faces[face_key_v(dim, F.cell_verts[(size_t)c], f / 2, f & 1)].push_back({c, f});
  double xq[8], wq[8];
  gauss01(nq, xq, wq);
  auto tang = [&](int d, int *t) {
    int n = 0;
    for (int e = 0; e < dim; ++e)
      if (e != d) t[n++] = e;
  };
  // periodic boundaries (KellyErrorEstimator's periodic neighbours): the active faces on each periodic id
  struct PFace {
    int64_t c;
    int f;
    V3 C[2][2];
  };
  auto face_corners = [&](int64_t c, int f, V3 (&C)[2][2]) {
    const auto &cv = F.cell_verts[(size_t)c];
    const int d = f / 2, s = f & 1;
    int t[2] = {0, 0}, nt = 0;
    for (int e = 0; e < dim; ++e)
      if (e != d) t[nt++] = e;
    for (int iu = 0; iu < 2; ++iu)
      for (int iv = 0; iv < 2; ++iv)
        C[iu][iv] = F.verts[(size_t)cv[(size_t)((s << d) | (iu << t[0]) | (dim == 3 ? iv << t[1] : 0))]];
  };
  std::map<int, std::vector<PFace>> pfaces;
  const double ptol = F.periodic.empty() ? 0.0 : periodic_tol(F.verts);
  for (const auto &pr : F.periodic)
    for (int64_t c = 0; c < nc; ++c)
      for (int f = 0; f < 2 * dim; ++f) {
        const int bid = F.face_bid[(size_t)(c * 2 * dim + f)];
        if (bid != pr[0] && bid != pr[1]) continue;
        PFace pf{c, f, {}};
        face_corners(c, f, pf.C);
        pfaces[bid].push_back(pf);
      }
  int64_t cnt = 0;
  for (int64_t a = 0; a < nc; ++a)
    for (int fa = 0; fa < 2 * dim; ++fa) {
      const auto &av = F.cell_verts[(size_t)a];
      const int da = fa / 2, sa = fa & 1;
      const auto &lst = faces[face_key_v(dim, av, da, sa)];
      int64_t b = -1;
      int fb = -1;
      bool irregular = false, periodic = false;
      std::array<double, 2> Pc[3];  // periodic pieces: a's face corners in b's face parameters
      if (lst.size() == 2) {
        const auto &o = lst[0].first == a ? lst[1] : lst[0];
        if (o.first < a) continue;  // emitted from the other side
        b = o.first;
        fb = o.second;
      } else {
        const int64_t h = F.hid[(size_t)a];
        const int64_t P = F.t_parent.empty() ? -1 : F.t_parent[(size_t)h];
        std::map<EKey, std::vector<std::pair<int64_t, int>>>::const_iterator it = faces.end();
        if (P >= 0 && ((F.t_pos[(size_t)h] >> da) & 1) == sa) it = faces.find(face_key_v(dim, F.t_verts[(size_t)P], da, sa));
        if (it != faces.end() && it->second.size() == 1) {
          b = it->second[0].first;
          fb = it->second[0].second;
          irregular = true;
        } else {  // a boundary face: a piece only across a periodic boundary
          const int bid = F.face_bid[(size_t)(a * 2 * dim + fa)];
          int other = -1, dir = 0;
          for (const auto &pr : F.periodic)
            if (bid == pr[0] || bid == pr[1]) {
              other = bid == pr[0] ? pr[1] : pr[0];
              dir = pr[2];
            }
          if (other < 0) continue;
          V3 Ca[2][2];
          face_corners(a, fa, Ca);
          V3 xc{0, 0, 0};
          for (int iu = 0; iu < 2; ++iu)
            for (int iv = 0; iv < (dim == 3 ? 2 : 1); ++iv) xc = add(xc, scl(Ca[iu][iv], dim == 3 ? 0.25 : 0.5));
          const PFace *hit = nullptr;
          double uv[2];
          for (const auto &pf : pfaces[other])
            if (periodic_face_params(dim, dir, pf.C, xc, ptol, uv)) {
              hit = &pf;
              break;
            }
          if (!hit) return gls_io_set_error(GLS_EINVAL, "Kelly faces: periodic face of cell %lld without a partner", (long long)a);
          b = hit->c;
          fb = hit->f;
          const int la = F.cell_level[(size_t)a], lb = F.cell_level[(size_t)b];
          if (lb > la) continue;                                             // the finer side emits the pieces
          if (lb == la && (b < a || (b == a && fb < fa))) continue;          // emitted from the other side
          irregular = lb < la;
          periodic = true;
          const int cu[3] = {0, 1, 0}, cvv[3] = {0, 0, 1};
          for (int i = 0; i < (dim == 3 ? 3 : 2); ++i) {
            if (!periodic_face_params(dim, dir, hit->C, Ca[cu[i]][cvv[i]], ptol, uv))
              return gls_io_set_error(GLS_EINVAL, "Kelly faces: periodic cells %lld / %lld do not share a face piece",
                                      (long long)a, (long long)b);
            Pc[i] = {uv[0], uv[1]};
          }
        }
      }
      if (!xi) {
        ++cnt;
        continue;
      }
      const int db = fb / 2, sb = fb & 1;
      int ta[2] = {0, 0}, tb[2] = {0, 0};
      tang(da, ta);
      tang(db, tb);
      const auto &bv = F.cell_verts[(size_t)b];
      // b's face lattice: vertex id -> face parameters (corners; with the midpoints when irregular);
      // periodic pieces have theirs from the geometry already
      std::map<int64_t, std::array<double, 2>> par;
      int64_t C[2][2] = {{-1, -1}, {-1, -1}};
      for (int iu = 0; iu < 2; ++iu)
        for (int iv = 0; iv < (dim == 3 ? 2 : 1); ++iv) {
          C[iu][iv] = bv[(size_t)((sb << db) | (iu << tb[0]) | (dim == 3 ? iv << tb[1] : 0))];
          par[C[iu][iv]] = {(double)iu, (double)iv};
        }
      if (irregular) {
        if (dim == 2) {
          auto it = F.line_mid.find(mkey({C[0][0], C[1][0]}));
          if (it != F.line_mid.end()) par[it->second] = {0.5, 0.0};
        } else {
          for (int i = 0; i < 2; ++i) {
            auto e1 = F.line_mid.find(mkey({C[0][i], C[1][i]}));
            if (e1 != F.line_mid.end()) par[e1->second] = {0.5, (double)i};
            auto e2 = F.line_mid.find(mkey({C[i][0], C[i][1]}));
            if (e2 != F.line_mid.end()) par[e2->second] = {(double)i, 0.5};
          }
          auto fc = F.face_mid.find(mkey({C[0][0], C[0][1], C[1][0], C[1][1]}));
          if (fc != F.face_mid.end()) par[fc->second] = {0.5, 0.5};
        }
      }
      // a's face corners (0,0), (1,0), (0,1) in b's face parameters
      const int cu[3] = {0, 1, 0}, cvv[3] = {0, 0, 1};
      for (int i = 0; i < (dim == 3 ? 3 : 2) && !periodic; ++i) {
        const int64_t vid = av[(size_t)((sa << da) | (cu[i] << ta[0]) | (dim == 3 ? cvv[i] << ta[1] : 0))];
        auto it = par.find(vid);
        if (it == par.end()) return gls_io_set_error(GLS_EINVAL, "Kelly faces: cells %lld / %lld do not share a face piece", (long long)a, (long long)b);
        Pc[i] = it->second;
      }
      ca[cnt] = (int32_t)a;
      cb[cnt] = (int32_t)b;
      for (int qb = 0; qb < (dim == 3 ? nq : 1); ++qb)
        for (int qa = 0; qa < nq; ++qa) {
          const int q = qa + nq * qb;
          const double u = xq[qa], v = dim == 3 ? xq[qb] : 0.0, w = wq[qa] * (dim == 3 ? wq[qb] : 1.0);
          double XA[3] = {0, 0, 0}, XB[3] = {0, 0, 0}, TuA[3] = {0, 0, 0}, TvA[3] = {0, 0, 0}, TuB[3] = {0, 0, 0}, TvB[3] = {0, 0, 0};
          XA[da] = sa;
          XA[ta[0]] = u;
          TuA[ta[0]] = 1.0;
          if (dim == 3) {
            XA[ta[1]] = v;
            TvA[ta[1]] = 1.0;
          }
          XB[db] = sb;
          for (int j = 0; j < dim - 1; ++j) {
            XB[tb[j]] = Pc[0][j] + u * (Pc[1][j] - Pc[0][j]) + v * (dim == 3 ? Pc[2][j] - Pc[0][j] : 0.0);
            TuB[tb[j]] = Pc[1][j] - Pc[0][j];
            if (dim == 3) TvB[tb[j]] = Pc[2][j] - Pc[0][j];
          }
          double JA[3][3], JB[3][3];
          jacobian(*sp, a, XA, JA);
          jacobian(*sp, b, XB, JB);
          const auto &JG = irregular ? JB : JA;
          const double *Tu = irregular ? TuB : TuA, *Tv = irregular ? TvB : TvA;
          V3 tu{0, 0, 0}, tv{0, 0, 0};
          for (int i = 0; i < dim; ++i)
            for (int e = 0; e < dim; ++e) {
              tu[i] += JG[i][e] * Tu[e];
              tv[i] += JG[i][e] * Tv[e];
            }
          V3 n;
          double area;
          if (dim == 2) {
            area = nrm(tu);
            n = {tu[1] / area, -tu[0] / area, 0.0};
          } else {
            n = cross(tu, tv);
            area = nrm(n);
            n = scl(n, 1.0 / area);
          }
          jxw[cnt * nqf + q] = area * w;
          double ga[3], gb[3];
          solve3(JA, n.data(), ga, dim);
          solve3(JB, n.data(), gb, dim);
          for (int d = 0; d < dim; ++d) {
            xi[((cnt * nqf + q) * 2 + 0) * dim + d] = XA[d];
            xi[((cnt * nqf + q) * 2 + 1) * dim + d] = XB[d];
            g[((cnt * nqf + q) * 2 + 0) * dim + d] = ga[d];
            g[((cnt * nqf + q) * 2 + 1) * dim + d] = gb[d];
          }
        }
      ++cnt;
    }
  *n_pieces = cnt;
  return GLS_OK;
}

// Node normals of the boundary faces with id `boundary_id` (VectorTools::
// compute_no_normal_flux_constraints, gls_navier_stokes.cc:100-110): at every velocity node on such a
// face, the normalised sum of the adjacent faces' outward unit normals (J^-T e_d of the cell's
// MappingQ at the node); zero elsewhere. normals: [n_vnodes][dim] host array.
int gls_fe_space_boundary_normals(const gls_fe_space *sp, int boundary_id, double *normals) {
  if (!sp || !sp->impl_ || !normals) return gls_io_set_error(GLS_EINVAL, "gls_fe_space_boundary_normals: arguments");
  const FESpaceImpl &F = *static_cast<const FESpaceImpl *>(sp->impl_);
  const int dim = sp->dim, k = sp->k, k1 = k + 1, nn = dim == 2 ? k1 * k1 : k1 * k1 * k1;
  std::fill(normals, normals + sp->n_vnodes * dim, 0.0);
  for (int64_t c = 0; c < sp->n_cells; ++c)
    for (int f = 0; f < 2 * dim; ++f) {
      if (F.face_bid[(size_t)(c * 2 * dim + f)] != boundary_id) continue;
      const int d = f / 2, s = f & 1;
      for (int a = 0; a < nn; ++a) {
        const int ia[3] = {a % k1, (a / k1) % k1, a / (k1 * k1)};
        if (ia[d] != s * k) continue;
        double xi[3] = {0, 0, 0}, J[3][3], e[3] = {0, 0, 0}, n[3] = {0, 0, 0};
        for (int t = 0; t < dim; ++t) xi[t] = (double)ia[t] / k;
        jacobian(*sp, c, xi, J);
        // J^-T e_d = (row d of J^-1)^T: solve J^T y = e_d
        double JT[3][3];
        for (int i = 0; i < 3; ++i)
          for (int j = 0; j < 3; ++j) JT[i][j] = J[j][i];
        e[d] = s ? 1.0 : -1.0;
        solve3(JT, e, n, dim);
        double l = 0;
        for (int t = 0; t < dim; ++t) l += n[t] * n[t];
        l = std::sqrt(l);
        const int64_t node = sp->cell_vnodes[c * nn + a];
        for (int t = 0; t < dim; ++t) normals[node * dim + t] += n[t] / l;
      }
    }
  for (int64_t v = 0; v < sp->n_vnodes; ++v) {
    double l = 0;
    for (int t = 0; t < dim; ++t) l += normals[v * dim + t] * normals[v * dim + t];
    if (l > 0)
      for (int t = 0; t < dim; ++t) normals[v * dim + t] /= std::sqrt(l);
  }
  return GLS_OK;
}

// The independent normal directions at every velocity node of the boundary faces with id
// `boundary_id`, for compute_no_normal_flux_constraints at edges and corners (gls_navier_stokes.cc:
// 100-110): the faces' outward unit normals at the node are grouped (a normal joins the first group
// whose mean direction is within 60 degrees, else it opens a group -- adjacent faces of a smooth
// curved wall share one group, the faces meeting at a box edge or corner do not); the group means
// are orthogonalised (Gram-Schmidt, tolerance 1e-3) and count[v] = the rank (0 off the boundary,
// 1 = one normal, 2 = an edge in 3D, dim = every component constrained). normals: [n_vnodes][3][dim],
// row 0 = the unit mean of the first group (the node normal of gls_fe_space_boundary_normals when
// count = 1), rows 1.. = the other group means (unit, not orthogonalised).
int gls_fe_space_boundary_normal_sets(const gls_fe_space *sp, int boundary_id, int32_t *count, double *normals) {
  if (!sp || !sp->impl_ || !count || !normals)
    return gls_io_set_error(GLS_EINVAL, "gls_fe_space_boundary_normal_sets: arguments");
  const FESpaceImpl &F = *static_cast<const FESpaceImpl *>(sp->impl_);
  const int dim = sp->dim, k = sp->k, k1 = k + 1, nn = dim == 2 ? k1 * k1 : k1 * k1 * k1;
  struct Group {
    double s[3];
  };
  std::vector<std::vector<Group>> groups((size_t)sp->n_vnodes);
  for (int64_t c = 0; c < sp->n_cells; ++c)
    for (int f = 0; f < 2 * dim; ++f) {
      if (F.face_bid[(size_t)(c * 2 * dim + f)] != boundary_id) continue;
      const int d = f / 2, s = f & 1;
      for (int a = 0; a < nn; ++a) {
        const int ia[3] = {a % k1, (a / k1) % k1, a / (k1 * k1)};
        if (ia[d] != s * k) continue;
        double xi[3] = {0, 0, 0}, J[3][3], e[3] = {0, 0, 0}, n[3] = {0, 0, 0}, JT[3][3];
        for (int t = 0; t < dim; ++t) xi[t] = (double)ia[t] / k;
        jacobian(*sp, c, xi, J);
        for (int i = 0; i < 3; ++i)
          for (int j = 0; j < 3; ++j) JT[i][j] = J[j][i];
        e[d] = s ? 1.0 : -1.0;
        solve3(JT, e, n, dim);
        double l = 0;
        for (int t = 0; t < dim; ++t) l += n[t] * n[t];
        l = std::sqrt(l);
        for (int t = 0; t < dim; ++t) n[t] /= l;
        auto &G = groups[(size_t)sp->cell_vnodes[c * nn + a]];
        bool joined = false;
        for (Group &g : G) {
          double gl = 0, dot = 0;
          for (int t = 0; t < dim; ++t) gl += g.s[t] * g.s[t];
          for (int t = 0; t < dim; ++t) dot += g.s[t] * n[t];
          if (dot > 0.5 * std::sqrt(gl)) {
            for (int t = 0; t < dim; ++t) g.s[t] += n[t];
            joined = true;
            break;
          }
        }
        if (!joined) G.push_back(Group{{n[0], n[1], dim == 3 ? n[2] : 0.0}});
      }
    }
  std::fill(normals, normals + sp->n_vnodes * 3 * dim, 0.0);
  for (int64_t v = 0; v < sp->n_vnodes; ++v) {
    const auto &G = groups[(size_t)v];
    double q[3][3] = {};  // orthonormal basis of the group means (rank)
    int r = 0;
    for (size_t i = 0; i < G.size(); ++i) {
      double m[3] = {0, 0, 0}, l = 0;
      for (int t = 0; t < dim; ++t) l += G[i].s[t] * G[i].s[t];
      l = std::sqrt(l);
      for (int t = 0; t < dim; ++t) m[t] = G[i].s[t] / l;
      if (i < 3)
        for (int t = 0; t < dim; ++t) normals[(v * 3 + (int64_t)i) * dim + t] = m[t];
      double w[3] = {m[0], m[1], m[2]};
      for (int j = 0; j < r; ++j) {
        double p = 0;
        for (int t = 0; t < dim; ++t) p += q[j][t] * w[t];
        for (int t = 0; t < dim; ++t) w[t] -= p * q[j][t];
      }
      double wl = 0;
      for (int t = 0; t < dim; ++t) wl += w[t] * w[t];
      wl = std::sqrt(wl);
      if (wl > 1e-3 && r < dim) {
        for (int t = 0; t < dim; ++t) q[r][t] = w[t] / wl;
        ++r;
      }
    }
    count[v] = r;
  }
  return GLS_OK;
}

int gls_umesh_set_periodic(gls_umesh *g, int n_periodic, const int32_t *periodic) {
  if (!g || n_periodic < 0 || (n_periodic > 0 && !periodic)) return gls_io_set_error(GLS_EINVAL, "gls_umesh_set_periodic: arguments");
  g->m.periodic.clear();
  for (int p = 0; p < n_periodic; ++p) {
    const int d = periodic[3 * p + 2];
    if (d < 0 || d >= g->m.dim || periodic[3 * p] == periodic[3 * p + 1])
      return gls_io_set_error(GLS_EINVAL, "gls_umesh_set_periodic: pair %d", p);
    g->m.periodic.push_back({periodic[3 * p], periodic[3 * p + 1], d});
  }
  return GLS_OK;
}

int gls_umesh_adapt(gls_umesh *g, const int32_t *refine, const int32_t *coarsen) {
  if (!g) return gls_io_set_error(GLS_EINVAL, "null mesh");
  return adapt(g->m, refine, coarsen);
}

int gls_umesh_prepare(const gls_umesh *g, int32_t *refine, int32_t *coarsen) {
  if (!g || !refine || !coarsen) return gls_io_set_error(GLS_EINVAL, "gls_umesh_prepare: arguments");
  init_tree(const_cast<UMesh &>(g->m));
  USmoother sm(g->m, refine, coarsen);
  const int loops = sm.run();
  for (size_t i = 0; i < g->m.active.size(); ++i) {
    refine[i] = sm.ref[i];
    coarsen[i] = sm.crs[i];
  }
  return loops;
}

}  // extern "C"
