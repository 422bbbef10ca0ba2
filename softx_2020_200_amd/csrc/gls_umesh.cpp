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
#include <map>
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

// ---- refinement (Triangulation::refine_global, deal.II 9.2 vertex placement)
int refine_once(UMesh &m) {
  const int dim = m.dim, nv = m.nvc(), nch = 1 << dim;
  const auto lines = local_lines(dim);
  std::map<EKey, int64_t> line_mid, face_mid;
  std::vector<std::array<int64_t, 8>> cells;
  std::vector<int> cmf;
  std::map<EKey, int> bface, lmf, fmf;
  cells.reserve(m.cells.size() * nch);
  for (size_t c = 0; c < m.cells.size(); ++c) {
    const auto &cv = m.cells[c];
    const int cellmf = m.cell_mf[c];
    // lattice of 3^dim points: index (i, j, l) in {0,1,2}
    int64_t lat[27];
    auto L = [&](int i, int j, int l) -> int64_t & { return lat[i + 3 * (j + 3 * l)]; };
    for (int v = 0; v < nv; ++v) L(2 * (v & 1), 2 * ((v >> 1) & 1), 2 * ((v >> 2) & 1)) = cv[v];
    // line midpoints
    std::vector<V3> lmid(lines.size());
    for (size_t li = 0; li < lines.size(); ++li) {
      const int a = lines[li][0], b = lines[li][1];
      const EKey k = mkey({cv[a], cv[b]});
      auto it = line_mid.find(k);
      int64_t id;
      if (it == line_mid.end()) {
        const V3 p = new_point(m, m.mf_of(m.line_mf, k), {m.X[(size_t)cv[a]], m.X[(size_t)cv[b]]}, {0.5, 0.5});
        id = (int64_t)m.X.size();
        m.X.push_back(p);
        line_mid[k] = id;
      } else {
        id = it->second;
      }
      lmid[li] = m.X[(size_t)id];
      int q[3];  // lattice: coordinate 1 along the line's direction
      for (int d = 0; d < 3; ++d) q[d] = ((a >> d) & 1) == ((b >> d) & 1) ? 2 * ((a >> d) & 1) : 1;
        L(q[0], q[1], dim > 2 ? q[2] : 0) = id;
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
    std::vector<V3> fmid;
    if (dim == 3) {
      for (int d = 0; d < 3; ++d)
        for (int s = 0; s < 2; ++s) {
          const EKey k = face_key(m, c, d, s);
          auto it = face_mid.find(k);
          int64_t id;
          if (it == face_mid.end()) {
            const V3 p = quad_center(m.mf_of(m.face_mf, k), face_verts(3, d, s));
            id = (int64_t)m.X.size();
            m.X.push_back(p);
            face_mid[k] = id;
          } else {
            id = it->second;
          }
          fmid.push_back(m.X[(size_t)id]);
          int q[3] = {1, 1, 1};
          q[d] = 2 * s;
          L(q[0], q[1], q[2]) = id;
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
    // children (parent-major, lexicographic child position)
    for (int ch = 0; ch < nch; ++ch) {
      const int cx = ch & 1, cy = (ch >> 1) & 1, cz = (ch >> 2) & 1;
      std::array<int64_t, 8> nc{};
      for (int v = 0; v < nv; ++v) nc[v] = L(cx + (v & 1), cy + ((v >> 1) & 1), dim == 3 ? cz + ((v >> 2) & 1) : 0);
      cells.push_back(nc);
      cmf.push_back(cellmf);
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
          mfv = m.mf_of(m.face_mf, face_key(m, c, endd[0], ends[0] / 2));
        } else {
          mfv = cellmf;
        }
        if (mfv >= 0) lmf[mkey({nc[ln[0]], nc[ln[1]]})] = mfv;
      }
      for (int d = 0; d < dim; ++d)
        for (int s = 0; s < 2; ++s) {
          const int pc = (d == 0 ? cx : d == 1 ? cy : cz) + s;  // parent-lattice coordinate of the face
          const auto fv = face_verts(dim, d, s);
          const EKey k = dim == 2 ? mkey({nc[fv[0]], nc[fv[1]]}) : mkey({nc[fv[0]], nc[fv[1]], nc[fv[2]], nc[fv[3]]});
          if (pc == 0 || pc == 2) {
            const EKey pk = face_key(m, c, d, pc / 2);
            auto b = m.bface.find(pk);
            if (b != m.bface.end()) bface[k] = b->second;
            if (dim == 3) {
              const int f = m.mf_of(m.face_mf, pk);
              if (f >= 0) fmf[k] = f;
            }
          } else if (dim == 3 && cellmf >= 0) {
            fmf[k] = cellmf;
          }
        }
    }
  }
  m.cells.swap(cells);
  m.cell_mf.swap(cmf);
  m.bface.swap(bface);
  m.line_mf.swap(lmf);
  m.face_mf.swap(fmf);
  return GLS_OK;
}

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
  std::vector<int32_t> cell_vnodes, cell_pnodes, cell_mapping;
  std::vector<double> vnode_x, pnode_x, cell_support, cell_measure;
  std::vector<uint32_t> vnode_bid, pnode_bid;
};

double lag1(int k, int a, double x) {  // Lagrange basis a of degree k on equidistant nodes (k <= 2)
  double v = 1.0;
  for (int b = 0; b <= k; ++b)
    if (b != a) v *= (x - (double)b / k) / ((double)(a - b) / k);
  return v;
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
  auto number = [&](int kk, std::vector<int32_t> &cn, std::vector<double> &nx, std::vector<uint32_t> &nb) -> int {
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
    // periodic identification: nodes on faces of id b map onto the translated nodes of id a
    std::vector<int64_t> rep(pos.size());
    for (size_t i = 0; i < rep.size(); ++i) rep[i] = (int64_t)i;
    for (int p = 0; p < nper; ++p) {
      const int ida = per[3 * p], idb = per[3 * p + 1], dir = per[3 * p + 2];
      std::vector<int64_t> A, B;
      for (size_t i = 0; i < pos.size(); ++i) {
        if ((bits[i] >> ida) & 1) A.push_back((int64_t)i);
        if ((bits[i] >> idb) & 1) B.push_back((int64_t)i);
      }
      double scale = 0;
      for (auto &x : pos) scale = std::max(scale, std::fabs(x[0]) + std::fabs(x[1]) + std::fabs(x[2]));
      const double tol = 1e-8 * std::max(scale, 1e-300);
      std::map<std::array<long long, 2>, std::vector<int64_t>> grid;
      const int o1 = (dir + 1) % 3, o2 = (dir + 2) % 3;
      auto cellk = [&](const V3 &x) { return std::array<long long, 2>{std::llround(x[o1] / (100 * tol)), std::llround(x[o2] / (100 * tol))}; };
      for (auto i : A) grid[cellk(pos[(size_t)i])].push_back(i);
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
        if (match < 0) return gls_io_set_error(GLS_EINVAL, "periodic boundaries %d / %d: node without a partner", ida, idb);
        rep[(size_t)j] = match;
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
    if (n > INT32_MAX) return gls_io_set_error(GLS_EINVAL, "too many nodes for int32 ids");
    return GLS_OK;
  };
  int rc = number(k, F.cell_vnodes, F.vnode_x, F.vnode_bid);
  if (rc) return rc;
  if (kp == k) {
    F.cell_pnodes = F.cell_vnodes;
    F.pnode_x = F.vnode_x;
    F.pnode_bid = F.vnode_bid;
  } else {
    rc = number(kp, F.cell_pnodes, F.pnode_x, F.pnode_bid);
    if (rc) return rc;
  }
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
  P.impl_ = &F;
  return GLS_OK;
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

// SolutionTransfer::interpolate for one global refinement (navier_stokes_base.cc:737-780): fine
// cell f is child (f & (2^dim - 1)) of coarse cell f >> dim; each fine node takes the coarse cell's
// Qk / Qkp interpolant at its reference position in the parent (Qk on the children contains the
// parent's Qk space, so this is exact)
int gls_fe_space_transfer(const gls_fe_space *co, const gls_fe_space *fi, const double *cvec, double *fvec) {
  if (!co || !fi || !cvec || !fvec || co->dim != fi->dim || co->k != fi->k || co->kp != fi->kp ||
      fi->n_cells != co->n_cells << co->dim)
    return gls_io_set_error(GLS_EINVAL, "gls_fe_space_transfer: the fine space must be one global refinement of the coarse");
  const int dim = co->dim;
  const int64_t voc = (int64_t)dim * co->n_vnodes, vof = (int64_t)dim * fi->n_vnodes;
  for (int pass = 0; pass < 2; ++pass) {
    const int kk = pass == 0 ? co->k : co->kp, kk1 = kk + 1, nn = dim == 2 ? kk1 * kk1 : kk1 * kk1 * kk1;
    const int32_t *cc = pass == 0 ? co->cell_vnodes : co->cell_pnodes, *fc = pass == 0 ? fi->cell_vnodes : fi->cell_pnodes;
    const int ncomp = pass == 0 ? dim : 1;
    for (int64_t f = 0; f < fi->n_cells; ++f) {
      const int64_t c = f >> dim;
      const int ch = (int)(f & ((1 << dim) - 1));
      for (int a = 0; a < nn; ++a) {
        const int ia[3] = {a % kk1, (a / kk1) % kk1, dim == 3 ? a / (kk1 * kk1) : 0};
        double xp[3];
        for (int d = 0; d < dim; ++d) xp[d] = 0.5 * ((double)ia[d] / kk + ((ch >> d) & 1));
        double val[3] = {0, 0, 0};
        for (int b = 0; b < nn; ++b) {
          const int ib[3] = {b % kk1, (b / kk1) % kk1, dim == 3 ? b / (kk1 * kk1) : 0};
          double w = 1.0;
          for (int d = 0; d < dim; ++d) w *= lag1(kk, ib[d], xp[d]);
          if (w == 0.0) continue;
          const int64_t node = cc[c * nn + b];
          for (int e = 0; e < ncomp; ++e) val[e] += w * cvec[pass == 0 ? node * dim + e : voc + node];
        }
        const int64_t fn = fc[f * nn + a];
        for (int e = 0; e < ncomp; ++e) fvec[pass == 0 ? fn * dim + e : vof + fn] = val[e];
      }
    }
  }
  return GLS_OK;
}

}  // extern "C"
