// gls_dist.cpp — domain decomposition for the multi-GPU GLS path.
//
// Partition (restates parallel::distributed::Triangulation's p4est ownership,
// source/solvers/navier_stokes_base.cc:55-60, gls_navier_stokes.cc:186-202):
//   * cells are in Morton (z-)order; rank r owns a contiguous range of whole 2x2x2 bricks
//     (equal counts, like p4est's equal-count partition of a uniform forest);
//   * a node is owned by the lowest rank among the cells that touch it (deal.II convention);
//   * the rank-local mesh numbers its nodes owned-first (ascending global id), then ghosts
//     (ascending (owner, global id)); the single-GPU kernels run unchanged on it.
// Exchange lists: import = owner -> ghosting ranks (ghost values before an operator apply);
// export-add = ghosting rank -> owner (ghost contributions after an apply, the analogue of
// Trilinos compress(add), gls_navier_stokes.cc:774-776). Both sides build the lists from the
// same global mesh, ordered by global id, so no handshake is needed.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <map>
#include <memory>
#include <unordered_map>
#include <vector>

#include "../../include/gls_native.h"

int gls_internal_set_err(int code, const char *msg);

struct gls_part {
  int64_t cell_begin = 0, cell_end = 0, n_owned = 0, n_local = 0;
  int nvpc = 0;
  std::vector<int32_t> local_cells;     // [n_owned_cells * nvpc] local node ids
  std::vector<int64_t> local_to_global; // [n_local]
  std::vector<int> nbrs;
  std::vector<int64_t> send_off, recv_off;
  std::vector<int32_t> send_nodes, recv_nodes;  // local node ids
};

extern "C" {

int gls_part_create(int n_cells, int nvpc, const int32_t *cell_vnodes, int n_vnodes, int rank, int world,
                    gls_part **out) {
  if (!out || !cell_vnodes || n_cells < 0 || nvpc <= 0 || n_vnodes <= 0 || world <= 0 || rank < 0 || rank >= world)
    return gls_internal_set_err(GLS_EINVAL, "gls_part_create: bad arguments");
  std::unique_ptr<gls_part> p(new gls_part);
  p->nvpc = nvpc;
  // contiguous ranges of whole bricks (or cells when not brick-structured)
  const bool bricks = n_cells % 8 == 0;
  const int64_t units = bricks ? n_cells / 8 : n_cells, usz = bricks ? 8 : 1;
  std::vector<int64_t> cb(world + 1);
  for (int r = 0; r <= world; ++r) cb[r] = usz * (units * r / world);
  p->cell_begin = cb[rank];
  p->cell_end = cb[rank + 1];
  auto rank_of_cell = [&](int64_t c) {
    int r = (int)std::min<int64_t>(world - 1, (c * world) / std::max<int64_t>(n_cells, 1));
    while (r > 0 && c < cb[r]) --r;
    while (r < world - 1 && c >= cb[r + 1]) ++r;
    return r;
  };
  // node owner = lowest rank touching it
  std::vector<int32_t> owner((size_t)n_vnodes, INT32_MAX);
  for (int64_t c = 0; c < n_cells; ++c) {
    const int r = rank_of_cell(c);
    for (int a = 0; a < nvpc; ++a) {
      const int32_t nd = cell_vnodes[c * nvpc + a];
      if (nd < 0 || nd >= n_vnodes) return gls_internal_set_err(GLS_EINVAL, "gls_part_create: node out of range");
      if (r < owner[nd]) owner[nd] = r;
    }
  }
  // local node set
  std::vector<int32_t> g2l((size_t)n_vnodes, -1);
  std::vector<int64_t> owned, ghosts;
  for (int64_t c = p->cell_begin; c < p->cell_end; ++c)
    for (int a = 0; a < nvpc; ++a) {
      const int32_t nd = cell_vnodes[c * nvpc + a];
      if (g2l[nd] == -1) {
        g2l[nd] = 0;
        (owner[nd] == rank ? owned : ghosts).push_back(nd);
      }
    }
  std::sort(owned.begin(), owned.end());
  std::sort(ghosts.begin(), ghosts.end(), [&](int64_t a, int64_t b) {
    return owner[a] != owner[b] ? owner[a] < owner[b] : a < b;
  });
  p->n_owned = (int64_t)owned.size();
  p->n_local = p->n_owned + (int64_t)ghosts.size();
  p->local_to_global.reserve(p->n_local);
  for (int64_t g : owned) p->local_to_global.push_back(g);
  for (int64_t g : ghosts) p->local_to_global.push_back(g);
  for (int64_t i = 0; i < p->n_local; ++i) g2l[p->local_to_global[i]] = (int32_t)i;
  p->local_cells.resize((size_t)(p->cell_end - p->cell_begin) * nvpc);
  for (int64_t c = p->cell_begin; c < p->cell_end; ++c)
    for (int a = 0; a < nvpc; ++a) p->local_cells[(c - p->cell_begin) * nvpc + a] = g2l[cell_vnodes[c * nvpc + a]];
  // exchange lists per neighbour rank
  std::map<int, std::vector<int32_t>> send, recv;
  for (int64_t i = p->n_owned; i < p->n_local; ++i) recv[owner[p->local_to_global[i]]].push_back((int32_t)i);
  std::vector<int32_t> mark((size_t)n_vnodes, -1);
  for (int s = 0; s < world; ++s) {
    if (s == rank) continue;
    std::vector<int64_t> lst;
    for (int64_t c = cb[s]; c < cb[s + 1]; ++c)
      for (int a = 0; a < nvpc; ++a) {
        const int32_t nd = cell_vnodes[c * nvpc + a];
        if (owner[nd] == rank && mark[nd] != s) {
          mark[nd] = s;
          lst.push_back(nd);
        }
      }
    if (lst.empty()) continue;
    std::sort(lst.begin(), lst.end());
    auto &v = send[s];
    for (int64_t g : lst) v.push_back(g2l[g]);
  }
  std::vector<int> nb;
  for (auto &kv : send) nb.push_back(kv.first);
  for (auto &kv : recv) nb.push_back(kv.first);
  std::sort(nb.begin(), nb.end());
  nb.erase(std::unique(nb.begin(), nb.end()), nb.end());
  p->nbrs = nb;
  p->send_off.assign(1, 0);
  p->recv_off.assign(1, 0);
  for (int r : nb) {
    auto its = send.find(r);
    if (its != send.end()) p->send_nodes.insert(p->send_nodes.end(), its->second.begin(), its->second.end());
    p->send_off.push_back((int64_t)p->send_nodes.size());
    auto itr = recv.find(r);
    if (itr != recv.end()) p->recv_nodes.insert(p->recv_nodes.end(), itr->second.begin(), itr->second.end());
    p->recv_off.push_back((int64_t)p->recv_nodes.size());
  }
  *out = p.release();
  return GLS_OK;
}

int gls_part_sizes(const gls_part *p, int64_t *cell_begin, int64_t *cell_end, int64_t *n_owned, int64_t *n_local,
                   int *n_nbrs, int64_t *n_send, int64_t *n_recv) {
  if (!p) return gls_internal_set_err(GLS_EINVAL, "null partition");
  if (cell_begin) *cell_begin = p->cell_begin;
  if (cell_end) *cell_end = p->cell_end;
  if (n_owned) *n_owned = p->n_owned;
  if (n_local) *n_local = p->n_local;
  if (n_nbrs) *n_nbrs = (int)p->nbrs.size();
  if (n_send) *n_send = (int64_t)p->send_nodes.size();
  if (n_recv) *n_recv = (int64_t)p->recv_nodes.size();
  return GLS_OK;
}

int gls_part_get(const gls_part *p, int32_t *local_cell_vnodes, int64_t *local_to_global, int *nbr_ranks,
                 int64_t *send_offsets, int32_t *send_nodes, int64_t *recv_offsets, int32_t *recv_nodes) {
  if (!p) return gls_internal_set_err(GLS_EINVAL, "null partition");
  if (local_cell_vnodes) std::memcpy(local_cell_vnodes, p->local_cells.data(), p->local_cells.size() * sizeof(int32_t));
  if (local_to_global) std::memcpy(local_to_global, p->local_to_global.data(), p->local_to_global.size() * sizeof(int64_t));
  if (nbr_ranks) std::memcpy(nbr_ranks, p->nbrs.data(), p->nbrs.size() * sizeof(int));
  if (send_offsets) std::memcpy(send_offsets, p->send_off.data(), p->send_off.size() * sizeof(int64_t));
  if (send_nodes) std::memcpy(send_nodes, p->send_nodes.data(), p->send_nodes.size() * sizeof(int32_t));
  if (recv_offsets) std::memcpy(recv_offsets, p->recv_off.data(), p->recv_off.size() * sizeof(int64_t));
  if (recv_nodes) std::memcpy(recv_nodes, p->recv_nodes.data(), p->recv_nodes.size() * sizeof(int32_t));
  return GLS_OK;
}

int gls_part_destroy(gls_part *p) {
  delete p;
  return GLS_OK;
}

}  // extern "C"

// ---------------------------------------------------------------------------------------------
// General meshes (row e2 of SURVEY §8: adaptive / unstructured forests across ranks, the p::d
// triangulation partition of navier_stokes_base.cc:55-60 re-done after every adaptation,
// :682-733): any dim, Qk-Qk' with separate pressure nodes, hanging-node (and slip) lines.
//  * cells: contiguous, equal-count ranges of the given cell order (the space-filling leaf order of
//    the adapted forest), one per rank;
//  * a node is owned by the lowest rank whose cells touch it; rank-local nodes are owned first
//    (ascending global id), then ghosts (ascending (owner, global id)) -- velocity and pressure
//    nodes separately;
//  * ghosts also include the masters of every line whose DoF sits on a local cell and that no
//    local cell touches (the coarse side of a hanging face across the partition), so C v and the
//    condensation C^T y of the local cells need only local values;
//  * exchange lists are DoF-level (one double per DoF): both sides derive them from the same
//    replicated global mesh, ordered by global DoF id (velocity node*dim+c, pressure dim*NV+p).
// ---------------------------------------------------------------------------------------------
struct gls_gpart {
  int dim = 0, nvl = 0, npl = 0;
  bool sep = false;
  int64_t cell_begin = 0, cell_end = 0;
  int64_t n_owned_v = 0, n_owned_p = 0;
  std::vector<int64_t> vl2g, pl2g;                  // local -> global node
  std::vector<int32_t> local_cv, local_cp;          // local cell node maps
  std::vector<int> nbrs;
  std::vector<int64_t> send_off, recv_off;
  std::vector<int32_t> send_dofs, recv_dofs;        // local DoF ids
  std::vector<int64_t> gdof2l_keys, gdof2l_vals;    // sorted global DoF -> local DoF (local DoFs only)
  int64_t n_local_dofs() const { return (int64_t)dim * (int64_t)vl2g.size() + (int64_t)(sep ? pl2g.size() : vl2g.size()); }
};

extern "C" {

int gls_gpart_create(int dim, int k, int kp, int64_t n_cells, const int32_t *cell_vnodes, const int32_t *cell_pnodes,
                     int64_t n_vnodes, int64_t n_pnodes, int64_t n_lines, const int64_t *line_dofs,
                     const int64_t *line_off, const int64_t *line_masters, int rank, int world, gls_gpart **out) {
  if (!out || (dim != 2 && dim != 3) || k < 1 || kp < 1 || n_cells < 0 || !cell_vnodes || n_vnodes <= 0 || world < 1 ||
      rank < 0 || rank >= world || n_lines < 0 || (n_lines > 0 && (!line_dofs || !line_off || !line_masters)))
    return gls_internal_set_err(GLS_EINVAL, "gls_gpart_create: bad arguments");
  std::unique_ptr<gls_gpart> p(new gls_gpart);
  p->dim = dim;
  p->nvl = 1;
  p->npl = 1;
  for (int d = 0; d < dim; ++d) {
    p->nvl *= k + 1;
    p->npl *= kp + 1;
  }
  p->sep = cell_pnodes != nullptr;
  if (!p->sep && (kp != k || n_pnodes != n_vnodes))
    return gls_internal_set_err(GLS_EINVAL, "gls_gpart_create: equal-order meshes share their nodes");
  const int nvl = p->nvl, npl = p->npl;
  const int64_t NV = n_vnodes, NP = p->sep ? n_pnodes : n_vnodes, NVD = (int64_t)dim * NV;
  std::vector<int64_t> cb((size_t)world + 1);
  for (int r = 0; r <= world; ++r) cb[(size_t)r] = n_cells * r / world;
  p->cell_begin = cb[(size_t)rank];
  p->cell_end = cb[(size_t)rank + 1];
  auto rank_of_cell = [&](int64_t c) {
    int r = (int)std::min<int64_t>(world - 1, c * world / std::max<int64_t>(n_cells, 1));
    while (r > 0 && c < cb[(size_t)r]) --r;
    while (r < world - 1 && c >= cb[(size_t)r + 1]) ++r;
    return r;
  };
  // owners: the lowest rank touching the node
  std::vector<int32_t> vown((size_t)NV, INT32_MAX), pown;
  for (int64_t c = 0; c < n_cells; ++c) {
    const int r = rank_of_cell(c);
    for (int a = 0; a < nvl; ++a) {
      const int32_t nd = cell_vnodes[c * nvl + a];
      if (nd < 0 || nd >= NV) return gls_internal_set_err(GLS_EINVAL, "gls_gpart_create: node out of range");
      vown[(size_t)nd] = std::min(vown[(size_t)nd], (int32_t)r);
    }
  }
  if (p->sep) {
    pown.assign((size_t)NP, INT32_MAX);
    for (int64_t c = 0; c < n_cells; ++c) {
      const int r = rank_of_cell(c);
      for (int a = 0; a < npl; ++a) {
        const int32_t nd = cell_pnodes[c * npl + a];
        if (nd < 0 || nd >= NP) return gls_internal_set_err(GLS_EINVAL, "gls_gpart_create: pressure node out of range");
        pown[(size_t)nd] = std::min(pown[(size_t)nd], (int32_t)r);
      }
    }
  }
  for (int64_t i = 0; i < NV; ++i)
    if (vown[(size_t)i] == INT32_MAX) return gls_internal_set_err(GLS_EINVAL, "gls_gpart_create: a velocity node lies in no cell");
  auto dof_owner = [&](int64_t g) -> int32_t {
    if (g < NVD) return vown[(size_t)(g / dim)];
    return p->sep ? pown[(size_t)(g - NVD)] : vown[(size_t)(g - NVD)];
  };
  // the lines of a global DoF
  std::vector<int64_t> lidx((size_t)(NVD + NP), -1);
  for (int64_t i = 0; i < n_lines; ++i) {
    if (line_dofs[i] < 0 || line_dofs[i] >= NVD + NP) return gls_internal_set_err(GLS_EINVAL, "gls_gpart_create: line DoF");
    lidx[(size_t)line_dofs[i]] = i;
  }
  // the global DoFs a rank needs: those of its cells and the masters of their lines
  auto needed = [&](int r, std::vector<int64_t> &dofs) {
    dofs.clear();
    for (int64_t c = cb[(size_t)r]; c < cb[(size_t)r + 1]; ++c) {
      for (int a = 0; a < nvl; ++a) {
        const int64_t nd = cell_vnodes[c * nvl + a];
        for (int cc = 0; cc < dim; ++cc) dofs.push_back(nd * dim + cc);
        if (!p->sep) dofs.push_back(NVD + nd);
      }
      if (p->sep)
        for (int a = 0; a < npl; ++a) dofs.push_back(NVD + cell_pnodes[c * npl + a]);
    }
    std::sort(dofs.begin(), dofs.end());
    dofs.erase(std::unique(dofs.begin(), dofs.end()), dofs.end());
    const size_t nc = dofs.size();
    for (size_t t = 0; t < nc; ++t) {
      const int64_t li = lidx[(size_t)dofs[t]];
      if (li < 0) continue;
      for (int64_t j = line_off[li]; j < line_off[li + 1]; ++j) dofs.push_back(line_masters[j]);
    }
    std::sort(dofs.begin(), dofs.end());
    dofs.erase(std::unique(dofs.begin(), dofs.end()), dofs.end());
  };
  std::vector<int64_t> mine;
  needed(rank, mine);
  // local nodes: the nodes of the needed DoFs (a node's DoFs come together), owned first
  std::vector<int64_t> vown_l, vgh_l, pown_l, pgh_l;
  {
    std::vector<char> vseen((size_t)NV, 0), pseen((size_t)NP, 0);
    for (int64_t g : mine) {
      if (g < NVD || !p->sep) {
        const int64_t nd = g < NVD ? g / dim : g - NVD;
        if (!vseen[(size_t)nd]) {
          vseen[(size_t)nd] = 1;
          (vown[(size_t)nd] == rank ? vown_l : vgh_l).push_back(nd);
        }
      } else {
        const int64_t nd = g - NVD;
        if (!pseen[(size_t)nd]) {
          pseen[(size_t)nd] = 1;
          (pown[(size_t)nd] == rank ? pown_l : pgh_l).push_back(nd);
        }
      }
    }
  }
  auto order_nodes = [&](std::vector<int64_t> &own, std::vector<int64_t> &gh, const std::vector<int32_t> &ow,
                         std::vector<int64_t> &l2g) {
    std::sort(own.begin(), own.end());
    std::sort(gh.begin(), gh.end(), [&](int64_t a, int64_t b) {
      return ow[(size_t)a] != ow[(size_t)b] ? ow[(size_t)a] < ow[(size_t)b] : a < b;
    });
    l2g = own;
    l2g.insert(l2g.end(), gh.begin(), gh.end());
  };
  order_nodes(vown_l, vgh_l, vown, p->vl2g);
  p->n_owned_v = (int64_t)vown_l.size();
  if (p->sep) {
    order_nodes(pown_l, pgh_l, pown, p->pl2g);
    p->n_owned_p = (int64_t)pown_l.size();
  } else {
    p->n_owned_p = p->n_owned_v;
  }
  const int64_t nvloc = (int64_t)p->vl2g.size();
  std::vector<int32_t> vg2l((size_t)NV, -1), pg2l;
  for (int64_t i = 0; i < nvloc; ++i) vg2l[(size_t)p->vl2g[(size_t)i]] = (int32_t)i;
  if (p->sep) {
    pg2l.assign((size_t)NP, -1);
    for (size_t i = 0; i < p->pl2g.size(); ++i) pg2l[(size_t)p->pl2g[i]] = (int32_t)i;
  }
  auto g2l_dof = [&](int64_t g) -> int64_t {
    if (g < NVD) {
      const int32_t l = vg2l[(size_t)(g / dim)];
      return l < 0 ? -1 : (int64_t)l * dim + g % dim;
    }
    const int32_t l = p->sep ? pg2l[(size_t)(g - NVD)] : vg2l[(size_t)(g - NVD)];
    return l < 0 ? -1 : (int64_t)dim * nvloc + l;
  };
  // local cells
  const int64_t ncl = p->cell_end - p->cell_begin;
  p->local_cv.resize((size_t)(ncl * nvl));
  for (int64_t c = 0; c < ncl; ++c)
    for (int a = 0; a < nvl; ++a) p->local_cv[(size_t)(c * nvl + a)] = vg2l[(size_t)cell_vnodes[(p->cell_begin + c) * nvl + a]];
  if (p->sep) {
    p->local_cp.resize((size_t)(ncl * npl));
    for (int64_t c = 0; c < ncl; ++c)
      for (int a = 0; a < npl; ++a) p->local_cp[(size_t)(c * npl + a)] = pg2l[(size_t)cell_pnodes[(p->cell_begin + c) * npl + a]];
  }
  // global -> local DoF map of the local DoFs (sorted pairs, for gls_gpart_map_dofs)
  {
    const int64_t nl = p->n_local_dofs();
    std::vector<std::pair<int64_t, int64_t>> kv;
    kv.reserve((size_t)nl);
    for (int64_t i = 0; i < nvloc; ++i)
      for (int cc = 0; cc < dim; ++cc) kv.push_back({p->vl2g[(size_t)i] * dim + cc, i * dim + cc});
    if (p->sep)
      for (size_t i = 0; i < p->pl2g.size(); ++i) kv.push_back({NVD + p->pl2g[i], (int64_t)dim * nvloc + (int64_t)i});
    else
      for (int64_t i = 0; i < nvloc; ++i) kv.push_back({NVD + p->vl2g[(size_t)i], (int64_t)dim * nvloc + i});
    std::sort(kv.begin(), kv.end());
    for (auto &e : kv) {
      p->gdof2l_keys.push_back(e.first);
      p->gdof2l_vals.push_back(e.second);
    }
  }
  // exchange lists: recv = my ghost DoFs by owner; send = my owned DoFs each other rank needs
  std::map<int, std::vector<int32_t>> send, recv;
  for (int64_t g : mine) {
    const int32_t o = dof_owner(g);
    if (o != rank) recv[o].push_back((int32_t)g2l_dof(g));
  }
  std::vector<int64_t> theirs;
  for (int s = 0; s < world; ++s) {
    if (s == rank) continue;
    needed(s, theirs);
    std::vector<int32_t> lst;
    for (int64_t g : theirs)
      if (dof_owner(g) == rank) lst.push_back((int32_t)g2l_dof(g));
    if (!lst.empty()) send[s] = lst;
  }
  std::vector<int> nb;
  for (auto &kv : send) nb.push_back(kv.first);
  for (auto &kv : recv) nb.push_back(kv.first);
  std::sort(nb.begin(), nb.end());
  nb.erase(std::unique(nb.begin(), nb.end()), nb.end());
  p->nbrs = nb;
  p->send_off.assign(1, 0);
  p->recv_off.assign(1, 0);
  for (int r : nb) {
    auto its = send.find(r);
    if (its != send.end()) p->send_dofs.insert(p->send_dofs.end(), its->second.begin(), its->second.end());
    p->send_off.push_back((int64_t)p->send_dofs.size());
    auto itr = recv.find(r);
    if (itr != recv.end()) p->recv_dofs.insert(p->recv_dofs.end(), itr->second.begin(), itr->second.end());
    p->recv_off.push_back((int64_t)p->recv_dofs.size());
  }
  *out = p.release();
  return GLS_OK;
}

// ---------------------------------------------------------------------------------------------
// The same plan from the rank's LOCAL PART of a distributed forest (no global mesh on the rank):
// the owned cells plus the ghost layer -- every cell coupled to an owned cell, where two cells are
// coupled when they share a node or one carries a hanging line whose master is a node of the other
// (p4est's ghost layer with corner connectivity, extended by the line closure; the p::d triangulation's
// locally relevant cells, navier_stokes_base.cc:55-60) -- each with its owner rank, and the lines whose
// DoF sits on a provided cell. Nodes are named by 64-bit keys unique across the forest (the global
// node id, or a lattice / vertex key; no global numbering is needed); a DoF is key * (dim + 1) + c,
// c = dim for pressure. Why the part is enough: a node an owned cell touches has all its cells coupled
// to that owned cell, so "lowest rank touching it" is exact for every DoF this rank holds, and any other
// rank's cell needing a DoF this rank owns is coupled to the owned cell touching that DoF, so both
// exchange lists come out of the part alone, in the same order on both sides ((velocity before
// pressure, key, component) order, which equals gls_gpart_create's global-id order when keys are global
// ids). Owned cells are the provided cells with owner == rank, in the given order. The result is a
// gls_gpart handle: gls_gpart_sizes / _get (vnode_l2g / pnode_l2g hold keys) / _map_dofs (DoF keys).
// ---------------------------------------------------------------------------------------------
int gls_dpart_create(int dim, int k, int kp, int64_t n_cells, const int32_t *cell_owner, const int64_t *cell_vkeys,
                     const int64_t *cell_pkeys, int64_t n_lines, const int64_t *line_dofs, const int64_t *line_off,
                     const int64_t *line_masters, int rank, int world, gls_gpart **out) {
  if (!out || (dim != 2 && dim != 3) || k < 1 || kp < 1 || n_cells < 0 || (n_cells > 0 && (!cell_owner || !cell_vkeys)) ||
      world < 1 || rank < 0 || rank >= world || n_lines < 0 || (n_lines > 0 && (!line_dofs || !line_off || !line_masters)))
    return gls_internal_set_err(GLS_EINVAL, "gls_dpart_create: bad arguments");
  std::unique_ptr<gls_gpart> p(new gls_gpart);
  p->dim = dim;
  p->nvl = 1;
  p->npl = 1;
  for (int d = 0; d < dim; ++d) {
    p->nvl *= k + 1;
    p->npl *= kp + 1;
  }
  p->sep = cell_pkeys != nullptr;
  if (!p->sep && kp != k) return gls_internal_set_err(GLS_EINVAL, "gls_dpart_create: equal-order meshes share their nodes");
  const int nvl = p->nvl, npl = p->npl, D1 = dim + 1;
  const int64_t kmax = INT64_MAX / D1 - 1;
  // owners of every node on a provided cell: the lowest rank touching it
  std::unordered_map<int64_t, int32_t> vown, pown;
  vown.reserve((size_t)(n_cells * 4 + 16));
  auto touch = [](std::unordered_map<int64_t, int32_t> &m, int64_t key, int32_t r) {
    auto it = m.find(key);
    if (it == m.end()) m.emplace(key, r);
    else if (r < it->second) it->second = r;
  };
  int64_t n_owned_cells = 0;
  for (int64_t c = 0; c < n_cells; ++c) {
    const int32_t r = cell_owner[c];
    if (r < 0 || r >= world) return gls_internal_set_err(GLS_EINVAL, "gls_dpart_create: cell owner out of range");
    n_owned_cells += r == rank;
    for (int a = 0; a < nvl; ++a) {
      const int64_t key = cell_vkeys[c * nvl + a];
      if (key < 0 || key > kmax) return gls_internal_set_err(GLS_EINVAL, "gls_dpart_create: node key out of range");
      touch(vown, key, r);
    }
    if (p->sep)
      for (int a = 0; a < npl; ++a) {
        const int64_t key = cell_pkeys[c * npl + a];
        if (key < 0 || key > kmax) return gls_internal_set_err(GLS_EINVAL, "gls_dpart_create: pressure key out of range");
        touch(pown, key, r);
      }
  }
  // DoF order: velocity before pressure, then key, then component (= DoF key order within each kind)
  auto is_p = [D1, dim](int64_t g) { return g % D1 == dim; };
  auto dof_less = [&](int64_t a, int64_t b) { return is_p(a) != is_p(b) ? !is_p(a) : a < b; };
  // owner of a DoF (-1: no provided cell touches its node -- not this rank's, whoever owns it). Exact because the
  // caller provides EVERY cell touching each node this rank needs, line masters included (the header's contract)
  auto dof_owner = [&](int64_t g) -> int32_t {
    const std::unordered_map<int64_t, int32_t> &m = (is_p(g) && p->sep) ? pown : vown;
    auto it = m.find(g / D1);
    return it == m.end() ? -1 : it->second;
  };
  std::unordered_map<int64_t, int64_t> lidx;
  for (int64_t i = 0; i < n_lines; ++i) {
    if (line_dofs[i] < 0) return gls_internal_set_err(GLS_EINVAL, "gls_dpart_create: line DoF key");
    lidx[line_dofs[i]] = i;
  }
  // the DoFs the cells of rank r (among the provided ones) need: their own and their lines' masters
  auto needed = [&](int r, std::vector<int64_t> &dofs) {
    dofs.clear();
    for (int64_t c = 0; c < n_cells; ++c) {
      if (cell_owner[c] != r) continue;
      for (int a = 0; a < nvl; ++a) {
        const int64_t key = cell_vkeys[c * nvl + a];
        for (int cc = 0; cc < dim; ++cc) dofs.push_back(key * D1 + cc);
        if (!p->sep) dofs.push_back(key * D1 + dim);
      }
      if (p->sep)
        for (int a = 0; a < npl; ++a) dofs.push_back(cell_pkeys[c * npl + a] * D1 + dim);
    }
    std::sort(dofs.begin(), dofs.end());
    dofs.erase(std::unique(dofs.begin(), dofs.end()), dofs.end());
    const size_t nc = dofs.size();
    for (size_t t = 0; t < nc; ++t) {
      auto it = lidx.find(dofs[t]);
      if (it == lidx.end()) continue;
      for (int64_t j = line_off[it->second]; j < line_off[it->second + 1]; ++j) dofs.push_back(line_masters[j]);
    }
    std::sort(dofs.begin(), dofs.end(), dof_less);
    dofs.erase(std::unique(dofs.begin(), dofs.end()), dofs.end());
  };
  std::vector<int64_t> mine;
  needed(rank, mine);
  for (int64_t g : mine)
    if (dof_owner(g) < 0)
      return gls_internal_set_err(GLS_EINVAL, "gls_dpart_create: a line master lies on no provided cell (the ghost "
                                              "layer must include the cells coupled through hanging lines)");
  // local nodes (a node's DoFs come together): owned first by key, then ghosts by (owner, key)
  std::vector<int64_t> vown_l, vgh_l, pown_l, pgh_l;
  {
    std::unordered_map<int64_t, char> vseen, pseen;
    for (int64_t g : mine) {
      const int64_t key = g / D1;
      const bool pres = is_p(g) && p->sep;
      auto &seen = pres ? pseen : vseen;
      if (seen.emplace(key, 1).second) {
        const bool own = dof_owner(g) == rank;
        (pres ? (own ? pown_l : pgh_l) : (own ? vown_l : vgh_l)).push_back(key);
      }
    }
  }
  auto order_nodes = [&](std::vector<int64_t> &own, std::vector<int64_t> &gh, const std::unordered_map<int64_t, int32_t> &ow,
                         std::vector<int64_t> &l2k) {
    std::sort(own.begin(), own.end());
    std::sort(gh.begin(), gh.end(), [&](int64_t a, int64_t b) {
      const int32_t oa = ow.at(a), ob = ow.at(b);
      return oa != ob ? oa < ob : a < b;
    });
    l2k = own;
    l2k.insert(l2k.end(), gh.begin(), gh.end());
  };
  order_nodes(vown_l, vgh_l, vown, p->vl2g);
  p->n_owned_v = (int64_t)vown_l.size();
  if (p->sep) {
    order_nodes(pown_l, pgh_l, pown, p->pl2g);
    p->n_owned_p = (int64_t)pown_l.size();
  } else {
    p->n_owned_p = p->n_owned_v;
  }
  const int64_t nvloc = (int64_t)p->vl2g.size();
  if (nvloc > INT32_MAX || n_owned_cells * nvl > INT32_MAX)
    return gls_internal_set_err(GLS_EINVAL, "gls_dpart_create: the local part exceeds 32-bit node ids");
  std::unordered_map<int64_t, int32_t> vk2l, pk2l;
  for (int64_t i = 0; i < nvloc; ++i) vk2l[p->vl2g[(size_t)i]] = (int32_t)i;
  for (size_t i = 0; i < p->pl2g.size(); ++i) pk2l[p->pl2g[i]] = (int32_t)i;
  auto k2l_dof = [&](int64_t g) -> int64_t {
    const int64_t key = g / D1;
    const int c = (int)(g % D1);
    if (c < dim) return (int64_t)vk2l.at(key) * dim + c;
    return (int64_t)dim * nvloc + (p->sep ? pk2l.at(key) : vk2l.at(key));
  };
  // owned cells, in the given order
  p->cell_begin = 0;
  p->cell_end = n_owned_cells;
  p->local_cv.reserve((size_t)(n_owned_cells * nvl));
  if (p->sep) p->local_cp.reserve((size_t)(n_owned_cells * npl));
  for (int64_t c = 0; c < n_cells; ++c) {
    if (cell_owner[c] != rank) continue;
    for (int a = 0; a < nvl; ++a) p->local_cv.push_back(vk2l.at(cell_vkeys[c * nvl + a]));
    if (p->sep)
      for (int a = 0; a < npl; ++a) p->local_cp.push_back(pk2l.at(cell_pkeys[c * npl + a]));
  }
  // DoF key -> local DoF (for gls_gpart_map_dofs)
  {
    std::vector<std::pair<int64_t, int64_t>> kv;
    kv.reserve(mine.size());
    for (int64_t g : mine) kv.push_back({g, k2l_dof(g)});
    std::sort(kv.begin(), kv.end());
    for (auto &e : kv) {
      p->gdof2l_keys.push_back(e.first);
      p->gdof2l_vals.push_back(e.second);
    }
  }
  // exchange lists: recv = my ghost DoFs by owner; send = my owned DoFs the provided cells of each other rank need
  std::map<int, std::vector<int32_t>> send, recv;
  for (int64_t g : mine) {
    const int32_t o = dof_owner(g);
    if (o != rank) recv[o].push_back((int32_t)k2l_dof(g));
  }
  std::vector<int> others;
  for (int64_t c = 0; c < n_cells; ++c)
    if (cell_owner[c] != rank) others.push_back(cell_owner[c]);
  std::sort(others.begin(), others.end());
  others.erase(std::unique(others.begin(), others.end()), others.end());
  std::vector<int64_t> theirs;
  for (int s : others) {
    needed(s, theirs);
    std::vector<int32_t> lst;
    for (int64_t g : theirs)
      if (dof_owner(g) == rank) lst.push_back((int32_t)k2l_dof(g));
    if (!lst.empty()) send[s] = lst;
  }
  std::vector<int> nb;
  for (auto &e : send) nb.push_back(e.first);
  for (auto &e : recv) nb.push_back(e.first);
  std::sort(nb.begin(), nb.end());
  nb.erase(std::unique(nb.begin(), nb.end()), nb.end());
  p->nbrs = nb;
  p->send_off.assign(1, 0);
  p->recv_off.assign(1, 0);
  for (int r : nb) {
    auto its = send.find(r);
    if (its != send.end()) p->send_dofs.insert(p->send_dofs.end(), its->second.begin(), its->second.end());
    p->send_off.push_back((int64_t)p->send_dofs.size());
    auto itr = recv.find(r);
    if (itr != recv.end()) p->recv_dofs.insert(p->recv_dofs.end(), itr->second.begin(), itr->second.end());
    p->recv_off.push_back((int64_t)p->recv_dofs.size());
  }
  *out = p.release();
  return GLS_OK;
}

int gls_gpart_sizes(const gls_gpart *p, int64_t *cell_begin, int64_t *cell_end, int64_t *n_vnodes, int64_t *n_pnodes,
                    int64_t *n_owned_vnodes, int64_t *n_owned_pnodes, int *n_nbrs, int64_t *n_send, int64_t *n_recv) {
  if (!p) return gls_internal_set_err(GLS_EINVAL, "null partition");
  if (cell_begin) *cell_begin = p->cell_begin;
  if (cell_end) *cell_end = p->cell_end;
  if (n_vnodes) *n_vnodes = (int64_t)p->vl2g.size();
  if (n_pnodes) *n_pnodes = p->sep ? (int64_t)p->pl2g.size() : (int64_t)p->vl2g.size();
  if (n_owned_vnodes) *n_owned_vnodes = p->n_owned_v;
  if (n_owned_pnodes) *n_owned_pnodes = p->n_owned_p;
  if (n_nbrs) *n_nbrs = (int)p->nbrs.size();
  if (n_send) *n_send = (int64_t)p->send_dofs.size();
  if (n_recv) *n_recv = (int64_t)p->recv_dofs.size();
  return GLS_OK;
}

int gls_gpart_get(const gls_gpart *p, int32_t *local_cell_vnodes, int32_t *local_cell_pnodes, int64_t *vnode_l2g,
                  int64_t *pnode_l2g, int *nbr_ranks, int64_t *send_offsets, int32_t *send_dofs, int64_t *recv_offsets,
                  int32_t *recv_dofs) {
  if (!p) return gls_internal_set_err(GLS_EINVAL, "null partition");
  if (local_cell_vnodes) std::memcpy(local_cell_vnodes, p->local_cv.data(), p->local_cv.size() * sizeof(int32_t));
  if (local_cell_pnodes && p->sep) std::memcpy(local_cell_pnodes, p->local_cp.data(), p->local_cp.size() * sizeof(int32_t));
  if (vnode_l2g) std::memcpy(vnode_l2g, p->vl2g.data(), p->vl2g.size() * sizeof(int64_t));
  if (pnode_l2g) {
    const std::vector<int64_t> &src = p->sep ? p->pl2g : p->vl2g;
    std::memcpy(pnode_l2g, src.data(), src.size() * sizeof(int64_t));
  }
  if (nbr_ranks) std::memcpy(nbr_ranks, p->nbrs.data(), p->nbrs.size() * sizeof(int));
  if (send_offsets) std::memcpy(send_offsets, p->send_off.data(), p->send_off.size() * sizeof(int64_t));
  if (send_dofs) std::memcpy(send_dofs, p->send_dofs.data(), p->send_dofs.size() * sizeof(int32_t));
  if (recv_offsets) std::memcpy(recv_offsets, p->recv_off.data(), p->recv_off.size() * sizeof(int64_t));
  if (recv_dofs) std::memcpy(recv_dofs, p->recv_dofs.data(), p->recv_dofs.size() * sizeof(int32_t));
  return GLS_OK;
}

// global DoF ids -> local DoF ids (-1: not local to this rank)
int gls_gpart_map_dofs(const gls_gpart *p, int64_t n, const int64_t *global_dofs, int64_t *local_dofs) {
  if (!p || n < 0 || (n > 0 && (!global_dofs || !local_dofs))) return gls_internal_set_err(GLS_EINVAL, "gls_gpart_map_dofs");
  for (int64_t i = 0; i < n; ++i) {
    auto it = std::lower_bound(p->gdof2l_keys.begin(), p->gdof2l_keys.end(), global_dofs[i]);
    local_dofs[i] = (it != p->gdof2l_keys.end() && *it == global_dofs[i]) ? p->gdof2l_vals[(size_t)(it - p->gdof2l_keys.begin())] : -1;
  }
  return GLS_OK;
}

int gls_gpart_destroy(gls_gpart *p) {
  delete p;
  return GLS_OK;
}

}  // extern "C"
