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
