// Host-side sparse-pattern algorithms behind the assembled ILU(k) preconditioner (gls_ilu_attach):
//  * iluk_pattern: the level-of-fill pattern of Ifpack's ILU(k) (Ifpack_IlukGraph, used through
//    deal.II's TrilinosWrappers::PreconditionILU by the reference's setup_ILU,
//    source/solvers/gls_navier_stokes.cc:1161-1176, 'ilu preconditioner fill',
//    source/core/parameters.cc:546). Original entries have level 0; eliminating row k from row i
//    creates (i, j) at level lev(i,k) + lev(k,j) + 1, kept when <= fill. ILU(0) on this pattern
//    (explicit zeros at the fill positions) is ILU(k) of the matrix, which is how the device factors it
//    (rocsparse csrilu0 on the enlarged pattern).
//  * cuthill_mckee_nodes: deal.II's DoFRenumbering::Cuthill_McKee (gls_navier_stokes.cc:70;
//    SparsityTools::reorder_Cuthill_McKee: start at the first DoF of least row length, then level by
//    level, each level's DoFs ordered by their number of not yet numbered neighbours, ties in the old
//    order), evaluated on the node graph (all DoFs of a node share one row of the cell-coupling
//    pattern).
#include <algorithm>
#include <climits>
#include <cstdint>
#include <cstring>
#include <vector>

#include "../../include/gls_native.h"
#include "gls_sparse.hpp"

namespace gls {

template <typename RP>
int iluk_pattern(int64_t n, const RP *rowp, const int32_t *col, int fill, std::vector<RP> &orow,
                 std::vector<int32_t> &ocol, std::vector<int32_t> *olev) {
  if (n < 0 || fill < 0 || !rowp || (n > 0 && !col)) return GLS_EINVAL;
  orow.assign((size_t)n + 1, 0);
  ocol.clear();
  if (olev) olev->clear();
  if (fill == 0) {  // ILU(0): the graph itself (rows sorted, the diagonal added); no U lists kept
    ocol.reserve((size_t)rowp[n] + (size_t)n);
    std::vector<int32_t> row;
    for (int64_t i = 0; i < n; ++i) {
      row.assign(col + rowp[i], col + rowp[i + 1]);
      row.push_back((int32_t)i);
      std::sort(row.begin(), row.end());
      row.erase(std::unique(row.begin(), row.end()), row.end());
      if (row.front() < 0 || row.back() >= n) return GLS_EINVAL;
      ocol.insert(ocol.end(), row.begin(), row.end());
      if (olev) olev->insert(olev->end(), row.size(), 0);
      if (sizeof(RP) < 8 && ocol.size() > (size_t)INT32_MAX) return GLS_ENOMEM;
      orow[(size_t)i + 1] = (RP)ocol.size();
    }
    return GLS_OK;
  }
  // U part (col > row) of every finished row with its levels: (ucol, ulev)[uoff[k] .. uoff[k+1])
  std::vector<int64_t> uoff((size_t)n + 1, 0);
  std::vector<int32_t> ucol, ulev;
  std::vector<int32_t> lev((size_t)n, 0), nxt((size_t)n + 1, 0);
  std::vector<int64_t> stamp((size_t)n, -1);
  std::vector<int32_t> row;
  const int32_t END = (int32_t)n;  // list terminator (larger than every column)
  for (int64_t i = 0; i < n; ++i) {
    row.assign(col + rowp[i], col + rowp[i + 1]);
    row.push_back((int32_t)i);  // the diagonal is always part of the graph
    std::sort(row.begin(), row.end());
    row.erase(std::unique(row.begin(), row.end()), row.end());
    if (row.front() < 0 || row.back() >= n) return GLS_EINVAL;
    // sorted linked list of the row's columns
    int32_t head = row[0];
    for (size_t t = 0; t < row.size(); ++t) {
      const int32_t c = row[t];
      nxt[(size_t)c] = t + 1 < row.size() ? row[t + 1] : END;
      lev[(size_t)c] = 0;
      stamp[(size_t)c] = i;
    }
    // eliminate with every prior row k of the (growing) L part, in increasing order
    for (int32_t k = head; k < i; k = nxt[(size_t)k]) {
      const int32_t lik = lev[(size_t)k];
      if (lik >= fill) continue;  // lik + lkj + 1 > fill for every j
      int32_t prev = k;
      for (int64_t t = uoff[(size_t)k]; t < uoff[(size_t)k + 1]; ++t) {
        const int32_t j = ucol[(size_t)t];
        const int32_t l = lik + ulev[(size_t)t] + 1;
        if (l > fill) continue;
        if (stamp[(size_t)j] == i) {
          if (l < lev[(size_t)j]) lev[(size_t)j] = l;
        } else {  // insert j (> prev) into the sorted list
          while (nxt[(size_t)prev] < j) prev = nxt[(size_t)prev];
          nxt[(size_t)j] = nxt[(size_t)prev];
          nxt[(size_t)prev] = j;
          lev[(size_t)j] = l;
          stamp[(size_t)j] = i;
        }
        prev = j;
      }
    }
    for (int32_t c = head; c != END; c = nxt[(size_t)c]) {
      ocol.push_back(c);
      if (olev) olev->push_back(lev[(size_t)c]);
      if (c > i) {
        ucol.push_back(c);
        ulev.push_back(lev[(size_t)c]);
      }
    }
    if (sizeof(RP) < 8 && ocol.size() > (size_t)INT32_MAX) return GLS_ENOMEM;
    orow[(size_t)i + 1] = (RP)ocol.size();
    uoff[(size_t)i + 1] = (int64_t)ucol.size();
  }
  return GLS_OK;
}
template int iluk_pattern<int32_t>(int64_t, const int32_t *, const int32_t *, int, std::vector<int32_t> &,
                                   std::vector<int32_t> &, std::vector<int32_t> *);
template int iluk_pattern<int64_t>(int64_t, const int64_t *, const int32_t *, int, std::vector<int64_t> &,
                                   std::vector<int32_t> &, std::vector<int32_t> *);

void cuthill_mckee_nodes(int64_t nnodes, const std::vector<int64_t> &adj_off, const std::vector<int64_t> &adj,
                         const std::vector<int64_t> &dof_off, const std::vector<int64_t> &dofs,
                         std::vector<int64_t> &order) {
  // old position of a DoF = its index in `dofs` (node-major); a node's DoFs are consecutive there
  const int64_t n = dof_off[(size_t)nnodes];
  order.clear();
  order.reserve((size_t)n);
  std::vector<int64_t> row_len((size_t)nnodes, 0), unnum((size_t)nnodes, 0);
  for (int64_t x = 0; x < nnodes; ++x) {
    unnum[(size_t)x] = dof_off[(size_t)x + 1] - dof_off[(size_t)x];
    for (int64_t t = adj_off[(size_t)x]; t < adj_off[(size_t)x + 1]; ++t)
      row_len[(size_t)x] += dof_off[(size_t)adj[(size_t)t] + 1] - dof_off[(size_t)adj[(size_t)t]];
  }
  std::vector<char> numbered((size_t)n, 0);
  std::vector<int64_t> node_of((size_t)n);
  for (int64_t x = 0; x < nnodes; ++x)
    for (int64_t t = dof_off[(size_t)x]; t < dof_off[(size_t)x + 1]; ++t) node_of[(size_t)t] = x;
  auto number = [&](int64_t pos) {
    numbered[(size_t)pos] = 1;
    --unnum[(size_t)node_of[(size_t)pos]];
    order.push_back(dofs[(size_t)pos]);
  };
  // find_unnumbered_starting_index: the first not yet numbered DoF of least row length
  int64_t scan = 0;
  auto start = [&]() -> int64_t {
    int64_t best = -1, bl = INT64_MAX;
    for (int64_t p = scan; p < n; ++p)
      if (!numbered[(size_t)p] && row_len[(size_t)node_of[(size_t)p]] < bl) {
        bl = row_len[(size_t)node_of[(size_t)p]];
        best = p;
      }
    while (scan < n && numbered[(size_t)scan]) ++scan;
    return best;
  };
  std::vector<int64_t> last, next;
  std::vector<int64_t> xst((size_t)nnodes, -1), yst((size_t)nnodes, -1);
  std::vector<std::pair<int64_t, int64_t>> keyed;  // (coordination, old position)
  std::vector<int64_t> coord((size_t)nnodes, 0);
  int64_t round = 0;
  while ((int64_t)order.size() < n) {
    if (last.empty()) {
      const int64_t s = start();
      number(s);
      last.assign(1, s);
      continue;
    }
    // neighbours of the last round's DoFs, not numbered yet (sorted by old position)
    ++round;
    next.clear();
    for (int64_t p : last) {
      const int64_t x = node_of[(size_t)p];
      if (xst[(size_t)x] == round) continue;
      xst[(size_t)x] = round;
      for (int64_t t = adj_off[(size_t)x]; t < adj_off[(size_t)x + 1]; ++t) {
        const int64_t y = adj[(size_t)t];
        if (yst[(size_t)y] == round) continue;  // y's DoFs already collected this round
        yst[(size_t)y] = round;
        for (int64_t q = dof_off[(size_t)y]; q < dof_off[(size_t)y + 1]; ++q)
          if (!numbered[(size_t)q]) next.push_back(q);
      }
    }
    std::sort(next.begin(), next.end());
    next.erase(std::unique(next.begin(), next.end()), next.end());
    if (next.empty()) {  // this component of the graph is numbered: start the next one
      last.clear();
      continue;
    }
    // coordination number: not yet numbered DoFs in the row (before this round is numbered)
    keyed.clear();
    int64_t prev_node = -1;
    for (int64_t p : next) {
      const int64_t x = node_of[(size_t)p];
      if (x != prev_node) {
        int64_t cn = 0;
        for (int64_t t = adj_off[(size_t)x]; t < adj_off[(size_t)x + 1]; ++t) cn += unnum[(size_t)adj[(size_t)t]];
        coord[(size_t)x] = cn;
        prev_node = x;
      }
      keyed.push_back({coord[(size_t)x], p});
    }
    std::stable_sort(keyed.begin(), keyed.end());
    for (auto &kp : keyed) number(kp.second);
    last = next;
  }
}

}  // namespace gls

// C-ABI export of the symbolic ILU(k) for host-side tests (no device involved)
extern "C" int gls_iluk_pattern(int64_t n, const int32_t *rowp, const int32_t *col, int fill, int32_t *out_rowp,
                                int32_t *out_col, int32_t *out_level, int64_t capacity, int64_t *out_nnz) {
  std::vector<int32_t> orow, ocol, olev;
  const int rc = gls::iluk_pattern(n, rowp, col, fill, orow, ocol, &olev);
  if (rc != GLS_OK) return rc;
  if (out_nnz) *out_nnz = (int64_t)ocol.size();
  if (!out_col && !out_rowp && !out_level) return GLS_OK;  // size query
  if ((int64_t)ocol.size() > capacity) return GLS_EINVAL;
  if (out_rowp) std::memcpy(out_rowp, orow.data(), sizeof(int32_t) * orow.size());
  if (out_col) std::memcpy(out_col, ocol.data(), sizeof(int32_t) * ocol.size());
  if (out_level) std::memcpy(out_level, olev.data(), sizeof(int32_t) * olev.size());
  return GLS_OK;
}

// C-ABI export of the Cuthill-McKee renumbering for host-side tests: order[new index] = DoF
extern "C" int gls_cuthill_mckee(int64_t n_nodes, const int64_t *adj_off, const int64_t *adj, const int64_t *dof_off,
                                 const int64_t *dofs, int64_t *order) {
  if (n_nodes < 0 || !adj_off || !dof_off || !order) return GLS_EINVAL;
  std::vector<int64_t> ao(adj_off, adj_off + n_nodes + 1), a(adj, adj + adj_off[n_nodes]);
  std::vector<int64_t> doff(dof_off, dof_off + n_nodes + 1), d(dofs, dofs + dof_off[n_nodes]), o;
  gls::cuthill_mckee_nodes(n_nodes, ao, a, doff, d, o);
  std::memcpy(order, o.data(), sizeof(int64_t) * o.size());
  return GLS_OK;
}
