// Host sparse-pattern algorithms for the assembled ILU(k) (gls_sparse.cpp)
#pragma once
#include <cstdint>
#include <vector>

namespace gls {
// Ifpack ILU(k) level-of-fill pattern of the CSR graph (rowp, col) of an n x n matrix; the diagonal is
// always included. Output rows sorted; olev (optional) holds each entry's level.
// RP: the row-pointer / entry-position type (int32_t, or int64_t for matrices past 2^31 entries).
template <typename RP>
int iluk_pattern(int64_t n, const RP *rowp, const int32_t *col, int fill, std::vector<RP> &orow,
                 std::vector<int32_t> &ocol, std::vector<int32_t> *olev = nullptr);
// deal.II Cuthill-McKee on a node graph (adj: a node's row nodes, itself included) whose nodes own
// the consecutive DoFs dofs[dof_off[x] .. dof_off[x+1]); order[new index] = DoF
void cuthill_mckee_nodes(int64_t nnodes, const std::vector<int64_t> &adj_off, const std::vector<int64_t> &adj,
                         const std::vector<int64_t> &dof_off, const std::vector<int64_t> &dofs,
                         std::vector<int64_t> &order);
}  // namespace gls
