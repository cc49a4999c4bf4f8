// renumber.cpp -- cell renumbering for coalesced, cache-local gathers (the role OpenFOAM's
// renumberMesh utility plays for CPU runs; SURVEY.md 7 "cells renumbered", north star
// "cells renumbered for coalesced HBM reads").
//
// The FV kernels are cell-centric gathers: thread c reads its own cell's values (coalesced in any
// order) and its neighbours' (scattered). In blockMesh / lexicographic order a cell's y- and
// z-neighbours sit a row and a plane away (128 and 16384 cells on a 128^3 box), so a plane of every
// gathered species array must stay in the 4 MB L2 of an XCD -- it does not, and the neighbours are
// read from HBM again and again (k_y_prep: 2.4x its algorithmic bytes). Ordering the cells along a
// Morton (Z-order) curve of their centres makes every aligned 2^k-cell run a compact brick (256
// consecutive cells = an 8x8x4 brick): most neighbours of a workgroup's cells are the workgroup's own
// cells or those of the workgroups just before/after it.
//
// Host-side, once per mesh, before dfmi_set_constant_indexes (as renumberMesh runs before the
// solver): the caller permutes its cell and face data with the returned maps. Faces are re-sorted into
// upper-triangular order (owner < neighbour, by owner then neighbour); a face whose owner and
// neighbour swap is flagged so the caller negates its area vector / fluxes (Sf, phi), mirrors its
// interpolation weight (w -> 1 - w) and reverses the centre-to-centre vector. A Morton order of an
// axis-aligned structured box is monotone in every coordinate, so there no face flips.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <numeric>
#include <stdexcept>
#include <string>
#include <vector>

namespace {

// spread the low 21 bits of v so that bit i lands at bit 3i
uint64_t spread3(uint64_t v) {
  v &= 0x1fffffULL;
  v = (v | v << 32) & 0x1f00000000ffffULL;
  v = (v | v << 16) & 0x1f0000ff0000ffULL;
  v = (v | v << 8) & 0x100f00f00f00f00fULL;
  v = (v | v << 4) & 0x10c30c30c30c30c3ULL;
  v = (v | v << 2) & 0x1249249249249249ULL;
  return v;
}

// Morton order of the cell centres: each axis quantised into 2^21 bins over the bounding box (an
// affine, monotone map, so the grid lines of a structured mesh never merge); ties keep the old order
void morton_order(int C, const double* cc, std::vector<int>& order) {
  double lo[3], hi[3];
  for (int k = 0; k < 3; ++k) { lo[k] = 1e300; hi[k] = -1e300; }
  for (int c = 0; c < C; ++c)
    for (int k = 0; k < 3; ++k) { lo[k] = std::min(lo[k], cc[3L * c + k]); hi[k] = std::max(hi[k], cc[3L * c + k]); }
  const double nb = (double)((1 << 21) - 1);
  std::vector<uint64_t> key(C);
  for (int c = 0; c < C; ++c) {
    uint64_t code = 0;
    for (int k = 0; k < 3; ++k) {
      const double span = hi[k] - lo[k];
      const double f = span > 0 ? (cc[3L * c + k] - lo[k]) / span : 0.0;
      code |= spread3((uint64_t)std::llround(f * nb)) << k;   // x in bit 0, y bit 1, z bit 2
    }
    key[c] = code;
  }
  order.resize(C);
  std::iota(order.begin(), order.end(), 0);
  std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return key[a] < key[b]; });
}

// Morton order of 8 x 8 x 4 bricks, lexicographic (x fastest) inside a brick: one 64-lane wave is an
// 8 x 8 layer of a brick, so its own-cell reads, its -x/-y neighbours (c-1, c-8) and its -z neighbours
// (the layer below, contiguous even across a brick boundary) coalesce, while the bricks themselves
// follow a Z-order curve, so a brick's neighbour bricks are a few bricks away at every level (and each
// XCD's contiguous eighth of the cells is a compact octant). Needs integer (i, j, k) cell coordinates
// (structured blocks); monotone in each coordinate, so no face flips.
void brick_order(int C, const double* ijk, std::vector<int>& order) {
  constexpr int BX = 8, BY = 8, BZ = 4;
  std::vector<uint64_t> key(C);
  for (int c = 0; c < C; ++c) {
    long v[3];
    for (int k = 0; k < 3; ++k) {
      const double d = ijk[3L * c + k];
      v[k] = std::lround(d);
      if (std::fabs(d - (double)v[k]) > 1e-9 || v[k] < 0) throw std::runtime_error("dfmi: renumber: bricks needs integer (i, j, k) cell coordinates >= 0");
    }
    const uint64_t b = spread3((uint64_t)(v[0] / BX)) | spread3((uint64_t)(v[1] / BY)) << 1 | spread3((uint64_t)(v[2] / BZ)) << 2;
    const uint64_t in = (uint64_t)(v[0] % BX) + BX * ((uint64_t)(v[1] % BY) + BY * (uint64_t)(v[2] % BZ));
    key[c] = b << 8 | in;
  }
  order.resize(C);
  std::iota(order.begin(), order.end(), 0);
  std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return key[a] < key[b]; });
}

// reverse Cuthill-McKee on the face graph (renumberMesh's default CuthillMcKee, reversed): needs no
// geometry; bandwidth-reducing rather than brick-forming
void rcm_order(int C, int F, const int* own, const int* nei, std::vector<int>& order) {
  std::vector<int> deg(C, 0), start(C + 1, 0), adj(2L * F);
  for (int f = 0; f < F; ++f) { deg[own[f]]++; deg[nei[f]]++; }
  for (int c = 0; c < C; ++c) start[c + 1] = start[c] + deg[c];
  std::vector<int> pos(start.begin(), start.end() - 1);
  for (int f = 0; f < F; ++f) { adj[pos[own[f]]++] = nei[f]; adj[pos[nei[f]]++] = own[f]; }
  for (int c = 0; c < C; ++c)
    std::sort(adj.begin() + start[c], adj.begin() + start[c + 1], [&](int a, int b) { return deg[a] < deg[b] || (deg[a] == deg[b] && a < b); });
  std::vector<char> seen(C, 0);
  order.clear();
  order.reserve(C);
  std::vector<int> byDeg(C);
  std::iota(byDeg.begin(), byDeg.end(), 0);
  std::stable_sort(byDeg.begin(), byDeg.end(), [&](int a, int b) { return deg[a] < deg[b]; });
  for (int s : byDeg) {   // one BFS per connected component, from a minimum-degree cell
    if (seen[s]) continue;
    size_t head = order.size();
    order.push_back(s);
    seen[s] = 1;
    while (head < order.size()) {
      const int c = order[head++];
      for (int e = start[c]; e < start[c + 1]; ++e)
        if (!seen[adj[e]]) { seen[adj[e]] = 1; order.push_back(adj[e]); }
    }
  }
  std::reverse(order.begin(), order.end());
}

}  // namespace

namespace dfmi {

void renumber_cells(int num_cells, const double* cell_centres, int num_faces, const int* owner, const int* neighbour,
                    const char* method, int* new_to_old) {
  if (num_cells <= 0 || !new_to_old || !method) throw std::runtime_error("dfmi: renumber: bad arguments");
  std::string m(method);
  std::vector<int> order;
  if (m == "morton") {
    if (!cell_centres) throw std::runtime_error("dfmi: renumber: morton needs the cell centres");
    morton_order(num_cells, cell_centres, order);
  } else if (m == "bricks") {
    if (!cell_centres) throw std::runtime_error("dfmi: renumber: bricks needs (i, j, k) cell coordinates");
    brick_order(num_cells, cell_centres, order);
  } else if (m == "rcm") {
    if (num_faces < 0 || (num_faces > 0 && (!owner || !neighbour))) throw std::runtime_error("dfmi: renumber: rcm needs owner/neighbour");
    rcm_order(num_cells, num_faces, owner, neighbour, order);
  } else if (m == "none") {
    order.resize(num_cells);
    std::iota(order.begin(), order.end(), 0);
  } else {
    throw std::runtime_error("dfmi: renumber: method must be 'bricks', 'morton', 'rcm' or 'none'");
  }
  std::memcpy(new_to_old, order.data(), sizeof(int) * num_cells);
}

void renumber_faces(int num_cells, int num_faces, const int* owner, const int* neighbour, const int* cell_new_to_old,
                    int* face_new_to_old, int* new_owner, int* new_neighbour, int* flipped) {
  if (num_cells <= 0 || num_faces < 0) throw std::runtime_error("dfmi: renumber: bad sizes");
  std::vector<int> inv(num_cells, -1);
  for (int n = 0; n < num_cells; ++n) {
    const int o = cell_new_to_old[n];
    if (o < 0 || o >= num_cells || inv[o] >= 0) throw std::runtime_error("dfmi: renumber: cell map is not a permutation");
    inv[o] = n;
  }
  std::vector<int> a(num_faces), b(num_faces), fl(num_faces), ord(num_faces);
  for (int f = 0; f < num_faces; ++f) {
    int x = inv[owner[f]], y = inv[neighbour[f]];
    fl[f] = x > y;
    if (fl[f]) std::swap(x, y);
    a[f] = x; b[f] = y;
  }
  std::iota(ord.begin(), ord.end(), 0);
  std::stable_sort(ord.begin(), ord.end(), [&](int p, int q) { return a[p] < a[q] || (a[p] == a[q] && b[p] < b[q]); });
  for (int n = 0; n < num_faces; ++n) {
    const int f = ord[n];
    face_new_to_old[n] = f;
    new_owner[n] = a[f];
    new_neighbour[n] = b[f];
    flipped[n] = fl[f];
  }
}

}  // namespace dfmi
