// amg_graph.h -- host-side aggregation of the AMG hierarchy (plain C++): shared by the gfx950 V-cycle
// (amg.hip, which uploads the result) and the CPU-A baseline (baseline/cpu_a), so both precondition
// with the same hierarchy. Algorithm: three greedy pairwise-matching passes per level on the strength
// graph |Sf| * deltaCoeffs (AmgX SIZE_2 selector applied three times: 2x2x2 on a uniform hex mesh);
// piecewise-constant prolongation; Galerkin coarse operators summed from fixed-order contribution lists.
#pragma once
#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdint>
#include <numeric>
#include <utility>
#include <vector>

namespace dfmi {

struct Graph {                  // symmetric strength graph, CSR, no self entries
  int n = 0;
  std::vector<int> start, adj;
  std::vector<double> w;
};

// strength graph of a mesh: face couplings (own, nei, strength) plus cyclic couplings (one entry per
// slot, from the slot's cell to its partner), parallel couplings summed
inline Graph strength_graph(int C, const std::vector<int>& fo, const std::vector<int>& fn, const std::vector<double>& fs,
                            const std::vector<int>& co, const std::vector<int>& cn, const std::vector<double>& cs) {
  std::vector<std::vector<std::pair<int, double>>> e(C);
  for (size_t f = 0; f < fo.size(); ++f) { e[fo[f]].push_back({fn[f], fs[f]}); e[fn[f]].push_back({fo[f], fs[f]}); }
  for (size_t i = 0; i < co.size(); ++i)
    if (co[i] != cn[i]) e[co[i]].push_back({cn[i], cs[i]});
  Graph g;
  g.n = C;
  g.start.assign(C + 1, 0);
  for (int c = 0; c < C; ++c) {
    auto& l = e[c];
    std::sort(l.begin(), l.end(), [](auto& u, auto& v) { return u.first < v.first; });
    std::vector<std::pair<int, double>> m;
    for (auto& p : l) {
      if (!m.empty() && m.back().first == p.first) m.back().second += p.second;
      else m.push_back(p);
    }
    for (auto& p : m) { g.adj.push_back(p.first); g.w.push_back(p.second); }
    g.start[c + 1] = (int)g.adj.size();
  }
  return g;
}

// one greedy pairwise matching on g: each unmatched vertex (in index order) pairs with its
// strongest unmatched neighbour (ties: lowest index). Returns group id per vertex, group count.
inline int pair_match(const Graph& g, std::vector<int>& grp) {
  grp.assign(g.n, -1);
  int ng = 0;
  for (int v = 0; v < g.n; ++v) {
    if (grp[v] >= 0) continue;
    int best = -1;
    double bw = -1.0;
    for (int e = g.start[v]; e < g.start[v + 1]; ++e) {
      const int u = g.adj[e];
      if (u == v || grp[u] >= 0) continue;
      // strengths within 1e-9 relative are ties (rounding must not break the geometric pattern)
      if (g.w[e] > bw * (1 + 1e-9)) { bw = g.w[e]; best = u; }
      else if (std::fabs(g.w[e] - bw) <= 1e-9 * bw && u < best) best = u;
    }
    grp[v] = ng;
    if (best >= 0) grp[best] = ng;
    ++ng;
  }
  return ng;
}

// collapse g by a grouping (edge strengths summed, intra-group edges dropped)
inline Graph collapse(const Graph& g, const std::vector<int>& grp, int ng) {
  std::vector<std::vector<std::pair<int, double>>> e(ng);
  for (int v = 0; v < g.n; ++v)
    for (int k = g.start[v]; k < g.start[v + 1]; ++k) {
      const int a = grp[v], b = grp[g.adj[k]];
      if (a != b) e[a].push_back({b, g.w[k]});
    }
  Graph c;
  c.n = ng;
  c.start.assign(ng + 1, 0);
  for (int a = 0; a < ng; ++a) {
    auto& l = e[a];
    std::sort(l.begin(), l.end(), [](auto& x, auto& y) { return x.first < y.first; });
    std::vector<std::pair<int, double>> m;
    for (auto& p : l) {
      if (!m.empty() && m.back().first == p.first) m.back().second += p.second;
      else m.push_back(p);
    }
    for (auto& p : m) { c.adj.push_back(p.first); c.w.push_back(p.second); }
    c.start[a + 1] = (int)c.adj.size();
  }
  return c;
}

// the next level below a fine level (ELL columns fcol [Wf][nf], columns >= nf are halo entries and
// dropped; padding repeats the row's own cell): aggregates, members, coarse ELL columns, Galerkin lists
struct AmgCoarse {
  int nc = 0, Wc = 1;
  std::vector<int> agg, mstart, members, ccol, gstart, gsrc;
  Graph cg;
};

// the member lists, coarse ELL columns and Galerkin contribution lists of a coarse level, given the
// fine -> coarse map r.agg (any numbering of the nc coarse cells; a coarse cell may have no members:
// its row is all padding and its diagonal list is empty)
inline void amg_level_data(const std::vector<int>& fcol, int Wf, int nf, int nc, AmgCoarse& r) {
  const std::vector<int>& agg = r.agg;
  r.nc = nc;
  r.mstart.assign(nc + 1, 0);
  r.members.resize(nf);
  for (int v = 0; v < nf; ++v) r.mstart[agg[v] + 1]++;
  for (int i = 0; i < nc; ++i) r.mstart[i + 1] += r.mstart[i];
  {
    std::vector<int> pos(r.mstart.begin(), r.mstart.end() - 1);
    for (int v = 0; v < nf; ++v) r.members[pos[agg[v]]++] = v;
  }
  // coarse ELL columns: sorted unique neighbour aggregates over rank-local fine couplings
  std::vector<std::vector<int>> nb(nc);
  for (int v = 0; v < nf; ++v)
    for (int k = 0; k < Wf; ++k) {
      const int j = fcol[(size_t)k * nf + v];
      if (j >= nf || j == v) continue;    // halo or padding
      const int A = agg[v], Bc = agg[j];
      if (A != Bc) nb[A].push_back(Bc);
    }
  int Wc = 1;
  for (auto& l : nb) {
    std::sort(l.begin(), l.end());
    l.erase(std::unique(l.begin(), l.end()), l.end());
    Wc = std::max(Wc, (int)l.size());
  }
  r.Wc = Wc;
  r.ccol.assign((size_t)Wc * nc, 0);
  for (int I = 0; I < nc; ++I)
    for (int k = 0; k < Wc; ++k) r.ccol[(size_t)k * nc + I] = k < (int)nb[I].size() ? nb[I][k] : I;
  // Galerkin contribution lists: slot k < Wc -> coarse entry (I, nb[I][k]); slot Wc -> diagonal.
  // Fine sources in (member ascending, fine slot ascending) order; fine diag first per member.
  // A source s >= 0 is fine entry s = k * nf + v of the ELL values; s < 0 is fine diagonal -s - 1.
  const int slots = Wc + 1;
  std::vector<std::vector<int>> lists((size_t)slots * nc);
  for (int I = 0; I < nc; ++I) {
    for (int e = r.mstart[I]; e < r.mstart[I + 1]; ++e) {
      const int v = r.members[e];
      lists[(size_t)Wc * nc + I].push_back(-(v + 1));
      for (int k = 0; k < Wf; ++k) {
        const int j = fcol[(size_t)k * nf + v];
        if (j >= nf || j == v) continue;
        const int src = k * nf + v;
        const int Bc = agg[j];
        if (Bc == I) lists[(size_t)Wc * nc + I].push_back(src);
        else {
          const int kk = (int)(std::lower_bound(nb[I].begin(), nb[I].end(), Bc) - nb[I].begin());
          lists[(size_t)kk * nc + I].push_back(src);
        }
      }
    }
  }
  r.gstart.assign((size_t)slots * nc + 1, 0);
  for (size_t s = 0; s < lists.size(); ++s) {
    for (int v : lists[s]) r.gsrc.push_back(v);
    r.gstart[s + 1] = (int)r.gsrc.size();
  }
  if (r.gsrc.empty()) r.gsrc.push_back(0);
}

inline AmgCoarse amg_coarsen(const std::vector<int>& fcol, int Wf, int nf, const Graph& g, int passes = 3) {
  AmgCoarse r;
  // `passes` pairwise passes -> aggregates of up to 2^passes cells (3: 2x2x2 on a hex mesh)
  std::vector<int>& agg = r.agg;
  agg.resize(nf);
  std::iota(agg.begin(), agg.end(), 0);
  Graph cur = g;
  int ng = nf;
  for (int pass = 0; pass < passes; ++pass) {
    std::vector<int> grp;
    ng = pair_match(cur, grp);
    for (int v = 0; v < nf; ++v) agg[v] = grp[agg[v]];
    cur = collapse(cur, grp, ng);
  }
  // renumber coarse cells by their first fine member (locality)
  std::vector<int> first(ng, INT32_MAX);
  for (int v = 0; v < nf; ++v) first[agg[v]] = std::min(first[agg[v]], v);
  std::vector<int> ord(ng);
  std::iota(ord.begin(), ord.end(), 0);
  std::sort(ord.begin(), ord.end(), [&](int a, int b) { return first[a] < first[b]; });
  std::vector<int> ren(ng);
  for (int i = 0; i < ng; ++i) ren[ord[i]] = i;
  for (int v = 0; v < nf; ++v) agg[v] = ren[agg[v]];
  const int nc = ng;
  r.cg = collapse(g, agg, nc);   // coarse strength graph (same collapse, renumbered)
  amg_level_data(fcol, Wf, nf, nc, r);
  return r;
}

}  // namespace dfmi
