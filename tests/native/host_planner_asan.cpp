// Host-code sanitizer check (test infrastructure): the C-ABI's host-side graph planners --
// gine_graph_order_locality (gine_graph.hip), gine_graph_plan_windows and
// gine_graph_plan_window_slots (gine_mpwin.hip) -- built with AddressSanitizer and
// UndefinedBehaviorSanitizer on the host side only (csrc/Makefile `hostasan`), run on
// synthetic CSRs, edge cases included, with every output checked for its contract.  No GPU
// call is made.  Exit status 0 = all checks passed.
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "gine_hip.h"

static int g_fail = 0;
#define CHECK(c, ...)                                              \
  do {                                                             \
    if (!(c)) {                                                    \
      std::fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__);    \
      std::fprintf(stderr, __VA_ARGS__);                           \
      std::fprintf(stderr, "\n");                                  \
      ++g_fail;                                                    \
    }                                                              \
  } while (0)

struct Csr {
  int n;
  std::vector<int32_t> rowptr, nbr;
};

// CSR of the node's neighbours from (src, dst) edges, grouped by dst (edge order kept)
static Csr make_csr(int n, const std::vector<std::pair<int, int>>& edges) {
  Csr c;
  c.n = n;
  c.rowptr.assign(n + 1, 0);
  for (auto& e : edges) ++c.rowptr[e.second + 1];
  for (int v = 0; v < n; ++v) c.rowptr[v + 1] += c.rowptr[v];
  c.nbr.resize(edges.size());
  std::vector<int32_t> fill(c.rowptr.begin(), c.rowptr.end() - 1);
  for (auto& e : edges) c.nbr[fill[e.second]++] = e.first;
  return c;
}

// k nearest on a ring (a station-graph stand-in), self loops, optional random long edges
static Csr ring_knn(int n, int k, int extra, std::mt19937& rng) {
  std::vector<std::pair<int, int>> e;
  for (int v = 0; v < n; ++v) {
    e.push_back({v, v});
    for (int j = 1; j <= k / 2 && n > 1; ++j) {
      e.push_back({(v + j) % n, v});
      e.push_back({(v - j + n) % n, v});
    }
  }
  for (int i = 0; i < extra && n > 0; ++i) e.push_back({(int)(rng() % n), (int)(rng() % n)});
  std::shuffle(e.begin(), e.end(), rng);
  return make_csr(n, e);
}

// power-law sources (hubs), isolated targets
static Csr hubs(int n, int m, std::mt19937& rng) {
  std::vector<std::pair<int, int>> e;
  std::uniform_real_distribution<double> u(0.0, 1.0);
  for (int i = 0; i < m && n > 2; ++i) {
    const int s = std::min(n - 1, (int)(n * u(rng) * u(rng) * u(rng)));
    e.push_back({s, (int)(rng() % (n - 2))});
  }
  return make_csr(n, e);
}

static void check_order(const Csr& g) {
  std::vector<int32_t> order(std::max(g.n, 1), -7);
  const int st = gine_graph_order_locality(g.rowptr.data(), g.nbr.empty() ? nullptr : g.nbr.data(),
                                           g.n, order.data());
  CHECK(st == GINE_OK, "order_locality status %d (n=%d)", st, g.n);
  std::vector<int> seen(g.n, 0);
  for (int i = 0; i < g.n; ++i) {
    CHECK(order[i] >= 0 && order[i] < g.n, "order[%d]=%d outside [0,%d)", i, order[i], g.n);
    if (order[i] >= 0 && order[i] < g.n) ++seen[order[i]];
  }
  for (int v = 0; v < g.n; ++v) CHECK(seen[v] == 1, "node %d placed %d times", v, seen[v]);
}

static void check_plan(const Csr& g, int max_rows, int max_nodes, int max_edges) {
  const int n = g.n;
  std::vector<int32_t> tb(n + 1, -1), lo(std::max(n, 1), -1), rows(std::max(n, 1), -1);
  int32_t T = -1, maxima[3] = {-1, -1, -1};
  const int st = gine_graph_plan_windows(g.rowptr.data(), g.nbr.empty() ? nullptr : g.nbr.data(),
                                         n, max_rows, max_nodes, max_edges, tb.data(), lo.data(),
                                         rows.data(), &T, maxima);
  CHECK(st == GINE_OK, "plan_windows status %d", st);
  CHECK(T >= 0 && T <= n, "num_tiles %d (n=%d)", T, n);
  if (T <= 0) return;  // no plan (a node wider than the window or with too many edges)
  CHECK(tb[0] == 0 && tb[T] == n, "tile bounds %d..%d", tb[0], tb[T]);
  int mr = 0, me = 0, mn = 0;
  for (int t = 0; t < T; ++t) {
    const int a = tb[t], b = tb[t + 1];
    CHECK(b > a, "empty tile %d", t);
    CHECK(b - a <= max_nodes, "tile %d has %d nodes > %d", t, b - a, max_nodes);
    const int edges = g.rowptr[b] - g.rowptr[a];
    CHECK(edges <= max_edges, "tile %d has %d edges > %d", t, edges, max_edges);
    CHECK(rows[t] >= 0 && rows[t] <= max_rows, "tile %d window %d rows", t, rows[t]);
    for (int e = g.rowptr[a]; e < g.rowptr[b]; ++e)
      CHECK(g.nbr[e] >= lo[t] && g.nbr[e] < lo[t] + rows[t], "tile %d misses neighbour %d",
            t, g.nbr[e]);
    mr = std::max(mr, (int)rows[t]);
    me = std::max(me, edges);
    mn = std::max(mn, b - a);
  }
  CHECK(maxima[0] == mr && maxima[1] == me && maxima[2] == mn, "maxima %d %d %d vs %d %d %d",
        maxima[0], maxima[1], maxima[2], mr, me, mn);
  if (max_nodes > 128) return;  // the work order is defined for the backward's tiles
  std::vector<int16_t> slot(n, -1);
  const int ss = gine_graph_plan_window_slots(g.rowptr.data(), tb.data(), T, slot.data());
  CHECK(ss == GINE_OK, "plan_window_slots status %d", ss);
  for (int t = 0; t < T; ++t) {
    const int a = tb[t], b = tb[t + 1];
    std::vector<int> seen(b - a, 0);
    for (int i = a; i < b; ++i) {
      CHECK(slot[i] >= 0 && slot[i] < b - a, "slot[%d]=%d outside tile %d", i, slot[i], t);
      if (slot[i] >= 0 && slot[i] < b - a) ++seen[slot[i]];
    }
    for (int i = 0; i < b - a; ++i) CHECK(seen[i] == 1, "tile %d position %d x%d", t, i, seen[i]);
  }
}

int main() {
  std::mt19937 rng(1234);
  std::vector<Csr> graphs;
  graphs.push_back(make_csr(0, {}));                       // empty
  graphs.push_back(make_csr(1, {}));                       // one node, no edges
  graphs.push_back(make_csr(1, {{0, 0}, {0, 0}, {0, 0}}));  // self loops only
  graphs.push_back(make_csr(7, {}));                       // isolated nodes
  graphs.push_back(ring_knn(500, 10, 0, rng));             // cfg2 station graph shape
  graphs.push_back(ring_knn(2000, 16, 50, rng));           // cfg3 shape + long edges
  graphs.push_back(ring_knn(3000, 32, 0, rng));            // in-degree 33
  graphs.push_back(hubs(200, 3000, rng));                  // hubs, unsorted, isolated
  graphs.push_back(hubs(5000, 40000, rng));
  for (const Csr& g : graphs) {
    check_order(g);
    for (int max_nodes : {1, 64, 128, 1000})
      for (int max_rows : {1, 64, 512, 2048}) check_plan(g, max_rows, max_nodes, 2560);
    check_plan(g, 512, 128, 8);  // edge budget below some nodes' degree: no plan
  }
  // invalid arguments are rejected, not dereferenced
  int32_t T = 0, maxima[3];
  CHECK(gine_graph_plan_windows(nullptr, nullptr, 4, 8, 8, 8, nullptr, nullptr, nullptr, &T,
                                maxima) != GINE_OK, "NULL rowptr accepted");
  CHECK(gine_graph_order_locality(nullptr, nullptr, 4, nullptr) != GINE_OK,
        "NULL order accepted");
  std::printf("host planner checks: %s (%d graphs)\n", g_fail ? "FAILED" : "ok",
              (int)graphs.size());
  return g_fail ? 1 : 0;
}
