// Strategy search over per-op parallel configurations.
//
// search_dp   — exact dynamic programming over the topologically ordered PCG with a *frontier*
//               state: the configs of ops whose outputs are still consumed later. Chains are
//               O(nodes x cands^2); residual/skip structure (BERT, ResNet, Inception) keeps the
//               frontier at 2-4 ops. A beam bounds the state count on wide graphs. This plays the
//               role of Unity's SearchHelper::graph_cost sequence/parallel splits
//               (reference src/runtime/substitution.cc, graph.cc:2047-2318) with an additive
//               compute + edge-transfer + (half-overlapped) gradient-sync objective.
// search_mcmc — the reference's Metropolis-Hastings search (model.cc:3286-3357, dead code there)
//               revived on the full overlapping task-graph simulator.
// search_unity— DP seed, then simulator-driven MCMC refinement (captures inter-op concurrency
//               and comm/compute overlap the additive DP cannot see).
#include <algorithm>
#include <cmath>
#include <map>
#include <unordered_map>

#include "pcg.h"

namespace ffcore {

namespace {

struct KeyHash {
  size_t operator()(const std::vector<int>& v) const {
    uint64_t h = 1469598103934665603ull;
    for (int x : v) h = (h ^ (uint64_t)(x + 1)) * 1099511628211ull;
    return (size_t)h;
  }
};

}  // namespace

SearchResult search_dp(const Problem& p, int beam) {
  const int N = (int)p.nodes.size();
  Simulator sim(p);
  // last consumer index of every node
  std::vector<int> last_use(N, -1);
  for (int i = 0; i < N; ++i)
    for (auto& in : p.nodes[i].inputs)
      if (in.first >= 0) last_use[in.first] = std::max(last_use[in.first], i);

  // state: ordered list of live node ids + their chosen configs
  std::vector<int> live;  // node ids (sorted by id)
  struct Entry {
    double cost;
    int back;  // index into previous step's entry list
    int cfg;   // config chosen for the node added at this step
  };
  std::vector<std::vector<Entry>> hist;
  std::vector<std::vector<std::vector<int>>> keys_hist;
  std::vector<std::vector<int>> cur_keys = {{}};
  std::vector<Entry> cur = {{0.0, -1, -1}};
  int64_t states = 0;

  for (int i = 0; i < N; ++i) {
    const Node& n = p.nodes[i];
    // positions of this node's producers within the live list
    std::vector<int> prod_pos(n.inputs.size(), -1);
    for (size_t s = 0; s < n.inputs.size(); ++s) {
      const int pr = n.inputs[s].first;
      if (pr < 0) continue;
      auto it = std::find(live.begin(), live.end(), pr);
      prod_pos[s] = (int)(it - live.begin());
    }
    // next live set
    std::vector<int> nlive;
    for (int x : live)
      if (last_use[x] > i) nlive.push_back(x);
    const bool keep_self = last_use[i] > i;
    if (keep_self) nlive.push_back(i);
    std::vector<int> keep_pos;
    for (size_t k = 0; k < live.size(); ++k)
      if (last_use[live[k]] > i) keep_pos.push_back((int)k);

    std::unordered_map<std::vector<int>, int, KeyHash> index;
    std::vector<std::vector<int>> nkeys;
    std::vector<Entry> next;
    std::vector<int> prod_cfg(n.inputs.size(), 0);
    for (size_t e = 0; e < cur.size(); ++e) {
      const auto& key = cur_keys[e];
      for (size_t s = 0; s < n.inputs.size(); ++s) prod_cfg[s] = prod_pos[s] >= 0 ? key[prod_pos[s]] : 0;
      for (int c = 0; c < (int)n.cands.size(); ++c) {
        const double cost = cur[e].cost + sim.node_cost(i, c, prod_cfg);
        std::vector<int> nk;
        nk.reserve(nlive.size());
        for (int kp : keep_pos) nk.push_back(key[kp]);
        if (keep_self) nk.push_back(c);
        auto it = index.find(nk);
        if (it == index.end()) {
          index.emplace(nk, (int)next.size());
          nkeys.push_back(std::move(nk));
          next.push_back({cost, (int)e, c});
        } else if (cost < next[it->second].cost) {
          next[it->second] = {cost, (int)e, c};
        }
        ++states;
      }
    }
    if ((int)next.size() > beam) {  // keep the best `beam` frontier states
      std::vector<int> ord(next.size());
      for (size_t k = 0; k < ord.size(); ++k) ord[k] = (int)k;
      std::nth_element(ord.begin(), ord.begin() + beam, ord.end(),
                       [&](int a, int b) { return next[a].cost < next[b].cost; });
      ord.resize(beam);
      std::vector<Entry> n2;
      std::vector<std::vector<int>> k2;
      for (int k : ord) {
        n2.push_back(next[k]);
        k2.push_back(nkeys[k]);
      }
      next.swap(n2);
      nkeys.swap(k2);
    }
    hist.push_back(next);
    keys_hist.push_back(nkeys);
    cur.swap(next);
    cur_keys.swap(nkeys);
    live.swap(nlive);
  }
  // best final state, then backtrack
  int best = 0;
  for (size_t e = 0; e < cur.size(); ++e)
    if (cur[e].cost < cur[best].cost) best = (int)e;
  SearchResult r;
  r.choice.assign(N, 0);
  r.dp_cost_ms = cur.empty() ? 0 : cur[best].cost;
  int e = best;
  for (int i = N - 1; i >= 0; --i) {
    r.choice[i] = hist[i][e].cfg;
    e = hist[i][e].back;
  }
  r.states = states;
  r.sim_ms = sim.simulate(r.choice).makespan_ms;
  r.cost_ms = r.sim_ms;
  return r;
}

SearchResult search_mcmc(const Problem& p, const std::vector<int>& init, int iterations, double alpha,
                         uint64_t seed) {
  const int N = (int)p.nodes.size();
  Simulator sim(p);
  std::mt19937_64 rng(seed);
  std::vector<int> cur = init;
  if ((int)cur.size() != N) cur.assign(N, 0);
  double cur_cost = sim.simulate(cur).makespan_ms;
  std::vector<int> best = cur;
  double best_cost = cur_cost;
  SearchResult r;
  std::vector<int> movable;
  for (int i = 0; i < N; ++i)
    if (p.nodes[i].cands.size() > 1) movable.push_back(i);
  if (movable.empty()) {
    r.choice = cur;
    r.cost_ms = r.sim_ms = cur_cost;
    return r;
  }
  std::uniform_real_distribution<double> U(0.0, 1.0);
  for (int it = 0; it < iterations; ++it) {
    const int node = movable[rng() % movable.size()];
    const int old = cur[node];
    int nc = (int)(rng() % p.nodes[node].cands.size());
    if (nc == old) nc = (nc + 1) % (int)p.nodes[node].cands.size();
    cur[node] = nc;
    // occasionally propagate the same config index to the neighbouring op (reference
    // enable_propagation: neighbours often want matching layouts)
    int prop_node = -1, prop_old = -1;
    if (U(rng) < 0.3) {
      for (auto& in : p.nodes[node].inputs) {
        const int pr = in.first;
        if (pr >= 0 && nc < (int)p.nodes[pr].cands.size() &&
            p.nodes[pr].cands[nc].degrees.size() == p.nodes[node].cands[nc].degrees.size()) {
          prop_node = pr;
          prop_old = cur[pr];
          cur[pr] = nc;
          break;
        }
      }
    }
    const double c = sim.simulate(cur).makespan_ms;
    const double delta = c - cur_cost;
    if (delta < 0 || U(rng) < std::exp(-alpha * delta / std::max(cur_cost, 1e-9) * 100.0)) {
      cur_cost = c;
      if (c < best_cost) {
        best_cost = c;
        best = cur;
      }
    } else {
      cur[node] = old;
      if (prop_node >= 0) cur[prop_node] = prop_old;
    }
    if ((it & 63) == 0) r.trace.push_back(best_cost);
  }
  r.choice = best;
  r.cost_ms = r.sim_ms = best_cost;
  r.iterations = iterations;
  return r;
}

SearchResult search_unity(const Problem& p, int beam, int refine_iters, double alpha, uint64_t seed) {
  SearchResult d = search_dp(p, beam);
  if (refine_iters <= 0) return d;
  SearchResult m = search_mcmc(p, d.choice, refine_iters, alpha, seed);
  if (m.cost_ms < d.cost_ms) {
    m.dp_cost_ms = d.dp_cost_ms;
    m.states = d.states;
    return m;
  }
  return d;
}

}  // namespace ffcore
