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

  // per-(node, config) compute cost and dense per-(node, slot) edge-cost matrices, filled lazily:
  // the state loop below reads them (states x candidates) times per node, so they are plain
  // arrays instead of the simulator's hashed edge cache
  std::vector<std::vector<double>> ncost(N);
  std::vector<std::vector<std::vector<double>>> ecost(N);
  for (int i = 0; i < N; ++i) {
    const Node& n = p.nodes[i];
    ncost[i].resize(n.cands.size());
    for (size_t c = 0; c < n.cands.size(); ++c) {
      const OpCandidate& oc = n.cands[c];
      double ms = oc.fwd_ms + (n.backward ? oc.bwd_ms : 0.0);
      if (n.backward) ms += sim.weight_sync_ms(i, (int)c) * (p.overlap_grad_sync ? 0.5 : 1.0);
      if (oc.mem_bytes > p.machine.mem_capacity) ms += 1e6;
      ncost[i][c] = ms;
    }
    ecost[i].resize(n.inputs.size());
    for (size_t s = 0; s < n.inputs.size(); ++s)
      if (n.inputs[s].first >= 0)
        ecost[i][s].assign(n.cands.size() * p.nodes[n.inputs[s].first].cands.size(), -1.0);
  }
  auto edge = [&](int i, int s, int c, int pc) {
    const size_t np = p.nodes[p.nodes[i].inputs[s].first].cands.size();
    double& v = ecost[i][s][(size_t)c * np + pc];
    if (v < 0) v = sim.edge_cost(i, s, c, pc);
    return v;
  };

  // A state is the configs of the live nodes (those with a later consumer), kept in a flat arena
  // (stride = live count) and indexed by an open-addressing hash table.
  struct Entry {
    double cost;
    int back;  // index into the previous step's entries
    int cfg;   // config chosen for the node added at this step
  };
  std::vector<std::vector<Entry>> hist;
  hist.reserve(N);
  std::vector<int> live;
  std::vector<int> cur_keys;  // flat, stride live.size()
  std::vector<Entry> cur = {{0.0, -1, -1}};
  int64_t states = 0;
  std::vector<int> table;

  for (int i = 0; i < N; ++i) {
    const Node& n = p.nodes[i];
    const int K = (int)live.size();
    std::vector<int> prod_pos(n.inputs.size(), -1);
    for (size_t s = 0; s < n.inputs.size(); ++s) {
      const int pr = n.inputs[s].first;
      if (pr < 0) continue;
      auto it = std::find(live.begin(), live.end(), pr);
      prod_pos[s] = (int)(it - live.begin());
    }
    std::vector<int> nlive, keep_pos;
    for (int k = 0; k < K; ++k)
      if (last_use[live[k]] > i) {
        nlive.push_back(live[k]);
        keep_pos.push_back(k);
      }
    const bool keep_self = last_use[i] > i;
    if (keep_self) nlive.push_back(i);
    const int K2 = (int)nlive.size();
    const int C = (int)n.cands.size();
    const size_t expect = std::min<size_t>((size_t)cur.size() * (keep_self ? C : 1), (size_t)1 << 22);
    size_t cap = 64;
    while (cap < 2 * expect) cap <<= 1;
    table.assign(cap, -1);
    std::vector<Entry> next;
    std::vector<int> nkeys;
    next.reserve(expect);
    nkeys.reserve(expect * K2);
    std::vector<int> prod_cfg(n.inputs.size(), 0);
    std::vector<double> cc(C);
    for (size_t e = 0; e < cur.size(); ++e) {
      const int* key = cur_keys.data() + e * K;
      uint64_t h0 = 1469598103934665603ull;
      for (int kp : keep_pos) h0 = (h0 ^ (uint64_t)(key[kp] + 1)) * 1099511628211ull;
      for (size_t s = 0; s < n.inputs.size(); ++s) prod_cfg[s] = prod_pos[s] >= 0 ? key[prod_pos[s]] : 0;
      for (int c = 0; c < C; ++c) {
        double cost = cur[e].cost + ncost[i][c];
        for (size_t s = 0; s < n.inputs.size(); ++s)
          if (n.inputs[s].first >= 0) cost += edge(i, (int)s, c, prod_cfg[s]);
        cc[c] = cost;
      }
      states += C;
      // without a later consumer this node's config does not enter the state: only the best
      // config per predecessor state can survive
      int c_lo = 0, c_hi = C;
      if (!keep_self) {
        int b = 0;
        for (int c = 1; c < C; ++c)
          if (cc[c] < cc[b]) b = c;
        c_lo = b;
        c_hi = b + 1;
      }
      for (int c = c_lo; c < c_hi; ++c) {
        const uint64_t h = keep_self ? (h0 ^ (uint64_t)(c + 1)) * 1099511628211ull : h0;
        size_t slot = (size_t)(h ^ (h >> 29)) & (cap - 1);
        int found = -1;
        while (table[slot] >= 0) {
          const int* k2 = nkeys.data() + (size_t)table[slot] * K2;
          bool eq = true;
          for (size_t q = 0; q < keep_pos.size() && eq; ++q) eq = k2[q] == key[keep_pos[q]];
          if (eq && keep_self) eq = k2[K2 - 1] == c;
          if (eq) {
            found = table[slot];
            break;
          }
          slot = (slot + 1) & (cap - 1);
        }
        if (found < 0) {
          table[slot] = (int)next.size();
          for (int kp : keep_pos) nkeys.push_back(key[kp]);
          if (keep_self) nkeys.push_back(c);
          next.push_back({cc[c], (int)e, c});
          if (next.size() * 2 > cap) {  // grow and rehash
            cap <<= 1;
            table.assign(cap, -1);
            for (size_t q = 0; q < next.size(); ++q) {
              const int* k2 = nkeys.data() + q * K2;
              uint64_t hh = 1469598103934665603ull;
              for (int t = 0; t < K2 - (keep_self ? 1 : 0); ++t) hh = (hh ^ (uint64_t)(k2[t] + 1)) * 1099511628211ull;
              if (keep_self) hh = (hh ^ (uint64_t)(k2[K2 - 1] + 1)) * 1099511628211ull;
              size_t sl = (size_t)(hh ^ (hh >> 29)) & (cap - 1);
              while (table[sl] >= 0) sl = (sl + 1) & (cap - 1);
              table[sl] = (int)q;
            }
          }
        } else if (cc[c] < next[found].cost) {
          next[found] = {cc[c], (int)e, c};
        }
      }
    }
    if ((int)next.size() > beam) {  // keep the best `beam` frontier states
      std::vector<int> ord(next.size());
      for (size_t k = 0; k < ord.size(); ++k) ord[k] = (int)k;
      std::nth_element(ord.begin(), ord.begin() + beam, ord.end(),
                       [&](int a, int b) { return next[a].cost < next[b].cost; });
      ord.resize(beam);
      std::vector<Entry> n2;
      std::vector<int> k2;
      n2.reserve(beam);
      k2.reserve((size_t)beam * K2);
      for (int k : ord) {
        n2.push_back(next[k]);
        k2.insert(k2.end(), nkeys.begin() + (size_t)k * K2, nkeys.begin() + (size_t)(k + 1) * K2);
      }
      next.swap(n2);
      nkeys.swap(k2);
    }
    hist.push_back(next);
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
  // The DP's objective is additive; the simulator overlaps comm with compute and runs ops on
  // disjoint devices concurrently, so the additive optimum over ALL placements can simulate worse
  // than the optimum over whole-machine placements (DLRM: tables split over device subsets by the
  // DP, 1.12 ms simulated, against 0.92 ms with every table over all 8 GPUs). Seed the refinement
  // with whichever of the two DP solutions simulates faster.
  {
    const int N = (int)p.nodes.size();
    Problem q = p;
    std::vector<std::vector<int>> cmap(N);
    bool differs = false;
    for (int i = 0; i < N; ++i) {
      size_t most = 0;
      for (auto& c : p.nodes[i].cands) most = std::max(most, c.devices.size());
      std::vector<OpCandidate> cc;
      for (size_t c = 0; c < p.nodes[i].cands.size(); ++c)
        if (p.nodes[i].cands[c].devices.size() == most) {
          cc.push_back(p.nodes[i].cands[c]);
          cmap[i].push_back((int)c);
        }
      differs |= cc.size() != p.nodes[i].cands.size();
      q.nodes[i].cands = std::move(cc);
    }
    if (differs) {
      SearchResult w = search_dp(q, beam);
      std::vector<int> ch(N);
      for (int i = 0; i < N; ++i) ch[i] = cmap[i][w.choice[i]];
      const double ws = Simulator(p).simulate(ch).makespan_ms;
      if (ws < d.cost_ms) {
        d.choice = ch;
        d.cost_ms = d.sim_ms = ws;
        d.states += w.states;
      }
    }
  }
  if (refine_iters <= 0) return d;
  SearchResult m = search_mcmc(p, d.choice, refine_iters, alpha, seed);
  if (m.cost_ms < d.cost_ms) {
    m.dp_cost_ms = d.dp_cost_ms;
    m.states = d.states;
    return m;
  }
  return d;
}

std::vector<int> sequence_bottlenecks(const Problem& p) {
  const int N = (int)p.nodes.size();
  std::vector<int> last_use(N, -1);
  for (int i = 0; i < N; ++i)
    for (auto& in : p.nodes[i].inputs)
      if (in.first >= 0) last_use[in.first] = std::max(last_use[in.first], i);
  std::vector<int> out;
  int reach = -1;  // furthest consumer of any node before i
  for (int i = 0; i < N; ++i) {
    if (reach <= i && i > 0) out.push_back(i);
    reach = std::max(reach, last_use[i]);
  }
  return out;
}

namespace {

// Sub-problem over `keep` (sorted node ids); nodes in `fixed` keep one candidate (their baseline
// config) and contribute only their edge costs; the other nodes keep the candidates whose devices
// all lie in [lo, hi). Returns false when some node has no such candidate.
bool sub_problem(const Problem& p, const std::vector<int>& keep, const std::vector<int>& base,
                 const std::vector<char>& fixed, int lo, int hi, Problem& out, std::vector<std::vector<int>>& cand_map) {
  out.machine = p.machine;
  out.update_ms_per_mb = p.update_ms_per_mb;
  out.overlap_grad_sync = p.overlap_grad_sync;
  out.nodes.clear();
  cand_map.clear();
  std::unordered_map<int, int> idx;
  for (size_t k = 0; k < keep.size(); ++k) idx[keep[k]] = (int)k;
  for (int id : keep) {
    Node n = p.nodes[id];
    for (auto& in : n.inputs) {
      auto it = idx.find(in.first);
      in.first = (in.first >= 0 && it != idx.end()) ? it->second : -1;
    }
    std::vector<int> m;
    std::vector<OpCandidate> cc;
    if (fixed[id]) {
      OpCandidate c = p.nodes[id].cands[base[id]];
      c.fwd_ms = c.bwd_ms = 0;
      c.w_layouts.clear();  // boundary op: charged in the whole-graph objective, not here
      cc.push_back(c);
      m.push_back(base[id]);
    } else {
      for (size_t c = 0; c < n.cands.size(); ++c) {
        bool in_range = true;
        for (int d : n.cands[c].devices) in_range &= (d >= lo && d < hi);
        if (in_range) {
          cc.push_back(n.cands[c]);
          m.push_back((int)c);
        }
      }
      if (cc.empty()) return false;
    }
    n.cands = std::move(cc);
    out.nodes.push_back(std::move(n));
    cand_map.push_back(std::move(m));
  }
  return true;
}

}  // namespace

SearchResult search_split(const Problem& p, const std::vector<int>& base, int beam) {
  const int N = (int)p.nodes.size();
  const int D = p.machine.num_devices();
  SearchResult r;
  r.choice = base;
  Simulator full(p);
  double cur_sim = full.simulate(r.choice).makespan_ms;
  std::vector<int> bott = sequence_bottlenecks(p);
  bott.insert(bott.begin(), 0);
  for (size_t b = 0; b + 1 < bott.size(); ++b) {
    const int s = bott[b], e = bott[b + 1];
    if (e - s < 3) continue;  // fewer than two internal nodes
    // independent branches: union-find over edges between internal nodes
    std::vector<int> par(N);
    for (int i = 0; i < N; ++i) par[i] = i;
    std::function<int(int)> find = [&](int x) { return par[x] == x ? x : par[x] = find(par[x]); };
    for (int i = s + 1; i < e; ++i)
      for (auto& in : p.nodes[i].inputs)
        if (in.first > s && in.first < e) par[find(in.first)] = find(i);
    std::map<int, std::vector<int>> comps;
    for (int i = s + 1; i < e; ++i) comps[find(i)].push_back(i);
    if (comps.size() < 2) continue;
    SplitInfo info;
    info.start = s;
    info.end = e;
    info.components = (int)comps.size();
    std::vector<std::vector<int>> branches;
    for (auto& kv : comps) branches.push_back(kv.second);
    // baseline additive cost of each branch (its nodes' costs incl. the fork -> branch edges)
    auto node_cost_base = [&](int i) {
      std::vector<int> prod(p.nodes[i].inputs.size(), 0);
      for (size_t t = 0; t < prod.size(); ++t)
        if (p.nodes[i].inputs[t].first >= 0) prod[t] = r.choice[p.nodes[i].inputs[t].first];
      return full.node_cost(i, r.choice[i], prod);
    };
    std::vector<double> bcost(branches.size(), 0.0);
    for (size_t k = 0; k < branches.size(); ++k)
      for (int i : branches[k]) bcost[k] += node_cost_base(i);
    // join-side edges are part of the region too
    double join_edges = 0;
    for (size_t t = 0; t < p.nodes[e].inputs.size(); ++t) {
      const int pr = p.nodes[e].inputs[t].first;
      if (pr > s && pr < e) join_edges += full.edge_cost(e, (int)t, r.choice[e], r.choice[pr]);
    }
    info.whole_ms = join_edges;
    for (double c : bcost) info.whole_ms += c;
    // try G = 2, 4, ... device groups (aligned blocks), branches dealt largest-first to the
    // least-loaded group (LPT), each group re-searched on its own devices
    double best_split = info.whole_ms, best_sim = 0;
    std::vector<int> best_choice, best_group;
    int best_G = 0;
    for (int G = 2; G <= std::min<int>((int)branches.size(), D); G *= 2) {
      if (D % G) break;
      std::vector<int> order(branches.size());
      for (size_t k = 0; k < order.size(); ++k) order[k] = (int)k;
      std::sort(order.begin(), order.end(), [&](int a, int c) { return bcost[a] > bcost[c]; });
      std::vector<double> load(G, 0.0);
      std::vector<int> group(branches.size(), 0);
      for (int k : order) {
        const int g = (int)(std::min_element(load.begin(), load.end()) - load.begin());
        group[k] = g;
        load[g] += bcost[k];
      }
      std::vector<int> trial = r.choice;
      double worst = 0;
      bool ok = true;
      for (int g = 0; g < G && ok; ++g) {
        std::vector<int> keep = {s};
        for (size_t k = 0; k < branches.size(); ++k)
          if (group[k] == g) keep.insert(keep.end(), branches[k].begin(), branches[k].end());
        if (keep.size() == 1) continue;
        keep.push_back(e);
        std::sort(keep.begin(), keep.end());
        std::vector<char> fixed(N, 0);
        fixed[s] = fixed[e] = 1;
        Problem sp;
        std::vector<std::vector<int>> cmap;
        if (!sub_problem(p, keep, r.choice, fixed, g * (D / G), (g + 1) * (D / G), sp, cmap)) {
          ok = false;
          break;
        }
        SearchResult sr = search_dp(sp, beam);
        worst = std::max(worst, sr.dp_cost_ms);
        for (size_t k = 0; k < keep.size(); ++k)
          if (!fixed[keep[k]]) trial[keep[k]] = cmap[k][sr.choice[k]];
      }
      if (!ok) continue;
      // every feasible grouping is simulated (the additive split cost only ranks, it cannot see
      // the fork / join re-layouts overlapping the other branches)
      const double sim_g = full.simulate(trial).makespan_ms;
      if (best_choice.empty() || sim_g < best_sim) {
        best_sim = sim_g;
        best_split = worst;
        best_choice = trial;
        best_group = group;
        best_G = G;
      }
    }
    info.groups = best_G;
    info.split_ms = best_choice.empty() ? info.whole_ms : best_split;
    info.sim_before_ms = cur_sim;
    info.sim_after_ms = best_choice.empty() ? cur_sim : best_sim;
    if (!best_choice.empty()) {
      info.group_of = best_group;
      if (best_sim < cur_sim) {
        r.choice = best_choice;
        cur_sim = best_sim;
        info.accepted = true;
      }
    }
    r.splits.push_back(info);
  }
  r.cost_ms = r.sim_ms = cur_sim;
  return r;
}

}  // namespace ffcore
