// Topology-aware network model: see network.h.
#include "network.h"

#include <algorithm>
#include <deque>
#include <limits>
#include <map>
#include <stdexcept>

namespace ffcore {

void NetworkTopology::add_link(int a, int b, double gbps) {
  if (a < 0 || b < 0 || a >= num_nodes || b >= num_nodes || a == b || gbps <= 0)
    throw std::invalid_argument("add_link: bad endpoints or bandwidth");
  links.push_back({a, b, gbps});
}

void NetworkTopology::build_routes() {
  const int n = num_nodes;
  // adjacency: (neighbor, directed link id); directed id 2i = a->b, 2i+1 = b->a
  std::vector<std::vector<std::pair<int, int>>> adj(n);
  for (size_t i = 0; i < links.size(); ++i) {
    adj[links[i].a].push_back({links[i].b, (int)(2 * i)});
    adj[links[i].b].push_back({links[i].a, (int)(2 * i + 1)});
  }
  nxt_.assign(n, std::vector<int>(n, -1));
  via_.assign(n, std::vector<int>(n, -1));
  dist_.assign(n, std::vector<int>(n, std::numeric_limits<int>::max()));
  // BFS from every destination over reversed edges gives, per source, the first hop of a
  // shortest path; among equal-hop paths keep the widest bottleneck
  for (int dst = 0; dst < n; ++dst) {
    std::vector<double> width(n, 0.0);
    dist_[dst][dst] = 0;
    width[dst] = std::numeric_limits<double>::infinity();
    std::deque<int> q{dst};
    std::vector<std::vector<int>> layers;
    while (!q.empty()) {
      const int v = q.front();
      q.pop_front();
      for (auto [u, lid] : adj[v]) {
        // u -> v uses the reverse direction of the stored id
        const int fwd = lid ^ 1;
        const double w = std::min(width[v], links[lid / 2].gbps);
        if (dist_[u][dst] == std::numeric_limits<int>::max()) {
          dist_[u][dst] = dist_[v][dst] + 1;
          width[u] = w;
          nxt_[u][dst] = v;
          via_[u][dst] = fwd;
          q.push_back(u);
        } else if (dist_[u][dst] == dist_[v][dst] + 1 && w > width[u]) {
          width[u] = w;
          nxt_[u][dst] = v;
          via_[u][dst] = fwd;
        }
      }
    }
  }
}

std::vector<int> NetworkTopology::route(int a, int b) const {
  std::vector<int> r;
  if (a == b) return r;
  if (nxt_.empty()) throw std::runtime_error("route: build_routes() not called");
  int v = a;
  while (v != b) {
    if (nxt_[v][b] < 0) throw std::runtime_error("route: unreachable");
    r.push_back(via_[v][b]);
    v = nxt_[v][b];
  }
  return r;
}

int NetworkTopology::hops(int a, int b) const { return (int)route(a, b).size(); }

double NetworkTopology::path_gbps(int a, int b) const {
  double w = std::numeric_limits<double>::infinity();
  for (int l : route(a, b)) w = std::min(w, links[l / 2].gbps);
  return w;
}

double NetworkTopology::transfers_ms(const std::vector<std::tuple<int, int, double>>& xfers) const {
  std::map<int, double> load;
  for (auto& [s, d, bytes] : xfers)
    for (int l : route(s, d)) load[l] += bytes;
  double worst = 0;
  for (auto& kv : load) worst = std::max(worst, kv.second / (links[kv.first / 2].gbps * 1e6));
  return worst;
}

// `steps` ring steps; each step, on each of the r-1 rotated rings k = 1..r-1, rank i sends
// chunk_bytes / (r-1) to rank (i + k) % r — all concurrently
double NetworkTopology::ring_steps_ms(const std::vector<int>& ranks, double chunk_bytes, int steps) const {
  const int r = (int)ranks.size();
  if (r <= 1 || steps <= 0) return 0.0;
  std::vector<std::tuple<int, int, double>> x;
  for (int k = 1; k < r; ++k)
    for (int i = 0; i < r; ++i) x.emplace_back(ranks[i], ranks[(i + k) % r], chunk_bytes / (r - 1));
  return steps * transfers_ms(x);
}

double NetworkTopology::allreduce_ms(const std::vector<int>& ranks, double bytes) const {
  const int r = (int)ranks.size();
  if (r <= 1) return 0.0;
  return ring_steps_ms(ranks, bytes / r, 2 * (r - 1));
}

double NetworkTopology::allgather_ms(const std::vector<int>& ranks, double bytes) const {
  const int r = (int)ranks.size();
  if (r <= 1) return 0.0;
  return ring_steps_ms(ranks, bytes / r, r - 1);
}

double NetworkTopology::ring_busbw(const std::vector<int>& ranks) const {
  const int r = (int)ranks.size();
  if (r <= 1) return 1e30;
  const double bytes = 1e9;
  const double ms = allreduce_ms(ranks, bytes);
  return 2.0 * (r - 1) / r * bytes / (ms * 1e6);
}

NetworkTopology make_mi355x_cluster(int nodes, int gpus_per_node, double xgmi_gbps, double nic_gbps,
                                    const std::string& kind, double oversub) {
  if (nodes < 1 || gpus_per_node < 1) throw std::invalid_argument("make_mi355x_cluster: empty machine");
  NetworkTopology t;
  t.num_gpus = nodes * gpus_per_node;
  t.num_nodes = t.num_gpus;
  for (int nd = 0; nd < nodes; ++nd)
    for (int i = 0; i < gpus_per_node; ++i)
      for (int j = i + 1; j < gpus_per_node; ++j)
        t.add_link(nd * gpus_per_node + i, nd * gpus_per_node + j, xgmi_gbps);
  if (nodes > 1) {
    if (kind == "big_switch") {
      const int sw = t.add_node();
      for (int g = 0; g < t.num_gpus; ++g) t.add_link(g, sw, nic_gbps);
    } else if (kind == "fat_tree") {
      const int spine = t.add_node();
      for (int nd = 0; nd < nodes; ++nd) {
        const int leaf = t.add_node();
        for (int i = 0; i < gpus_per_node; ++i) t.add_link(nd * gpus_per_node + i, leaf, nic_gbps);
        t.add_link(leaf, spine, gpus_per_node * nic_gbps / std::max(1.0, oversub));
      }
    } else {
      throw std::invalid_argument("make_mi355x_cluster: kind must be big_switch or fat_tree");
    }
  }
  t.build_routes();
  return t;
}

}  // namespace ffcore
