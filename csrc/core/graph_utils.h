// Native graph / machine utilities of the PCG compiler (header-only).
//
// Reference counterparts (behaviour, not code):
//   include/flexflow/dominators.h          -> Digraph + topo_order / dominators / post_dominators /
//                                             imm_dominators / transitive_reduction / components
//   include/flexflow/basic_graph.h         -> Digraph (dense int node ids, sorted adjacency)
//   include/flexflow/utils/disjoint_set.h  -> DisjointSet (path halving + union by size)
//   include/flexflow/utils/random_utils.h  -> select_random (weighted pick)
//   include/flexflow/utils/hash_utils.h    -> hash_combine
//   include/flexflow/machine_view.h        -> MachineView / MachineResource (machine_view.cc)
//
// Design: graphs are small (a PCG has 10^2..10^4 nodes) and built once per search, so nodes are
// dense ints with sorted adjacency vectors, dominator sets are bitsets over a topological order
// (one pass in topo order: dom(v) = {v} U AND_{p in pred(v)} dom(p)) and the immediate dominator
// is the dominator with the highest topological rank. bottlenecks() adds a virtual source and
// sink so multi-root / multi-leaf graphs split the same way.
#pragma once
#include <algorithm>
#include <cstdint>
#include <functional>
#include <numeric>
#include <queue>
#include <random>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace ffcore {

inline void hash_combine(uint64_t& seed, uint64_t v) {
  // 64-bit golden-ratio mix (boost-style), used to key search caches by (node, view) tuples
  seed ^= v + 0x9e3779b97f4a7c15ULL + (seed << 12) + (seed >> 4);
}

class DisjointSet {
 public:
  explicit DisjointSet(int n = 0) { resize(n); }
  void resize(int n) {
    parent_.resize(n);
    size_.assign(n, 1);
    std::iota(parent_.begin(), parent_.end(), 0);
  }
  int find(int x) {
    while (parent_[x] != x) {
      parent_[x] = parent_[parent_[x]];
      x = parent_[x];
    }
    return x;
  }
  bool unite(int a, int b) {
    a = find(a);
    b = find(b);
    if (a == b) return false;
    if (size_[a] < size_[b]) std::swap(a, b);
    parent_[b] = a;
    size_[a] += size_[b];
    return true;
  }
  bool same(int a, int b) { return find(a) == find(b); }
  int size() const { return (int)parent_.size(); }

 private:
  std::vector<int> parent_, size_;
};

// Weighted random pick: index i with probability w[i] / sum(w) (u in [0, 1) supplied by the caller
// so the search stays reproducible under its own seeded RNG).
inline int select_random(const std::vector<double>& w, double u) {
  double tot = 0;
  for (double x : w) tot += std::max(0.0, x);
  if (w.empty() || tot <= 0) throw std::invalid_argument("select_random: no positive weight");
  double acc = 0, t = u * tot;
  for (size_t i = 0; i < w.size(); ++i) {
    acc += std::max(0.0, w[i]);
    if (t < acc) return (int)i;
  }
  return (int)w.size() - 1;
}

class Digraph {
 public:
  explicit Digraph(int n = 0) : succ_(n), pred_(n) {}
  int num_nodes() const { return (int)succ_.size(); }
  int add_node() {
    succ_.emplace_back();
    pred_.emplace_back();
    return num_nodes() - 1;
  }
  void add_edge(int a, int b) {
    check(a);
    check(b);
    auto it = std::lower_bound(succ_[a].begin(), succ_[a].end(), b);
    if (it != succ_[a].end() && *it == b) return;
    succ_[a].insert(it, b);
    pred_[b].insert(std::lower_bound(pred_[b].begin(), pred_[b].end(), a), a);
  }
  void remove_edge(int a, int b) {
    auto it = std::lower_bound(succ_[a].begin(), succ_[a].end(), b);
    if (it == succ_[a].end() || *it != b) return;
    succ_[a].erase(it);
    pred_[b].erase(std::lower_bound(pred_[b].begin(), pred_[b].end(), a));
  }
  bool has_edge(int a, int b) const { return std::binary_search(succ_[a].begin(), succ_[a].end(), b); }
  const std::vector<int>& successors(int v) const { return succ_[v]; }
  const std::vector<int>& predecessors(int v) const { return pred_[v]; }
  std::vector<std::pair<int, int>> edges() const {
    std::vector<std::pair<int, int>> e;
    for (int a = 0; a < num_nodes(); ++a)
      for (int b : succ_[a]) e.emplace_back(a, b);
    return e;
  }
  std::vector<int> roots() const {
    std::vector<int> r;
    for (int v = 0; v < num_nodes(); ++v)
      if (pred_[v].empty()) r.push_back(v);
    return r;
  }
  std::vector<int> leaves() const {
    std::vector<int> r;
    for (int v = 0; v < num_nodes(); ++v)
      if (succ_[v].empty()) r.push_back(v);
    return r;
  }
  Digraph reversed() const {
    Digraph g(num_nodes());
    g.succ_ = pred_;
    g.pred_ = succ_;
    return g;
  }

  // Kahn's algorithm, FIFO over ready nodes in id order; throws on a cycle.
  std::vector<int> topo_order() const {
    std::vector<int> indeg(num_nodes()), order;
    std::queue<int> q;
    for (int v = 0; v < num_nodes(); ++v)
      if ((indeg[v] = (int)pred_[v].size()) == 0) q.push(v);
    while (!q.empty()) {
      int v = q.front();
      q.pop();
      order.push_back(v);
      for (int s : succ_[v])
        if (--indeg[s] == 0) q.push(s);
    }
    if ((int)order.size() != num_nodes()) throw std::runtime_error("topo_order: graph has a cycle");
    return order;
  }

  // dom[v] = sorted list of nodes that lie on every path from a root to v (v included). With
  // several roots a virtual root dominates everything; it is not listed (as in the reference,
  // a node reached from two roots is dominated only by itself and its true bottlenecks).
  std::vector<std::vector<int>> dominators() const {
    const int n = num_nodes();
    const auto order = topo_order();
    std::vector<int> rank(n);
    for (int i = 0; i < n; ++i) rank[order[i]] = i;
    const int W = (n + 63) / 64;
    std::vector<std::vector<uint64_t>> dom(n, std::vector<uint64_t>(W, 0));
    for (int v : order) {
      auto& d = dom[v];
      bool first = true;
      for (int p : pred_[v]) {
        if (first) {
          d = dom[p];
          first = false;
        } else {
          for (int k = 0; k < W; ++k) d[k] &= dom[p][k];
        }
      }
      d[rank[v] / 64] |= 1ULL << (rank[v] % 64);
    }
    std::vector<std::vector<int>> out(n);
    for (int v = 0; v < n; ++v) {
      for (int i = 0; i < n; ++i)
        if (dom[v][i / 64] >> (i % 64) & 1) out[v].push_back(order[i]);
      std::sort(out[v].begin(), out[v].end());
    }
    return out;
  }
  std::vector<std::vector<int>> post_dominators() const { return reversed().dominators(); }

  // idom[v] = the strict dominator of v latest in topological order; v itself when v has no strict
  // dominator (a root, or a node whose paths from different roots share no node but itself).
  std::vector<int> imm_dominators() const {
    const auto order = topo_order();
    std::vector<int> rank(num_nodes());
    for (int i = 0; i < num_nodes(); ++i) rank[order[i]] = i;
    const auto dom = dominators();
    std::vector<int> idom(num_nodes());
    for (int v = 0; v < num_nodes(); ++v) {
      int best = -1;
      for (int d : dom[v])
        if (d != v && (best < 0 || rank[d] > rank[best])) best = d;
      idom[v] = best >= 0 ? best : v;
    }
    return idom;
  }
  std::vector<int> imm_post_dominators() const { return reversed().imm_dominators(); }

  // Nodes through which every root->leaf path passes (the sequence-split points of Unity's DP:
  // the PCG can be cut there into a pre- and a post-graph joined by one tensor).
  std::vector<int> bottlenecks() const {
    const int n = num_nodes();
    if (n == 0) return {};
    // virtual source/sink so that multi-root / multi-leaf graphs are handled uniformly
    Digraph g = *this;
    const int src = g.add_node(), snk = g.add_node();
    for (int r : roots()) g.add_edge(src, r);
    for (int l : leaves()) g.add_edge(l, snk);
    const auto dom = g.dominators();
    std::vector<int> out;
    for (int d : dom[snk])
      if (d != src && d != snk) out.push_back(d);
    const auto order = topo_order();
    std::vector<int> rank(n);
    for (int i = 0; i < n; ++i) rank[order[i]] = i;
    std::sort(out.begin(), out.end(), [&](int a, int b) { return rank[a] < rank[b]; });
    return out;
  }

  std::vector<int> descendants(int v, bool undirected = false) const {
    std::vector<char> seen(num_nodes(), 0);
    std::vector<int> out, st = {v};
    seen[v] = 1;
    while (!st.empty()) {
      int x = st.back();
      st.pop_back();
      out.push_back(x);
      auto visit = [&](int y) {
        if (!seen[y]) {
          seen[y] = 1;
          st.push_back(y);
        }
      };
      for (int s : succ_[x]) visit(s);
      if (undirected)
        for (int p : pred_[x]) visit(p);
    }
    std::sort(out.begin(), out.end());
    return out;
  }

  std::vector<std::vector<int>> weakly_connected_components() const {
    DisjointSet ds(num_nodes());
    for (auto& e : edges()) ds.unite(e.first, e.second);
    std::vector<std::vector<int>> comps;
    std::vector<int> idx(num_nodes(), -1);
    for (int v = 0; v < num_nodes(); ++v) {
      int r = ds.find(v);
      if (idx[r] < 0) {
        idx[r] = (int)comps.size();
        comps.emplace_back();
      }
      comps[idx[r]].push_back(v);
    }
    return comps;
  }

  // Drop every edge a->b for which another path a->...->b exists (DAGs only).
  Digraph transitive_reduction() const {
    const auto order = topo_order();
    const int n = num_nodes();
    std::vector<int> rank(n);
    for (int i = 0; i < n; ++i) rank[order[i]] = i;
    const int W = (n + 63) / 64;
    // reach[v]: nodes reachable from v by a path of length >= 1 (bitset by node id)
    std::vector<std::vector<uint64_t>> reach(n, std::vector<uint64_t>(W, 0));
    for (int i = n - 1; i >= 0; --i) {
      int v = order[i];
      for (int s : succ_[v]) {
        reach[v][s / 64] |= 1ULL << (s % 64);
        for (int k = 0; k < W; ++k) reach[v][k] |= reach[s][k];
      }
    }
    Digraph r(n);
    for (int a = 0; a < n; ++a)
      for (int b : succ_[a]) {
        bool indirect = false;
        for (int c : succ_[a])
          if (c != b && (reach[c][b / 64] >> (b % 64) & 1)) {
            indirect = true;
            break;
          }
        if (!indirect) r.add_edge(a, b);
      }
    return r;
  }

 private:
  void check(int v) const {
    if (v < 0 || v >= num_nodes()) throw std::out_of_range("Digraph: node id out of range");
  }
  std::vector<std::vector<int>> succ_, pred_;
};

// ------------------------------------------------------------------------------ machine views
// A device grid: part p with grid coordinates (c_0..c_{ndims-1}) runs on device
// start_device_id + sum_i c_i * stride[i]. 1-D views with stride 1 are contiguous GPU blocks;
// 2-D views (nodes x GPUs, stride {gpus_per_node, 1}) and strided 1-D views (one GPU per node)
// express the multi-node placements the reference left commented out (graph.cc:2346-2359).
struct MachineView {
  enum DeviceType { GPU = 0, CPU = 1 };
  int device_type = GPU;
  int start_device_id = 0;
  std::vector<int> dim, stride;

  int ndims() const { return (int)dim.size(); }
  int num_parts() const {
    int n = 1;
    for (int d : dim) n *= d;
    return n;
  }
  int device_id(const std::vector<int>& coord) const {
    if ((int)coord.size() != ndims()) throw std::invalid_argument("MachineView: coordinate rank mismatch");
    int id = start_device_id;
    for (int i = 0; i < ndims(); ++i) {
      if (coord[i] < 0 || coord[i] >= dim[i]) throw std::out_of_range("MachineView: coordinate out of range");
      id += coord[i] * stride[i];
    }
    return id;
  }
  // devices of parts in row-major part order (last grid dim fastest)
  std::vector<int> device_ids() const {
    std::vector<int> ids;
    const int n = num_parts();
    std::vector<int> c(ndims(), 0);
    for (int p = 0; p < n; ++p) {
      ids.push_back(device_id(c));
      for (int i = ndims() - 1; i >= 0; --i) {
        if (++c[i] < dim[i]) break;
        c[i] = 0;
      }
    }
    return ids;
  }
  uint64_t hash() const {
    uint64_t h = 0;
    hash_combine(h, (uint64_t)device_type);
    hash_combine(h, (uint64_t)start_device_id);
    hash_combine(h, (uint64_t)ndims());
    for (int i = 0; i < ndims(); ++i) {
      hash_combine(h, (uint64_t)dim[i]);
      hash_combine(h, (uint64_t)stride[i]);
    }
    return h;
  }
  bool operator==(const MachineView& o) const {
    return device_type == o.device_type && start_device_id == o.start_device_id && dim == o.dim &&
           stride == o.stride;
  }
  std::string str() const {
    std::string s = "MachineView(start=" + std::to_string(start_device_id) + ", dims=[";
    for (int i = 0; i < ndims(); ++i) s += (i ? "," : "") + std::to_string(dim[i]);
    s += "], strides=[";
    for (int i = 0; i < ndims(); ++i) s += (i ? "," : "") + std::to_string(stride[i]);
    return s + "])";
  }
};

struct MachineResource {
  int num_nodes = 1;
  int all_gpus_per_node = 8;
  int available_gpus_per_node = 8;
  int start_gpu_id = 0;

  // every device of the view exists and lies inside the available slice of each node
  bool is_valid_machine_view(const MachineView& v) const {
    if (v.device_type != MachineView::GPU || v.num_parts() < 1) return false;
    for (int i = 0; i < v.ndims(); ++i)
      if (v.dim[i] < 1 || v.stride[i] < 1) return false;
    for (int id : v.device_ids()) {
      if (id < 0) return false;
      const int node = id / all_gpus_per_node, local = id % all_gpus_per_node;
      if (node >= num_nodes) return false;
      const int lo = start_gpu_id % all_gpus_per_node;
      if (local < lo || local >= lo + available_gpus_per_node) return false;
    }
    return true;
  }

  // All views with num_parts | total devices: contiguous 1-D blocks at aligned starts
  // (the reference's `i | N` views), strided 1-D views across nodes (one GPU per node), and
  // 2-D node x GPU grids. Deduplicated by device list + shape.
  std::vector<MachineView> enumerate_views(int max_parts = 0) const {
    std::vector<MachineView> out;
    const int G = available_gpus_per_node, N = num_nodes, total = G * N;
    const int base = start_gpu_id;
    auto push = [&](MachineView v) {
      if ((max_parts > 0 && v.num_parts() > max_parts) || !is_valid_machine_view(v)) return;
      for (auto& o : out)
        if (o == v) return;
      out.push_back(std::move(v));
    };
    for (int p = 1; p <= total; ++p) {
      if (total % p) continue;
      if (p <= G) {  // inside one node
        for (int node = 0; node < N; ++node)
          for (int st = 0; st + p <= G; st += p) {
            MachineView v;
            v.start_device_id = base + node * all_gpus_per_node + st;
            v.dim = {p};
            v.stride = {1};
            push(v);
          }
      }
      if (p % G == 0 && p / G <= N) {  // whole nodes, 1-D contiguous (node-major)
        for (int node = 0; node + p / G <= N; node += p / G) {
          MachineView v;
          v.start_device_id = base + node * all_gpus_per_node;
          v.dim = {p / G, G};
          v.stride = {all_gpus_per_node, 1};
          push(v);
        }
      }
      if (N > 1 && p <= N && N % p == 0) {  // one GPU on each of p nodes
        for (int g = 0; g < G; ++g) {
          MachineView v;
          v.start_device_id = base + g;
          v.dim = {p};
          v.stride = {all_gpus_per_node};
          push(v);
        }
      }
    }
    return out;
  }
};

}  // namespace ffcore
