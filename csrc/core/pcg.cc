// Layouts, MI355X machine model, transfer costing and the task-graph simulator.
#include "pcg.h"

#include <algorithm>
#include <mutex>
#include <string>
#include <unordered_map>
#include <cmath>
#include <numeric>
#include <set>

namespace ffcore {

std::vector<int> Layout::block_coords(int b) const {
  std::vector<int> c(degrees.size());
  for (int i = (int)degrees.size() - 1; i >= 0; --i) {
    c[i] = b % degrees[i];
    b /= degrees[i];
  }
  return c;
}

int Layout::part_index(const std::vector<int>& blk, int rep) const {
  int b = 0;
  for (size_t i = 0; i < degrees.size(); ++i) b = b * degrees[i] + blk[i];
  return b * replicas + rep;
}

std::vector<int> Layout::replica_group(const std::vector<int>& blk) const {
  std::vector<int> g;
  for (int r = 0; r < replicas; ++r) g.push_back(devices[part_index(blk, r)]);
  return g;
}

double MachineModel::ring_busbw(const std::vector<int>& ranks) const {
  const int r = (int)ranks.size();
  if (r <= 1) return 1e30;
  if (topo) return coll_eff * topo->ring_busbw(ranks);
  bool one_node = true;
  for (int x : ranks)
    if (!same_node(x, ranks[0])) one_node = false;
  // fully connected xGMI: a ring collective can drive (r-1) point-to-point links per GPU
  const double intra = coll_eff * std::min((double)(r - 1), links_per_gpu) * link_gbps;
  if (one_node) return intra;
  return std::min(intra, coll_eff * inter_node_gbps);
}

namespace {

int find_split_dim(const Layout& a, const Layout& b, int factor) {
  int cand = -1;
  for (size_t d = 0; d < a.degrees.size(); ++d) {
    if (a.degrees[d] == b.degrees[d]) continue;
    if (b.degrees[d] == a.degrees[d] * factor && cand < 0) cand = (int)d;
    else return -1;
  }
  return cand;
}

bool subblocks_match(const Layout& coarse, const Layout& fine, int d, int k, bool subset) {
  for (int b = 0; b < coarse.num_blocks(); ++b) {
    auto blk = coarse.block_coords(b);
    auto rg = coarse.replica_group(blk);
    std::set<int> rep(rg.begin(), rg.end());
    std::set<int> sub;
    for (int j = 0; j < k; ++j) {
      auto fb = blk;
      fb[d] = blk[d] * k + j;
      sub.insert(fine.devices[fine.part_index(fb, 0)]);
    }
    if ((int)sub.size() != k) return false;
    if (subset) {
      for (int x : sub)
        if (!rep.count(x)) return false;
    } else if (sub != rep) {
      return false;
    }
  }
  return true;
}

struct Region {
  std::vector<int64_t> lo, hi;
};

Region part_region(const Layout& L, int p, bool with_halo) {
  Region r;
  const int rep = p % L.replicas;
  (void)rep;
  auto blk = L.block_coords(p / L.replicas);
  for (size_t i = 0; i < L.shape.size(); ++i) {
    const int64_t bs = L.shape[i] / L.degrees[i];
    int64_t lo = blk[i] * bs, hi = lo + bs;
    if (with_halo && !L.halo.empty()) {
      lo = std::max<int64_t>(0, lo - L.halo[i]);
      hi = std::min<int64_t>(L.shape[i], hi + L.halo[i]);
    }
    r.lo.push_back(lo);
    r.hi.push_back(hi);
  }
  return r;
}

int64_t overlap(const Region& a, const Region& b) {
  int64_t n = 1;
  for (size_t i = 0; i < a.lo.size(); ++i) {
    const int64_t lo = std::max(a.lo[i], b.lo[i]), hi = std::min(a.hi[i], b.hi[i]);
    if (lo >= hi) return 0;
    n *= hi - lo;
  }
  return n;
}

}  // namespace

// D re-partitions S from dim a to dim b, k ways, on the same devices, no replicas (runtime:
// flexflow_amd.parallel.comm._a2a_dims, executed as one all_to_all per group).
static bool is_all_to_all(const Layout& S, const Layout& D) {
  if (S.replicas != 1 || D.replicas != 1 || !S.halo.empty() || !D.halo.empty() || S.degrees.size() != D.degrees.size())
    return false;
  int a = -1, b = -1, ndiff = 0;
  for (size_t d = 0; d < S.degrees.size(); ++d) {
    if (S.degrees[d] == D.degrees[d]) continue;
    ++ndiff;
    if (S.degrees[d] > 1 && D.degrees[d] == 1) a = (int)d;
    else if (D.degrees[d] > 1 && S.degrees[d] == 1) b = (int)d;
  }
  if (ndiff != 2 || a < 0 || b < 0 || S.degrees[a] != D.degrees[b]) return false;
  const int k = S.degrees[a];
  for (int blk = 0; blk < S.num_blocks(); ++blk) {
    auto c = S.block_coords(blk);
    if (c[a] != 0) continue;
    std::set<int> sd, dd;
    for (int i = 0; i < k; ++i) {
      auto o = c;
      o[a] = i;
      sd.insert(S.devices[S.part_index(o, 0)]);
      o = c;
      o[a] = 0;
      o[b] = i;
      dd.insert(D.devices[D.part_index(o, 0)]);
    }
    if ((int)sd.size() != k || sd != dd) return false;
  }
  return true;
}

static XferCost transfer_cost_uncached(const Layout& S, const Layout& D, bool sp, int eb, const MachineModel& mm) {
  XferCost x;
  const bool same_blocks = S.degrees == D.degrees;
  const double lat = mm.latency_us * 1e-3;
  if (!sp && same_blocks && S.replicas == D.replicas && S.devices == D.devices && S.halo == D.halo) {
    x.kind = XferKind::IDENTITY;
    return x;
  }
  std::set<int> devs(S.devices.begin(), S.devices.end());
  devs.insert(D.devices.begin(), D.devices.end());
  x.devices.assign(devs.begin(), devs.end());
  const bool halo = !S.halo.empty() || !D.halo.empty();
  if (!halo) {
    if (sp && same_blocks && S.replicas == D.replicas) {
      bool ok = true;
      for (int b = 0; b < S.num_blocks() && ok; ++b) {
        auto blk = S.block_coords(b);
        auto a = S.replica_group(blk), c = D.replica_group(blk);
        ok = std::set<int>(a.begin(), a.end()) == std::set<int>(c.begin(), c.end());
      }
      if (ok) {
        x.kind = XferKind::ALL_REDUCE;
        double worst = 0;
        for (int b = 0; b < S.num_blocks(); ++b) {
          auto g = S.replica_group(S.block_coords(b));
          const double bytes = (double)S.block_numel() * eb;
          const int r = (int)g.size();
          worst = std::max(worst, 2.0 * (r - 1) / r * bytes / (mm.ring_busbw(g) * 1e6));
          x.bytes += 2.0 * (r - 1) * bytes;
        }
        x.ms = worst + lat;
        return x;
      }
    }
    if (sp && D.replicas == 1 && S.replicas > 1) {
      const int d = find_split_dim(S, D, S.replicas);
      if (d >= 0 && subblocks_match(S, D, d, S.replicas, false)) {
        x.kind = XferKind::REDUCE_SCATTER;
        double worst = 0;
        for (int b = 0; b < S.num_blocks(); ++b) {
          auto g = S.replica_group(S.block_coords(b));
          const int r = (int)g.size();
          const double bytes = (double)S.block_numel() * eb;
          worst = std::max(worst, (double)(r - 1) / r * bytes / (mm.ring_busbw(g) * 1e6));
          x.bytes += (r - 1) * bytes;
        }
        x.ms = worst + lat;
        return x;
      }
    }
    if (!sp && S.replicas == 1 && D.replicas > 1) {
      const int d = find_split_dim(D, S, D.replicas);
      if (d >= 0 && subblocks_match(D, S, d, D.replicas, false)) {
        x.kind = XferKind::ALL_GATHER;
        double worst = 0;
        for (int b = 0; b < D.num_blocks(); ++b) {
          auto g = D.replica_group(D.block_coords(b));
          const int r = (int)g.size();
          const double bytes = (double)D.block_numel() * eb;
          worst = std::max(worst, (double)(r - 1) / r * bytes / (mm.ring_busbw(g) * 1e6));
          x.bytes += (r - 1) * bytes;
        }
        x.ms = worst + lat;
        return x;
      }
    }
    if (!sp && S.replicas > 1 && D.replicas == 1) {
      const int d = find_split_dim(S, D, S.replicas);
      if (d >= 0 && subblocks_match(S, D, d, S.replicas, true)) {
        x.kind = XferKind::LOCAL_SLICE;
        x.ms = (double)D.block_numel() * eb * 2 / (mm.hbm_gbps * 1e6);
        return x;
      }
    }
  }
  // generic point-to-point plan: same region-intersection rule as the runtime's plan_transfer;
  // an all-to-all is priced the same way (every pair over its own xGMI link at once)
  x.kind = (!sp && is_all_to_all(S, D)) ? XferKind::ALL_TO_ALL : XferKind::GENERIC;
  std::map<std::pair<int, int>, double> link;
  const bool halo_sum = !S.halo.empty() && sp;
  for (int q = 0; q < D.num_parts(); ++q) {
    Region rq = part_region(D, q, true);
    const int dq = D.devices[q];
    if (halo_sum) {
      for (int p = 0; p < S.num_parts(); ++p) {
        const int64_t n = overlap(part_region(S, p, true), rq);
        if (n && S.devices[p] != dq) link[{S.devices[p], dq}] += (double)n * eb;
      }
      continue;
    }
    for (int b = 0; b < S.num_blocks(); ++b) {
      auto blk = S.block_coords(b);
      const int64_t n = overlap(part_region(S, S.part_index(blk, 0), false), rq);
      if (!n) continue;
      if (sp) {
        for (int r = 0; r < S.replicas; ++r) {
          const int sd = S.devices[S.part_index(blk, r)];
          if (sd != dq) link[{sd, dq}] += (double)n * eb;
        }
      } else {
        int src = -1;
        for (int r = 0; r < S.replicas; ++r)
          if (S.devices[S.part_index(blk, r)] == dq) src = dq;
        if (src < 0) src = S.devices[S.part_index(blk, q % S.replicas)];
        if (src != dq) link[{src, dq}] += (double)n * eb;
      }
    }
  }
  if (mm.topo) {  // routed, per-link contention
    std::vector<std::tuple<int, int, double>> xs;
    for (auto& kv : link) {
      xs.emplace_back(kv.first.first, kv.first.second, kv.second);
      x.bytes += kv.second;
    }
    x.ms = link.empty() ? 0.0 : mm.topo->transfers_ms(xs) / mm.coll_eff + lat;
    return x;
  }
  std::map<int, double> egress, ingress;
  double worst_link = 0;
  for (auto& kv : link) {
    const double t = kv.second / (mm.p2p_gbps(kv.first.first, kv.first.second) * 1e6);
    worst_link = std::max(worst_link, t);
    egress[kv.first.first] += kv.second;
    ingress[kv.first.second] += kv.second;
    x.bytes += kv.second;
  }
  double worst_dev = 0;
  for (auto& kv : egress) worst_dev = std::max(worst_dev, kv.second / (mm.links_per_gpu * mm.link_gbps * 1e6));
  for (auto& kv : ingress) worst_dev = std::max(worst_dev, kv.second / (mm.links_per_gpu * mm.link_gbps * 1e6));
  x.ms = link.empty() ? 0.0 : std::max(worst_link, worst_dev) + lat;
  return x;
}

// The joint search costs every rewritten graph with a fresh Problem, and the frontier DP prices
// (producer config x consumer config) edges lazily: without a shared memo the same layout pairs
// were priced again per graph (~1 s of a 3 s Inception-v3 N=8 search). Transfer costs depend only
// on the two layouts, the partial flag, the element size and the machine; the memo is keyed by all
// of them (the topology by identity) and cleared when it grows past 1 M entries.
namespace {
void key_put(std::string& k, int64_t v) { k.append(reinterpret_cast<const char*>(&v), sizeof(v)); }
void key_put(std::string& k, const Layout& L) {
  key_put(k, (int64_t)L.shape.size());
  for (auto v : L.shape) key_put(k, v);
  for (auto v : L.degrees) key_put(k, v);
  key_put(k, L.replicas);
  key_put(k, (int64_t)L.devices.size());
  for (auto v : L.devices) key_put(k, v);
  key_put(k, (int64_t)L.halo.size());
  for (auto v : L.halo) key_put(k, v);
}
std::mutex g_xfer_memo_mu;
std::unordered_map<std::string, XferCost> g_xfer_memo;
}  // namespace

XferCost transfer_cost(const Layout& S, const Layout& D, bool sp, int eb, const MachineModel& mm) {
  std::string k;
  k.reserve(256);
  key_put(k, S);
  key_put(k, D);
  key_put(k, (int64_t)sp * 2 + (int64_t)S.partial);
  key_put(k, eb);
  const double mf[] = {mm.link_gbps, mm.links_per_gpu, mm.coll_eff, mm.inter_node_gbps, mm.latency_us, mm.hbm_gbps};
  k.append(reinterpret_cast<const char*>(mf), sizeof(mf));
  key_put(k, (int64_t)mm.num_nodes * 4096 + mm.gpus_per_node);
  key_put(k, (int64_t)(intptr_t)mm.topo.get());
  {
    std::lock_guard<std::mutex> g(g_xfer_memo_mu);
    auto it = g_xfer_memo.find(k);
    if (it != g_xfer_memo.end()) return it->second;
  }
  XferCost x = transfer_cost_uncached(S, D, sp, eb, mm);
  std::lock_guard<std::mutex> g(g_xfer_memo_mu);
  if (g_xfer_memo.size() > (1u << 20)) g_xfer_memo.clear();
  g_xfer_memo.emplace(std::move(k), x);
  return x;
}

static uint64_t mix(uint64_t h, uint64_t v) {
  h ^= v + 0x9e3779b97f4a7c15ull + (h << 6) + (h >> 2);
  return h;
}

double Simulator::edge_cost(int node, int slot, int cfg, int prod_cfg) const {
  const Node& n = prob_.nodes[node];
  const auto in = n.inputs[slot];
  if (in.first < 0) return 0.0;
  uint64_t key = mix(mix(mix(mix(1469598103934665603ull, node), slot), cfg), prod_cfg);
  auto it = edge_cache_.find(key);
  if (it != edge_cache_.end()) return it->second;
  const Node& pn = prob_.nodes[in.first];
  const Layout& src = pn.cands[prod_cfg].out_layouts[in.second];
  const Layout& dst = n.cands[cfg].in_layouts[slot];
  double ms = transfer_cost(src, dst, src.partial, n.elem_bytes, prob_.machine).ms;
  const bool needs_grad = slot < (int)n.input_needs_grad.size() ? n.input_needs_grad[slot] : true;
  if (needs_grad && n.backward) {
    Layout s2 = dst, d2 = src;
    s2.partial = false;
    d2.partial = false;
    ms += transfer_cost(s2, d2, dst.replicas > 1 || !dst.halo.empty(), n.elem_bytes, prob_.machine).ms;
  }
  edge_cache_[key] = ms;
  return ms;
}

const XferCost& Simulator::edge_xfer(int node, int slot, int cfg, int prod_cfg, bool backward) const {
  uint64_t key = mix(mix(mix(mix(mix(7ull, node), slot), cfg), prod_cfg), backward ? 1 : 0);
  auto it = xfer_cache_.find(key);
  if (it != xfer_cache_.end()) return it->second;
  const Node& n = prob_.nodes[node];
  const auto in = n.inputs[slot];
  const Node& pn = prob_.nodes[in.first];
  XferCost x;
  if (!backward) {
    const Layout& src = pn.cands[prod_cfg].out_layouts[in.second];
    x = transfer_cost(src, n.cands[cfg].in_layouts[slot], src.partial, n.elem_bytes, prob_.machine);
  } else {
    Layout dst = pn.cands[prod_cfg].out_layouts[in.second];
    Layout src = n.cands[cfg].in_layouts[slot];
    const bool sp = src.replicas > 1 || !src.halo.empty();
    src.partial = false;
    dst.partial = false;
    x = transfer_cost(src, dst, sp, n.elem_bytes, prob_.machine);
  }
  return xfer_cache_.emplace(key, std::move(x)).first->second;
}

double Simulator::weight_sync_ms(int node, int cfg) const {
  const OpCandidate& c = prob_.nodes[node].cands[cfg];
  double ms = 0;
  for (const Layout& w : c.w_layouts) {
    if (w.replicas <= 1) continue;
    double worst = 0;
    for (int b = 0; b < w.num_blocks(); ++b) {
      auto g = w.replica_group(w.block_coords(b));
      const int r = (int)g.size();
      const double bytes = (double)w.block_numel() * 4;  // fp32 gradients
      worst = std::max(worst, 2.0 * (r - 1) / r * bytes / (prob_.machine.ring_busbw(g) * 1e6));
    }
    ms += worst;
  }
  return ms;
}

double Simulator::node_cost(int node, int cfg, const std::vector<int>& prod) const {
  const Node& n = prob_.nodes[node];
  const OpCandidate& c = n.cands[cfg];
  double ms = c.fwd_ms + (n.backward ? c.bwd_ms : 0.0);
  // bucketed gradient all-reduce overlaps the rest of the backward pass: charge half
  if (n.backward) ms += weight_sync_ms(node, cfg) * (prob_.overlap_grad_sync ? 0.5 : 1.0);
  for (size_t s = 0; s < n.inputs.size(); ++s)
    if (n.inputs[s].first >= 0) ms += edge_cost(node, (int)s, cfg, prod[s]);
  if (c.mem_bytes > prob_.machine.mem_capacity) ms += 1e6;
  return ms;
}

// Greedy in-order list scheduling over per-device compute and comm resources (the reference's
// Simulator::simulate_runtime builds the same fwd/bwd/xfer/update task graph with a ready queue).
SimResult Simulator::simulate(const std::vector<int>& choice) const {
  const int N = (int)prob_.nodes.size();
  const int D = prob_.machine.num_devices();
  std::vector<double> comp_free(D, 0), comm_free(D, 0), comp_busy(D, 0), comm_busy(D, 0), mem(D, 0);
  std::vector<double> fwd_end(N, 0), bwd_end(N, 0);
  std::vector<std::vector<double>> grad_ready(N);  // per node: when all output grads arrived
  std::vector<double> out_grad_time(N, 0);

  auto run = [&](const std::vector<int>& devs, bool comm, double ready, double dur) {
    double st = ready;
    for (int d : devs) st = std::max(st, comm ? comm_free[d] : comp_free[d]);
    const double en = st + dur;
    for (int d : devs) {
      if (comm) { comm_free[d] = en; comm_busy[d] += dur; }
      else { comp_free[d] = en; comp_busy[d] += dur; }
    }
    return en;
  };

  // forward
  for (int i = 0; i < N; ++i) {
    const Node& n = prob_.nodes[i];
    const OpCandidate& c = n.cands[choice[i]];
    double ready = 0;
    for (size_t s = 0; s < n.inputs.size(); ++s) {
      const int p = n.inputs[s].first;
      if (p < 0) continue;
      const XferCost& x = edge_xfer(i, (int)s, choice[i], choice[p], false);
      double t = fwd_end[p];
      if (x.kind != XferKind::IDENTITY && x.ms > 0) t = run(x.devices, true, t, x.ms);
      ready = std::max(ready, t);
    }
    fwd_end[i] = run(c.devices, false, ready, c.fwd_ms);
    for (int d : c.devices) mem[d] += c.mem_bytes;
  }
  // backward (reverse topological order); output-grad arrival times accumulate in out_grad_time
  std::vector<double> last_user_bwd(N, 0);
  double last_fwd = 0;
  for (int i = 0; i < N; ++i) last_fwd = std::max(last_fwd, fwd_end[i]);
  std::fill(out_grad_time.begin(), out_grad_time.end(), 0.0);
  std::vector<double> sync_end(D, 0);
  for (int i = N - 1; i >= 0; --i) {
    const Node& n = prob_.nodes[i];
    if (!n.backward) continue;
    const OpCandidate& c = n.cands[choice[i]];
    const double ready = std::max(out_grad_time[i], i == N - 1 ? last_fwd : fwd_end[i]);
    bwd_end[i] = run(c.devices, false, ready, c.bwd_ms);
    // weight gradient all-reduce (overlaps later backward work on the comm resources)
    for (const Layout& w : c.w_layouts) {
      if (w.replicas <= 1) continue;
      for (int b = 0; b < w.num_blocks(); ++b) {
        auto g = w.replica_group(w.block_coords(b));
        const int r = (int)g.size();
        const double bytes = (double)w.block_numel() * 4;
        const double dur = 2.0 * (r - 1) / r * bytes / (prob_.machine.ring_busbw(g) * 1e6) +
                           prob_.machine.latency_us * 1e-3;
        const double e = run(g, true, bwd_end[i], dur);
        for (int d : g) sync_end[d] = std::max(sync_end[d], e);
      }
    }
    for (size_t s = 0; s < n.inputs.size(); ++s) {
      const int p = n.inputs[s].first;
      if (p < 0) continue;
      const bool ng = s < n.input_needs_grad.size() ? n.input_needs_grad[s] : true;
      if (!ng) continue;
      const XferCost& x = edge_xfer(i, (int)s, choice[i], choice[p], true);
      double t = bwd_end[i];
      if (x.kind != XferKind::IDENTITY && x.ms > 0) t = run(x.devices, true, t, x.ms);
      out_grad_time[p] = std::max(out_grad_time[p], t);
    }
  }
  SimResult r;
  double end = 0;
  for (int d = 0; d < D; ++d) {
    double e = std::max({comp_free[d], comm_free[d], sync_end[d]});
    end = std::max(end, e);
    r.compute_ms = std::max(r.compute_ms, comp_busy[d]);
    r.comm_ms = std::max(r.comm_ms, comm_busy[d]);
    r.max_mem = std::max(r.max_mem, mem[d]);
  }
  // optimizer update: one fused kernel per arena, proportional to local parameter bytes
  std::vector<double> wmb(D, 0);
  for (int i = 0; i < N; ++i) {
    const OpCandidate& c = prob_.nodes[i].cands[choice[i]];
    for (const Layout& w : c.w_layouts)
      for (int p = 0; p < w.num_parts(); ++p) wmb[w.devices[p]] += (double)w.block_numel() * 4 / 1e6;
  }
  double upd = 0;
  for (int d = 0; d < D; ++d) upd = std::max(upd, wmb[d] * prob_.update_ms_per_mb);
  r.makespan_ms = end + upd;
  r.oom = r.max_mem > prob_.machine.mem_capacity;
  if (r.oom) r.makespan_ms += 1e6;
  return r;
}

}  // namespace ffcore
