// Native runtime core: parallel computation graph (PCG) search problem, MI355X machine model,
// task-graph simulator, Unity-style DP search, MCMC search and graph substitutions.
//
// Reference counterparts (re-designed, not ported):
//   include/flexflow/parallel_tensor.h / machine_view.h   -> Layout / OpCandidate
//   src/runtime/machine_model.cc, network.cc              -> MachineModel (xGMI point-to-point)
//   src/runtime/simulator.cc (simulate_runtime)           -> Simulator::simulate
//   src/runtime/graph.cc, substitution.cc (Unity DP)      -> search_dp / search_unity
//   src/runtime/model.cc:3286-3357 (mcmc_optimize, dead)  -> search_mcmc (revived)
//   src/runtime/substitution_loader.cc                    -> load_rules / match_rule
#pragma once
#include <cstdint>
#include <functional>
#include <map>
#include <memory>
#include <random>
#include <string>
#include <tuple>
#include <unordered_map>
#include <vector>

#include "network.h"

namespace ffcore {

// A sharded tensor layout (mirror of flexflow_amd.parallel.layout.Layout).
struct Layout {
  std::vector<int64_t> shape;
  std::vector<int> degrees;
  int replicas = 1;
  std::vector<int> devices;  // part -> device, part = row-major(block coords..., replica)
  bool partial = false;
  std::vector<int64_t> halo;  // empty = none

  int num_blocks() const {
    int n = 1;
    for (int d : degrees) n *= d;
    return n;
  }
  int num_parts() const { return num_blocks() * replicas; }
  int64_t numel() const {
    int64_t n = 1;
    for (auto s : shape) n *= s;
    return n;
  }
  int64_t block_numel() const {
    int64_t n = 1;
    for (size_t i = 0; i < shape.size(); ++i) n *= shape[i] / degrees[i];
    return n;
  }
  std::vector<int> block_coords(int b) const;
  int part_index(const std::vector<int>& blk, int rep) const;
  std::vector<int> replica_group(const std::vector<int>& blk) const;
  bool same(const Layout& o) const {
    return shape == o.shape && degrees == o.degrees && replicas == o.replicas && devices == o.devices &&
           halo == o.halo;
  }
};

// One candidate parallelization of an op (an OpConfig plus everything the cost model needs).
struct OpCandidate {
  std::vector<int> degrees;
  std::vector<int> devices;
  double fwd_ms = 0, bwd_ms = 0;  // per-part compute time (parts run concurrently)
  double mem_bytes = 0;           // per-device bytes (activations + weights + grads + optimizer)
  std::vector<Layout> in_layouts;
  std::vector<Layout> out_layouts;
  std::vector<Layout> w_layouts;
};

struct Node {
  std::string name;
  std::string op_type;
  std::vector<std::pair<int, int>> inputs;  // (producer node, producer output index); producer -1 = none
  std::vector<bool> input_needs_grad;
  int elem_bytes = 2;
  bool backward = true;
  std::vector<OpCandidate> cands;
};

struct MachineModel {
  int num_nodes = 1;
  int gpus_per_node = 8;
  // one xGMI link, one direction, GB/s: MI355X's Infinity Fabric link is 153.6 GB/s counting both
  // directions (7 links per GPU, 1075 GB/s aggregate peer bandwidth, the vendor data sheet figure
  // this task quotes as "7 links x ~153 GB/s"), so 76.8 per direction; r1-r4 used MI300X's
  // 128 / 2 = 64. A spec figure, not a measurement: no multi-GPU box was available to this work
  // (coll_eff below is the assumed achieved fraction of it).
  double link_gbps = 76.8;
  double links_per_gpu = 7;        // fully connected 8-GPU node
  double coll_eff = 0.75;          // achieved fraction of the (r-1) x link ring-bus bandwidth
  double inter_node_gbps = 50.0;   // per-GPU NIC bandwidth
  double latency_us = 8.0;         // per collective / P2P batch
  double hbm_gbps = 5800.0;        // achievable HBM bandwidth (local copies)
  double mem_capacity = 288e9;     // HBM3E per GPU
  // machine_model_version 1: explicit topology (routes, per-link contention); null = analytic
  std::shared_ptr<const NetworkTopology> topo;
  int num_devices() const { return num_nodes * gpus_per_node; }
  bool same_node(int a, int b) const { return a / gpus_per_node == b / gpus_per_node; }
  // bus bandwidth (GB/s) of a ring collective over `ranks`
  double ring_busbw(const std::vector<int>& ranks) const;
  double p2p_gbps(int a, int b) const {
    if (topo) return topo->path_gbps(a, b);
    return same_node(a, b) ? link_gbps : inter_node_gbps;
  }
};

// Collective classification of a layout conversion (mirror of flexflow_amd.parallel.comm.Transfer).
enum class XferKind { IDENTITY, LOCAL_SLICE, ALL_REDUCE, REDUCE_SCATTER, ALL_GATHER, ALL_TO_ALL, GENERIC };

struct XferCost {
  XferKind kind = XferKind::IDENTITY;
  double ms = 0;                       // wall time of the transfer
  std::vector<int> devices;            // devices that participate
  double bytes = 0;                    // total bytes moved over links
};

XferCost transfer_cost(const Layout& src, const Layout& dst, bool src_partial, int elem_bytes,
                       const MachineModel& mm);

struct Problem {
  std::vector<Node> nodes;  // topological order
  MachineModel machine;
  // fused Adam over a flat arena, per MB of fp32 parameters: ~30 B of traffic per parameter at the
  // 4.3 TB/s the kernel measures (BERT-Large: 2.58 ms for 366 M parameters, scripts/calibrate_sim.py)
  double update_ms_per_mb = 0.00176;
  bool overlap_grad_sync = true;
};

struct SimResult {
  double makespan_ms = 0;
  double compute_ms = 0;  // max per-device busy compute time
  double comm_ms = 0;     // max per-device busy comm time
  double max_mem = 0;     // max per-device memory
  bool oom = false;
};

class Simulator {
 public:
  explicit Simulator(const Problem& p) : prob_(p) {}
  SimResult simulate(const std::vector<int>& choice) const;
  // additive (non-overlapped) cost of one node given its config and producers' configs; used by DP
  double node_cost(int node, int cfg, const std::vector<int>& producer_cfg) const;
  double edge_cost(int node, int slot, int cfg, int prod_cfg) const;
  double weight_sync_ms(int node, int cfg) const;

 private:
  const Problem& prob_;
  mutable std::unordered_map<uint64_t, double> edge_cache_;
  // simulate(): the transfer of one edge for (node, slot, config, producer config), forward and
  // backward (MCMC re-simulates the whole graph per move; layouts never change within a Problem)
  mutable std::unordered_map<uint64_t, XferCost> xfer_cache_;
  const XferCost& edge_xfer(int node, int slot, int cfg, int prod_cfg, bool backward) const;
};

// One parallel-branch region examined by the non-sequence (resource-split) refinement.
struct SplitInfo {
  int start = -1, end = -1;      // bottleneck nodes bracketing the region (fork, join)
  int components = 0;            // independent branches between them
  int groups = 0;                // device groups tried (0: no feasible split)
  std::vector<int> group_of;     // branch -> device group of the best split
  double whole_ms = 0;           // additive region cost with every branch on the baseline configs
  double split_ms = 0;           // max over device groups of the groups' additive costs
  double sim_before_ms = 0, sim_after_ms = 0;  // whole-graph simulated makespans
  bool accepted = false;
};

struct SearchResult {
  std::vector<SplitInfo> splits;
  std::vector<int> choice;
  double cost_ms = 0;
  double dp_cost_ms = 0;
  double sim_ms = 0;
  int64_t states = 0;
  int iterations = 0;
  std::vector<double> trace;  // best cost over time (MCMC)
};

SearchResult search_dp(const Problem& p, int beam);
SearchResult search_mcmc(const Problem& p, const std::vector<int>& init, int iterations, double alpha, uint64_t seed);
SearchResult search_unity(const Problem& p, int beam, int refine_iters, double alpha, uint64_t seed);
// Sequence split points: node i such that no producer -> consumer edge jumps over it.
std::vector<int> sequence_bottlenecks(const Problem& p);
// Non-sequence split refinement (reference SearchHelper::execute_nonsequence_split, graph.cc:188-330,
// GraphSearchHelper::find_split_node, substitution.cc:2094): between two bottlenecks, independent
// branches are re-searched on disjoint device groups; a split is kept when the simulator's makespan
// (which runs branches on disjoint devices concurrently) improves.
SearchResult search_split(const Problem& p, const std::vector<int>& base, int beam);

// ------------------------------------------------------------------------------ substitutions
struct RuleParam {
  std::string key;
  int value;
};
struct RuleTensor {
  int op_id;  // < 0: external input (-1, -2, ...)
  int ts_id;
};
struct RuleOp {
  std::string type;
  std::vector<RuleTensor> inputs;
  std::vector<RuleParam> params;
};
struct RuleMapOutput {
  int src_op, src_ts, dst_op, dst_ts;
};
struct Rule {
  std::string name;
  std::vector<RuleOp> src, dst;
  std::vector<RuleMapOutput> mapped;
};

std::vector<Rule> load_rules(const std::string& path);

// Lightweight typed graph for substitution matching.
struct GNode {
  std::string type;
  std::map<std::string, int> params;
  std::vector<std::pair<int, int>> inputs;  // (node, out idx); node < 0 = graph input / weight
  int num_outputs = 1;
};
struct Match {
  std::vector<int> op_nodes;              // graph node for each rule src op
  std::map<int, std::pair<int, int>> ext;  // rule external tensor id -> graph (node, idx)
};
std::vector<Match> match_rule(const Rule& r, const std::vector<GNode>& g, int max_matches);

}  // namespace ffcore
