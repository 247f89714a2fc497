// Topology-aware network model for the simulator (machine_model_version 1).
//
// Reference counterpart: src/runtime/network.cc + include/flexflow/simulator.h
// (NetworkedMachineModel, FatTreeNetworkTopologyGenerator, BigSwitchNetworkTopologyGenerator,
// WeightedShortestPathRoutingStrategy) — re-designed for MI355X nodes: 8 GPUs per node fully
// connected by xGMI (7 point-to-point links per GPU), one NIC per GPU into a switch fabric.
//
// The model is a graph of devices (GPUs first, then switches) joined by full-duplex links. A
// transfer follows a shortest-hop route (ties broken by the widest bottleneck); a set of
// concurrent transfers costs the time of its most loaded directed link. Collectives are costed
// the way RCCL runs them on this hardware: on a fully connected node a ring collective is split
// over r-1 rotated rings (every direct link carries 1/(r-1) of the data), across nodes the same
// rings contend on the NIC uplinks.
#pragma once
#include <cstdint>
#include <string>
#include <tuple>
#include <vector>

namespace ffcore {

struct NetLink {
  int a = 0, b = 0;      // endpoints (device or switch id)
  double gbps = 0;       // per direction, GB/s
};

class NetworkTopology {
 public:
  int num_gpus = 0;
  int num_nodes = 0;  // total vertices (GPUs + switches)
  std::vector<NetLink> links;

  int add_node() { return num_nodes++; }
  void add_link(int a, int b, double gbps);
  // all-pairs routes; call after the last add_link
  void build_routes();

  // directed link ids (2 * link index + direction) along the route a -> b
  std::vector<int> route(int a, int b) const;
  // bottleneck bandwidth (GB/s) of the route a -> b
  double path_gbps(int a, int b) const;
  int hops(int a, int b) const;
  // time (ms) of concurrent transfers (src, dst, bytes): the most loaded directed link
  double transfers_ms(const std::vector<std::tuple<int, int, double>>& xfers) const;
  // ring all-reduce / all-gather (or reduce-scatter) of `bytes` over `ranks`, time in ms
  double allreduce_ms(const std::vector<int>& ranks, double bytes) const;
  double allgather_ms(const std::vector<int>& ranks, double bytes) const;
  // effective bus bandwidth (GB/s) of a ring all-reduce over `ranks` (large-message limit)
  double ring_busbw(const std::vector<int>& ranks) const;

 private:
  std::vector<std::vector<int>> nxt_;   // next hop vertex
  std::vector<std::vector<int>> via_;   // directed link id of the first hop
  std::vector<std::vector<int>> dist_;  // hop count
  double ring_steps_ms(const std::vector<int>& ranks, double chunk_bytes, int steps) const;
};

// MI355X cluster: `nodes` x `gpus_per_node` GPUs, xGMI all-to-all inside a node, one NIC per GPU
// (`nic_gbps`) into a fabric: kind "big_switch" (one non-blocking switch) or "fat_tree" (a leaf
// switch per node, `oversub`-times oversubscribed uplinks to one spine).
NetworkTopology make_mi355x_cluster(int nodes, int gpus_per_node, double xgmi_gbps, double nic_gbps,
                                    const std::string& kind, double oversub);

}  // namespace ffcore
