// pybind11 bindings of the native core: flexflow_amd._core
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "dataloader.h"
#include "graph_utils.h"
#include "pcg.h"
#include "request_queue.h"

namespace py = pybind11;
using namespace ffcore;

namespace {

// BatchRing over a numpy dataset and a list of pinned numpy views (one per slot)
class PyBatchRing {
 public:
  PyBatchRing(py::array data, int64_t batch, py::list bufs) : data_(data), bufs_(bufs) {
    auto info = data_.request();
    if (!(data_.flags() & py::array::c_style)) throw std::runtime_error("dataset must be C-contiguous");
    const int64_t n = info.shape[0];
    const int64_t sb = n ? (int64_t)(info.size * info.itemsize / n) : 0;
    std::vector<char*> ptrs;
    for (auto b : bufs) {
      py::array a = py::reinterpret_borrow<py::array>(b);
      auto bi = a.request();
      if ((int64_t)(bi.size * bi.itemsize) < sb * batch) throw std::runtime_error("ring buffer too small");
      ptrs.push_back((char*)bi.ptr);
    }
    ring_.reset(new BatchRing((const char*)info.ptr, n, sb, batch, ptrs));
  }
  int next() {
    py::gil_scoped_release nogil;
    return ring_->next();
  }
  void release(int s) { ring_->release(s); }
  void reset(int64_t start) { ring_->reset(start); }
  int depth() const { return ring_->depth(); }

 private:
  py::array data_;
  py::list bufs_;
  std::unique_ptr<BatchRing> ring_;
};

}  // namespace

PYBIND11_MODULE(_core, m) {
  m.doc() = "flexflow_amd native core: PCG search problem, MI355X machine model, simulator, Unity/MCMC search, "
            "substitutions, data-loader ring";

  py::class_<Layout>(m, "Layout")
      .def(py::init<>())
      .def_readwrite("shape", &Layout::shape)
      .def_readwrite("degrees", &Layout::degrees)
      .def_readwrite("replicas", &Layout::replicas)
      .def_readwrite("devices", &Layout::devices)
      .def_readwrite("partial", &Layout::partial)
      .def_readwrite("halo", &Layout::halo);

  py::class_<OpCandidate>(m, "OpCandidate")
      .def(py::init<>())
      .def_readwrite("degrees", &OpCandidate::degrees)
      .def_readwrite("devices", &OpCandidate::devices)
      .def_readwrite("fwd_ms", &OpCandidate::fwd_ms)
      .def_readwrite("bwd_ms", &OpCandidate::bwd_ms)
      .def_readwrite("mem_bytes", &OpCandidate::mem_bytes)
      .def_readwrite("in_layouts", &OpCandidate::in_layouts)
      .def_readwrite("out_layouts", &OpCandidate::out_layouts)
      .def_readwrite("w_layouts", &OpCandidate::w_layouts);

  py::class_<Node>(m, "Node")
      .def(py::init<>())
      .def_readwrite("name", &Node::name)
      .def_readwrite("op_type", &Node::op_type)
      .def_readwrite("inputs", &Node::inputs)
      .def_readwrite("input_needs_grad", &Node::input_needs_grad)
      .def_readwrite("elem_bytes", &Node::elem_bytes)
      .def_readwrite("backward", &Node::backward)
      .def_readwrite("cands", &Node::cands);

  py::class_<MachineModel>(m, "MachineModel")
      .def(py::init<>())
      .def_readwrite("num_nodes", &MachineModel::num_nodes)
      .def_readwrite("gpus_per_node", &MachineModel::gpus_per_node)
      .def_readwrite("link_gbps", &MachineModel::link_gbps)
      .def_readwrite("links_per_gpu", &MachineModel::links_per_gpu)
      .def_readwrite("coll_eff", &MachineModel::coll_eff)
      .def_readwrite("inter_node_gbps", &MachineModel::inter_node_gbps)
      .def_readwrite("latency_us", &MachineModel::latency_us)
      .def_readwrite("hbm_gbps", &MachineModel::hbm_gbps)
      .def_readwrite("mem_capacity", &MachineModel::mem_capacity)
      .def("num_devices", &MachineModel::num_devices)
      .def("ring_busbw", &MachineModel::ring_busbw)
      .def("p2p_gbps", &MachineModel::p2p_gbps)
      .def("set_topology", [](MachineModel& mm, const NetworkTopology& t) {
        mm.topo = std::make_shared<const NetworkTopology>(t);
      })
      .def("clear_topology", [](MachineModel& mm) { mm.topo.reset(); })
      .def_property_readonly("has_topology", [](const MachineModel& mm) { return (bool)mm.topo; });

  py::class_<NetworkTopology>(m, "NetworkTopology")
      .def(py::init<>())
      .def_readwrite("num_gpus", &NetworkTopology::num_gpus)
      .def_readonly("num_nodes", &NetworkTopology::num_nodes)
      .def("add_node", &NetworkTopology::add_node)
      .def("add_link", &NetworkTopology::add_link)
      .def("build_routes", &NetworkTopology::build_routes)
      .def("route", &NetworkTopology::route)
      .def("hops", &NetworkTopology::hops)
      .def("path_gbps", &NetworkTopology::path_gbps)
      .def("transfers_ms", &NetworkTopology::transfers_ms)
      .def("allreduce_ms", &NetworkTopology::allreduce_ms)
      .def("allgather_ms", &NetworkTopology::allgather_ms)
      .def("ring_busbw", &NetworkTopology::ring_busbw)
      .def_property_readonly("num_links", [](const NetworkTopology& t) { return t.links.size(); });
  m.def("make_mi355x_cluster", &make_mi355x_cluster, py::arg("nodes"), py::arg("gpus_per_node"),
        py::arg("xgmi_gbps") = 64.0, py::arg("nic_gbps") = 50.0, py::arg("kind") = "fat_tree",
        py::arg("oversub") = 1.0);

  py::class_<Problem>(m, "Problem")
      .def(py::init<>())
      .def_readwrite("nodes", &Problem::nodes)
      .def_readwrite("machine", &Problem::machine)
      .def_readwrite("update_ms_per_mb", &Problem::update_ms_per_mb)
      .def_readwrite("overlap_grad_sync", &Problem::overlap_grad_sync);

  py::class_<SimResult>(m, "SimResult")
      .def_readonly("makespan_ms", &SimResult::makespan_ms)
      .def_readonly("compute_ms", &SimResult::compute_ms)
      .def_readonly("comm_ms", &SimResult::comm_ms)
      .def_readonly("max_mem", &SimResult::max_mem)
      .def_readonly("oom", &SimResult::oom);

  py::class_<SplitInfo>(m, "SplitInfo")
      .def_readonly("start", &SplitInfo::start)
      .def_readonly("end", &SplitInfo::end)
      .def_readonly("components", &SplitInfo::components)
      .def_readonly("groups", &SplitInfo::groups)
      .def_readonly("group_of", &SplitInfo::group_of)
      .def_readonly("whole_ms", &SplitInfo::whole_ms)
      .def_readonly("split_ms", &SplitInfo::split_ms)
      .def_readonly("sim_before_ms", &SplitInfo::sim_before_ms)
      .def_readonly("sim_after_ms", &SplitInfo::sim_after_ms)
      .def_readonly("accepted", &SplitInfo::accepted);

  py::class_<SearchResult>(m, "SearchResult")
      .def_readonly("splits", &SearchResult::splits)
      .def_readonly("choice", &SearchResult::choice)
      .def_readonly("cost_ms", &SearchResult::cost_ms)
      .def_readonly("dp_cost_ms", &SearchResult::dp_cost_ms)
      .def_readonly("sim_ms", &SearchResult::sim_ms)
      .def_readonly("states", &SearchResult::states)
      .def_readonly("iterations", &SearchResult::iterations)
      .def_readonly("trace", &SearchResult::trace);

  py::enum_<XferKind>(m, "XferKind")
      .value("IDENTITY", XferKind::IDENTITY)
      .value("LOCAL_SLICE", XferKind::LOCAL_SLICE)
      .value("ALL_REDUCE", XferKind::ALL_REDUCE)
      .value("REDUCE_SCATTER", XferKind::REDUCE_SCATTER)
      .value("ALL_GATHER", XferKind::ALL_GATHER)
      .value("ALL_TO_ALL", XferKind::ALL_TO_ALL)
      .value("GENERIC", XferKind::GENERIC);

  py::class_<XferCost>(m, "XferCost")
      .def_readonly("kind", &XferCost::kind)
      .def_readonly("ms", &XferCost::ms)
      .def_readonly("devices", &XferCost::devices)
      .def_readonly("bytes", &XferCost::bytes);

  m.def("transfer_cost", &transfer_cost, py::arg("src"), py::arg("dst"), py::arg("src_partial"),
        py::arg("elem_bytes"), py::arg("machine"));
  m.def("simulate", [](const Problem& p, const std::vector<int>& choice) { return Simulator(p).simulate(choice); });
  m.def("search_dp", &search_dp, py::arg("problem"), py::arg("beam") = 4096,
        py::call_guard<py::gil_scoped_release>());
  m.def("search_mcmc", &search_mcmc, py::arg("problem"), py::arg("init"), py::arg("iterations"),
        py::arg("alpha") = 1.2, py::arg("seed") = 0, py::call_guard<py::gil_scoped_release>());
  m.def("search_unity", &search_unity, py::arg("problem"), py::arg("beam") = 4096, py::arg("refine_iters") = 500,
        py::arg("alpha") = 1.2, py::arg("seed") = 0, py::call_guard<py::gil_scoped_release>());

  m.def("sequence_bottlenecks", &sequence_bottlenecks, py::arg("problem"));
  m.def("search_split", &search_split, py::arg("problem"), py::arg("base"), py::arg("beam") = 4096,
        py::call_guard<py::gil_scoped_release>());

  py::class_<RuleParam>(m, "RuleParam").def_readonly("key", &RuleParam::key).def_readonly("value", &RuleParam::value);
  py::class_<RuleTensor>(m, "RuleTensor").def_readonly("op_id", &RuleTensor::op_id).def_readonly("ts_id", &RuleTensor::ts_id);
  py::class_<RuleOp>(m, "RuleOp")
      .def_readonly("type", &RuleOp::type)
      .def_readonly("inputs", &RuleOp::inputs)
      .def_readonly("params", &RuleOp::params);
  py::class_<RuleMapOutput>(m, "RuleMapOutput")
      .def_readonly("src_op", &RuleMapOutput::src_op)
      .def_readonly("src_ts", &RuleMapOutput::src_ts)
      .def_readonly("dst_op", &RuleMapOutput::dst_op)
      .def_readonly("dst_ts", &RuleMapOutput::dst_ts);
  py::class_<Rule>(m, "Rule")
      .def_readonly("name", &Rule::name)
      .def_readonly("src", &Rule::src)
      .def_readonly("dst", &Rule::dst)
      .def_readonly("mapped", &Rule::mapped);
  m.def("load_rules", &load_rules);

  py::class_<GNode>(m, "GNode")
      .def(py::init<>())
      .def_readwrite("type", &GNode::type)
      .def_readwrite("params", &GNode::params)
      .def_readwrite("inputs", &GNode::inputs)
      .def_readwrite("num_outputs", &GNode::num_outputs);
  py::class_<Match>(m, "Match").def_readonly("op_nodes", &Match::op_nodes).def_readonly("ext", &Match::ext);
  m.def("match_rule", &match_rule, py::arg("rule"), py::arg("graph"), py::arg("max_matches") = 64);

  py::class_<PyBatchRing>(m, "BatchRing")
      .def(py::init<py::array, int64_t, py::list>())
      .def("next", &PyBatchRing::next)
      .def("release", &PyBatchRing::release)
      .def("reset", &PyBatchRing::reset)
      .def("depth", &PyBatchRing::depth);

  // ---------------------------------------------------------------- graph / machine utilities
  py::class_<Digraph>(m, "Digraph")
      .def(py::init<int>(), py::arg("n") = 0)
      .def(py::init([](int n, const std::vector<std::pair<int, int>>& edges) {
             Digraph g(n);
             for (auto& e : edges) g.add_edge(e.first, e.second);
             return g;
           }),
           py::arg("n"), py::arg("edges"))
      .def("num_nodes", &Digraph::num_nodes)
      .def("add_node", &Digraph::add_node)
      .def("add_edge", &Digraph::add_edge)
      .def("remove_edge", &Digraph::remove_edge)
      .def("has_edge", &Digraph::has_edge)
      .def("successors", &Digraph::successors)
      .def("predecessors", &Digraph::predecessors)
      .def("edges", &Digraph::edges)
      .def("roots", &Digraph::roots)
      .def("leaves", &Digraph::leaves)
      .def("topo_order", &Digraph::topo_order)
      .def("dominators", &Digraph::dominators)
      .def("post_dominators", &Digraph::post_dominators)
      .def("imm_dominators", &Digraph::imm_dominators)
      .def("imm_post_dominators", &Digraph::imm_post_dominators)
      .def("bottlenecks", &Digraph::bottlenecks)
      .def("descendants", &Digraph::descendants, py::arg("v"), py::arg("undirected") = false)
      .def("weakly_connected_components", &Digraph::weakly_connected_components)
      .def("transitive_reduction", &Digraph::transitive_reduction);

  py::class_<DisjointSet>(m, "DisjointSet")
      .def(py::init<int>())
      .def("find", &DisjointSet::find)
      .def("unite", &DisjointSet::unite)
      .def("same", &DisjointSet::same)
      .def("size", &DisjointSet::size);
  m.def("select_random", &select_random, py::arg("weights"), py::arg("u"));
  m.def("hash_combine", [](uint64_t seed, uint64_t v) {
    hash_combine(seed, v);
    return seed;
  });

  py::class_<MachineView>(m, "MachineView")
      .def(py::init([](int start, std::vector<int> dim, std::vector<int> stride) {
             if (dim.size() != stride.size()) throw std::invalid_argument("MachineView: dim/stride rank mismatch");
             MachineView v;
             v.start_device_id = start;
             v.dim = std::move(dim);
             v.stride = std::move(stride);
             return v;
           }),
           py::arg("start_device_id") = 0, py::arg("dim") = std::vector<int>{1}, py::arg("stride") = std::vector<int>{1})
      .def_readwrite("device_type", &MachineView::device_type)
      .def_readwrite("start_device_id", &MachineView::start_device_id)
      .def_readwrite("dim", &MachineView::dim)
      .def_readwrite("stride", &MachineView::stride)
      .def_property_readonly("ndims", &MachineView::ndims)
      .def("num_parts", &MachineView::num_parts)
      .def("device_id", &MachineView::device_id)
      .def("device_ids", &MachineView::device_ids)
      .def("hash", &MachineView::hash)
      .def("__eq__", &MachineView::operator==)
      .def("__hash__", [](const MachineView& v) { return (int64_t)(v.hash() >> 1); })
      .def("__repr__", &MachineView::str);

  py::class_<MachineResource>(m, "MachineResource")
      .def(py::init([](int nodes, int gpus, int avail, int start) {
             MachineResource r;
             r.num_nodes = nodes;
             r.all_gpus_per_node = gpus;
             r.available_gpus_per_node = avail < 0 ? gpus : avail;
             r.start_gpu_id = start;
             return r;
           }),
           py::arg("num_nodes") = 1, py::arg("gpus_per_node") = 8, py::arg("available_gpus_per_node") = -1,
           py::arg("start_gpu_id") = 0)
      .def_readwrite("num_nodes", &MachineResource::num_nodes)
      .def_readwrite("all_gpus_per_node", &MachineResource::all_gpus_per_node)
      .def_readwrite("available_gpus_per_node", &MachineResource::available_gpus_per_node)
      .def_readwrite("start_gpu_id", &MachineResource::start_gpu_id)
      .def("is_valid_machine_view", &MachineResource::is_valid_machine_view)
      .def("enumerate_views", &MachineResource::enumerate_views, py::arg("max_parts") = 0);
  py::class_<RequestQueue>(m, "RequestQueue")
      .def(py::init<int64_t, int64_t, std::vector<int64_t>>(), py::arg("max_rows"), py::arg("max_delay_us"),
           py::arg("preferred") = std::vector<int64_t>{})
      .def("push", &RequestQueue::push)
      .def("pop", &RequestQueue::pop, py::arg("timeout_us") = -1, py::call_guard<py::gil_scoped_release>())
      .def("close", &RequestQueue::close)
      .def("queued_requests", &RequestQueue::queued_requests)
      .def("queued_rows", &RequestQueue::queued_rows)
      .def("stats", &RequestQueue::stats);
}
