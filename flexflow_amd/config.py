"""FFConfig: run configuration, CLI flag parsing and machine discovery.

Flag names mirror the reference (`FFConfig::parse_args`, src/runtime/model.cc:3566-3730; fields
include/flexflow/config.h:92-160) so existing launch scripts keep working. Machine discovery is
MI355X/SPMD-native: one process per GPU, world/rank from the torchrun environment
(WORLD_SIZE / RANK / LOCAL_RANK / LOCAL_WORLD_SIZE) instead of Realm machine queries; `-ll:gpu`
is accepted and used only when no launcher environment is present.
"""
from __future__ import annotations

import os
import warnings
import sys
import time

from .type import CompMode, DataType


# short flags we share with launchers that may leave their argv in sys.argv (pytest: -p plugin)
_FOREIGN_COLLISIONS = frozenset({"-p"})


class FFConfig:
    # reference DefaultConfig (model.cc:3470-3499)
    DEFAULT_BATCH_SIZE = 64

    def __init__(self, argv: list[str] | None = None):
        self.epochs = 1
        self.batch_size = self.DEFAULT_BATCH_SIZE
        self.print_freq = 10
        self.learning_rate = 0.01
        self.weight_decay = 0.0001
        self.profiling = False
        self.work_space_size = 1 << 30
        self.device_mem = 0.0
        self.num_nodes = 1
        self.cpus_per_node = 0
        self.workers_per_node = 0
        self.dataset_path = ""
        self.search_budget = -1
        self.search_alpha = 1.2
        # wall-clock bound (s) of the joint graph search loop on rank 0 (the other ranks wait in a
        # broadcast meanwhile); <= 0: unbounded. FF_SEARCH_TIME_S overrides.
        self.search_time_s = float(os.environ.get("FF_SEARCH_TIME_S", "120"))
        self.search_overlap_backward_update = False
        self.computation_mode = CompMode.TRAINING
        self.only_data_parallel = False
        self.enable_sample_parallel = True
        self.enable_parameter_parallel = False
        self.enable_attribute_parallel = False
        self.enable_inplace_optimizations = False
        self.allow_tensor_op_math_conversion = False
        self.import_strategy_file = ""
        self.export_strategy_file = ""
        self.import_rewrites_file = ""  # graph rewrites of a joint search (strategy JSON or a list)
        self.export_strategy_task_graph_file = ""
        self.export_strategy_computation_graph_file = ""
        self.include_costs_dot_graph = False
        self.machine_model_version = 0
        self.machine_model_file = ""
        self.simulator_segment_size = 16 * 1024 * 1024
        self.simulator_max_num_segments = 1
        self.enable_propagation = False
        self.search_num_nodes = None
        self.search_num_workers = None
        self.base_optimize_threshold = 10
        self.enable_control_replication = True
        self.python_data_loader_type = 2
        self.substitution_json_path = None
        self.perform_fusion = False
        self.perform_memory_search = False
        self.synthetic_input = False
        # MI355X-native additions
        self.compute_dtype = DataType.DT_FLOAT  # models built in fp32 unless --dtype bf16
        # hipGraph capture of the train step: "auto" captures only when the eager step is short
        # enough for launch overhead to matter (runtime/graph.py), True always, False never
        self.hip_graphs = "auto"
        self.graph_min_step_ms = 15.0
        # eager steps up to this long are captured on trial (runtime/graph.py); FF_GRAPH_TRIAL_MAX_MS
        self.graph_trial_max_ms = float(os.environ.get("FF_GRAPH_TRIAL_MAX_MS", "30"))
        self.search_algo = "unity"  # unity | mcmc | dp (data-parallel only) | none
        self.mcmc_iterations = 2000
        self.grad_bucket_mb = 64.0
        self.grad_comm_dtype = "fp32"  # --grad-comm-dtype bf16: gradient buckets travel as bf16
        self.zero_optimizer = False   # --zero: ZeRO-1 sharded optimizer state / update on DP arenas
        # train_step runs each gradient bucket's optimizer update on a side stream as soon as the
        # bucket is final (all-reduced), overlapping the rest of the backward (runtime/executor.py
        # 'overlapped update'; bitwise-identical, BERT-Large 47.56 -> 47.35 ms/step on one
        # MI355X); --overlap-update / --no-overlap-update, FF_OVERLAP_UPDATE=0|1
        self.overlap_update = os.environ.get("FF_OVERLAP_UPDATE", "1") != "0"
        self.seed = 1234
        self.cpu_only = False  # -ll:gpu 0 / --device cpu: run on the host even with a GPU present
        self.trace_dir = ""
        self.check_nan_every = 0      # --check-nan N: loss finite-check every N steps (0 = off)
        self.watchdog_s = 0.0         # --watchdog S: dump all stacks if a step exceeds S seconds
        self.dist_timeout_s = 1800.0  # --dist-timeout S: torch.distributed collective timeout
        self.iter_config_seq_length = -1
        self._traces: dict = {}
        self._trace_active = None  # begin_trace / end_trace -> hipGraphs (runtime/trace.py)
        self._trace_state: dict = {}

        self._discover_machine()
        if argv is None:
            from .jupyter import jupyter_argv  # notebook flags from a config file (flexflow_amd/jupyter.py)
            argv = jupyter_argv() + sys.argv[1:]
        self.parse_args(argv)

    # -------------------------------------------------------------------- machine
    def _discover_machine(self):
        env = os.environ
        if "WORLD_SIZE" in env:
            self.world_size = int(env["WORLD_SIZE"])
            self.rank = int(env.get("RANK", "0"))
            self.local_rank = int(env.get("LOCAL_RANK", str(self.rank)))
            self.local_world_size = int(env.get("LOCAL_WORLD_SIZE", str(self.world_size)))
        else:
            self.world_size, self.rank, self.local_rank, self.local_world_size = 1, 0, 0, 1
        self.num_nodes = max(1, self.world_size // max(1, self.local_world_size))
        self.workers_per_node = self.local_world_size

    # -------------------------------------------------------------------- flags
    def parse_args(self, argv: list[str]):
        i = 0
        n = len(argv)

        def nxt():
            nonlocal i
            i += 1
            return argv[i] if i < n else None

        while i < n:
            a = argv[i]
            try:
                if a in ("-e", "--epochs"):
                    self.epochs = int(nxt())
                elif a in ("-b", "--batch-size"):
                    self.batch_size = int(nxt())
                elif a in ("--lr", "--learning-rate"):
                    self.learning_rate = float(nxt())
                elif a in ("--wd", "--weight-decay"):
                    self.weight_decay = float(nxt())
                elif a in ("-p", "--print-freq"):
                    self.print_freq = int(nxt())
                elif a in ("-d", "--dataset"):
                    self.dataset_path = nxt()
                elif a in ("--budget", "--search-budget"):
                    self.search_budget = int(nxt())
                elif a == "--search-time-s":
                    self.search_time_s = float(nxt())
                elif a in ("--alpha", "--search-alpha"):
                    self.search_alpha = float(nxt())
                elif a in ("--import", "--import-strategy"):
                    self.import_strategy_file = nxt()
                elif a in ("--export", "--export-strategy"):
                    self.export_strategy_file = nxt()
                elif a == "--import-rewrites":
                    self.import_rewrites_file = nxt()
                elif a == "--only-data-parallel":
                    self.only_data_parallel = True
                elif a == "--enable-parameter-parallel":
                    self.enable_parameter_parallel = True
                elif a == "--enable-attribute-parallel":
                    self.enable_attribute_parallel = True
                elif a == "-ll:gpu":
                    v = int(nxt())
                    if v == 0:  # the reference's CPU-only run (-ll:gpu 0)
                        self.cpu_only = True
                    elif "WORLD_SIZE" not in os.environ:
                        self.workers_per_node = v
                elif a == "--device":
                    self.cpu_only = nxt() == "cpu"
                elif a == "-ll:fsize":
                    self.device_mem = float(nxt())
                elif a == "--nodes":
                    self.num_nodes = int(nxt())
                elif a == "-ll:cpu":
                    self.cpus_per_node = int(nxt())
                elif a == "--profiling":
                    self.profiling = True
                elif a == "--allow-tensor-op-math-conversion":
                    self.allow_tensor_op_math_conversion = True
                elif a == "--fusion":
                    self.perform_fusion = True
                elif a == "--overlap":
                    self.search_overlap_backward_update = True
                elif a == "--taskgraph":
                    self.export_strategy_task_graph_file = nxt()
                elif a == "--include-costs-dot-graph":
                    self.include_costs_dot_graph = True
                elif a == "--compgraph":
                    self.export_strategy_computation_graph_file = nxt()
                elif a == "--machine-model-version":
                    self.machine_model_version = int(nxt())
                elif a == "--machine-model-file":
                    self.machine_model_file = nxt()
                elif a == "--simulator-segment-size":
                    self.simulator_segment_size = int(nxt())
                elif a == "--simulator-max-num-segments":
                    self.simulator_max_num_segments = int(nxt())
                elif a == "--enable-propagation":
                    self.enable_propagation = True
                elif a == "--enable-inplace-optimizations":
                    self.enable_inplace_optimizations = True
                elif a == "--search-num-nodes":
                    self.search_num_nodes = int(nxt())
                elif a == "--search-num-workers":
                    self.search_num_workers = int(nxt())
                elif a == "--base-optimize-threshold":
                    self.base_optimize_threshold = int(nxt())
                elif a == "--disable-control-replication":
                    self.enable_control_replication = False
                elif a == "--python-data-loader-type":
                    self.python_data_loader_type = int(nxt())
                elif a == "--substitution-json":
                    self.substitution_json_path = nxt()
                elif a == "--memory-search":
                    self.perform_memory_search = True
                # ---- MI355X-native flags
                elif a == "--dtype":
                    v = nxt()
                    self.compute_dtype = {"bf16": DataType.DT_BF16, "fp32": DataType.DT_FLOAT,
                                          "float": DataType.DT_FLOAT}[v]
                elif a == "--no-hip-graphs":
                    self.hip_graphs = False
                elif a == "--hip-graphs":
                    self.hip_graphs = True
                elif a == "--search":
                    self.search_algo = nxt()
                elif a == "--mcmc-iterations":
                    self.mcmc_iterations = int(nxt())
                elif a == "--zero":
                    self.zero_optimizer = True
                elif a == "--overlap-update":
                    self.overlap_update = True
                elif a == "--no-overlap-update":
                    self.overlap_update = False
                elif a == "--grad-bucket-mb":
                    self.grad_bucket_mb = float(nxt())
                elif a == "--grad-comm-dtype":
                    self.grad_comm_dtype = nxt()
                    if self.grad_comm_dtype not in ("fp32", "bf16"):
                        raise ValueError(f"--grad-comm-dtype must be fp32 or bf16, not {self.grad_comm_dtype!r}")
                elif a == "--seed":
                    self.seed = int(nxt())
                elif a == "--trace-dir":
                    self.trace_dir = nxt()
                elif a == "--check-nan":
                    self.check_nan_every = int(nxt())
                elif a == "--watchdog":
                    self.watchdog_s = float(nxt())
                elif a == "--dist-timeout":
                    self.dist_timeout_s = float(nxt())
            except (TypeError, ValueError):
                v = argv[i] if i < n else None
                if v is not None and not v.startswith("-") and a not in _FOREIGN_COLLISIONS:
                    raise ValueError(f"FFConfig: bad value {v!r} for flag {a!r}") from None
                # a flag of another program (pytest's `-p no:cacheprovider`) or a flag whose value
                # is missing / is the next flag: keep the default and re-read the next flag. (The
                # reference's atoi/atof parser would set 0 instead, src/runtime/model.cc:3567-3580.)
                warnings.warn(f"FFConfig: ignoring flag {a!r} (value {v!r} not ours to parse)")
                if v is not None and v.startswith("-"):
                    i -= 1
            i += 1
        if self.only_data_parallel:
            self.search_algo = "dp"

    # -------------------------------------------------------------------- helpers
    @property
    def batchSize(self):  # reference C++ spelling
        return self.batch_size

    @property
    def workersPerNode(self):
        return self.workers_per_node

    @property
    def numNodes(self):
        return self.num_nodes

    @property
    def num_devices(self) -> int:
        """Devices the search plans for (reference: search_num_nodes * search_num_workers)."""
        if self.search_num_workers is not None:
            return (self.search_num_nodes or 1) * self.search_num_workers
        return self.world_size

    def get_current_time(self) -> float:
        """Microseconds, like Realm::Clock::current_time_in_microseconds."""
        return time.perf_counter() * 1e6

    def begin_trace(self, trace_id: int):
        """Start of a traced iteration body: repeated bodies are captured into a hipGraph and
        replayed (runtime/trace.py), the counterpart of the reference's Legion tracing."""
        from .runtime import trace
        self._traces[trace_id] = True
        trace.begin(self, trace_id)

    def end_trace(self, trace_id: int):
        from .runtime import trace
        self._traces.pop(trace_id, None)
        trace.end(self, trace_id)

    def get_batch_size(self):
        return self.batch_size

    def get_workers_per_node(self):
        return self.workers_per_node

    def get_num_nodes(self):
        return self.num_nodes

    def get_epochs(self):
        return self.epochs

    def get_enable_control_replication(self):
        return self.enable_control_replication

    def get_python_data_loader_type(self):
        return self.python_data_loader_type


class FFIterationConfig:
    def __init__(self):
        self.seq_length = -1

    def reset(self):
        self.seq_length = -1
