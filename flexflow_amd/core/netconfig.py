"""Example-config helpers (reference flexflow_cffi.py NetConfig:2404-2414, DLRMConfig:2415-2450)."""
import sys


class NetConfig:
    def __init__(self, argv=None):
        argv = sys.argv[1:] if argv is None else argv
        self.dataset_path = ""
        for i, a in enumerate(argv):
            if a in ("-d", "--dataset") and i + 1 < len(argv):
                self.dataset_path = argv[i + 1]


class DLRMConfig:
    def __init__(self, argv=None):
        argv = sys.argv[1:] if argv is None else argv
        self.sparse_feature_size = 64
        self.sigmoid_bot = -1
        self.sigmoid_top = -1
        self.embedding_bag_size = 1
        self.loss_threshold = 0.0
        self.embedding_size = [1000000] * 8
        self.mlp_bot = [4, 64, 64]
        self.mlp_top = [64, 64, 2]
        self.arch_interaction_op = "cat"
        self.dataset_path = ""
        self.data_size = -1
        i = 0
        while i < len(argv):
            a = argv[i]
            nxt = argv[i + 1] if i + 1 < len(argv) else None
            if a == "--arch-sparse-feature-size":
                self.sparse_feature_size = int(nxt); i += 1
            elif a == "--arch-embedding-size":
                self.embedding_size = [int(x) for x in nxt.split("-")]; i += 1
            elif a == "--embedding-bag-size":
                self.embedding_bag_size = int(nxt); i += 1
            elif a == "--arch-mlp-bot":
                self.mlp_bot = [int(x) for x in nxt.split("-")]; i += 1
            elif a == "--arch-mlp-top":
                self.mlp_top = [int(x) for x in nxt.split("-")]; i += 1
            elif a == "--loss-threshold":
                self.loss_threshold = float(nxt); i += 1
            elif a == "--sigmoid-top":
                self.sigmoid_top = int(nxt); i += 1
            elif a == "--sigmoid-bot":
                self.sigmoid_bot = int(nxt); i += 1
            elif a == "--arch-interaction-op":
                self.arch_interaction_op = nxt; i += 1
            elif a == "--dataset":
                self.dataset_path = nxt; i += 1
            elif a == "--data-size":
                self.data_size = int(nxt); i += 1
            i += 1
