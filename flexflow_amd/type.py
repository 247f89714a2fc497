"""Enumerations of the FlexFlow API.

Numeric values are kept identical to the reference (include/flexflow/ffconst.h:1-240 and
python/flexflow/type.py) because the `.ff` model files written by the torch frontend and the
JSON strategy / substitution files name operators and modes by these values/names.
"""
from enum import Enum, IntEnum


class ActiMode(Enum):
    AC_MODE_NONE = 10
    AC_MODE_RELU = 11
    AC_MODE_SIGMOID = 12
    AC_MODE_TANH = 13
    AC_MODE_GELU = 14


class RegularizerMode(Enum):
    REG_MODE_NONE = 17
    REG_MODE_L1 = 18
    REG_MODE_L2 = 19


class AggrMode(Enum):
    AGGR_MODE_NONE = 20
    AGGR_MODE_SUM = 21
    AGGR_MODE_AVG = 22


class PoolType(Enum):
    POOL_MAX = 30
    POOL_AVG = 31


class DataType(Enum):
    DT_BOOLEAN = 40
    DT_INT32 = 41
    DT_INT64 = 42
    DT_HALF = 43
    DT_FLOAT = 44
    DT_DOUBLE = 45
    DT_BF16 = 46  # new: CDNA4 compute dtype (not in the reference, which has no bf16)
    DT_NONE = 49


class LossType(Enum):
    LOSS_CATEGORICAL_CROSSENTROPY = 50
    LOSS_SPARSE_CATEGORICAL_CROSSENTROPY = 51
    LOSS_MEAN_SQUARED_ERROR_AVG_REDUCE = 52
    LOSS_MEAN_SQUARED_ERROR_SUM_REDUCE = 53
    LOSS_IDENTITY = 54


class CompMode(Enum):
    TRAINING = 70
    INFERENCE = 71


class ParameterSyncType(Enum):
    NONE = 80
    PS = 81
    NCCL = 82


class MetricsType(Enum):
    METRICS_ACCURACY = 1001
    METRICS_CATEGORICAL_CROSSENTROPY = 1002
    METRICS_SPARSE_CATEGORICAL_CROSSENTROPY = 1004
    METRICS_MEAN_SQUARED_ERROR = 1008
    METRICS_ROOT_MEAN_SQUARED_ERROR = 1016
    METRICS_MEAN_ABSOLUTE_ERROR = 1032


class OperatorType(IntEnum):
    """Internal operator types (reference include/flexflow/ffconst.h OperatorType, TASO order)."""
    OP_INPUT = 0
    OP_WEIGHT = 1
    OP_NOOP = 2
    OP_CONV2D = 3
    OP_DROPOUT = 4
    OP_LINEAR = 5
    OP_BATCHMATMUL = 6
    OP_POOL2D = 7
    OP_SCALAR_MULTIPLY = 8
    OP_SCALAR_ADD = 9
    OP_SCALAR_FLOOR_DIV = 10
    OP_SCALAR_TRUE_DIV = 11
    OP_SCALAR_SUB = 12
    OP_RELU = 13
    OP_IDENTITY = 14
    OP_SIGMOID = 15
    OP_TANH = 16
    OP_ELU = 17
    OP_FLAT = 18
    OP_SOFTMAX = 19
    OP_BATCHNORM = 20
    OP_CONCAT = 21
    OP_SPLIT = 22
    OP_EMBEDDING = 23
    OP_GROUP_BY = 24
    OP_CACHE = 25
    OP_AGGREGATE = 26
    OP_AGG_SPEC = 27
    OP_RESHAPE = 28
    OP_REVERSE = 29
    OP_TRANSPOSE = 30
    OP_EW_ADD = 31
    OP_EW_MUL = 32
    OP_MATMUL = 33
    OP_MUL = 34
    OP_ENLARGE = 35
    OP_MERGE_GCONV = 36
    OP_CONSTANT_IMM = 37
    OP_CONSTANT_ICONV = 38
    OP_CONSTANT_ONE = 39
    OP_CONSTANT_POOL = 40
    OP_SQUEEZE = 41
    OP_UNSQUEEZE = 42
    OP_EW_SUB = 43
    OP_EW_DIV = 44
    OP_EW_EQUAL = 45
    OP_EW_GREATER = 46
    OP_EW_LESS = 47
    OP_EW_MAX = 48
    OP_EW_MIN = 49
    OP_REDUCE_ARGMAX = 50
    OP_REDUCE_ARGMIN = 51
    OP_REDUCE_MAX = 52
    OP_REDUCE_MEAN = 53
    OP_REDUCE_MIN = 54
    OP_REDUCE_PROD = 55
    OP_REDUCE_SUM = 56
    OP_PAD = 57
    OP_SHAPE = 58
    OP_SIZE = 59
    OP_TOPK = 60
    OP_WHERE = 61
    OP_CEIL = 62
    OP_CAST = 63
    OP_EXP = 64
    OP_ROUND = 65
    OP_LOG = 66
    OP_LOGICAL_NOT = 67
    OP_SQRT = 68
    OP_SIN = 69
    OP_COS = 70
    OP_LEAKYRELU = 71
    OP_SLICE = 72
    OP_RESIZE = 73
    OP_PRELU = 74
    OP_GELU = 75
    OP_MULTIHEAD_ATTENTION = 76
    OP_FUSED = 77
    OP_RSQRT = 78
    OP_POW = 79
    OP_MEAN = 80
    OP_LAYERNORM = 81
    OP_GATHER = 82
    # Parallel ops
    OP_REPARTITION = 83
    OP_COMBINE = 84
    OP_REPLICATE = 85
    OP_REDUCTION = 86
    OP_PIPELINE = 87
    OP_FUSED_PARALLEL = 88
    OP_ALLREDUCE = 89  # extension: explicit all-reduce parallel op (not in the reference snapshot's enum)
    OP_INVALID = 89
    OP_LSTM = 100  # extension: LSTM layer (the reference's legacy nmt/ app, outside FFModel)
    OP_RMS_NORM = 101  # extension: RMS norm (T5 / LLaMA), met by the HuggingFace import path


class OpType(Enum):
    """Frontend (python) op types used by the torch `.ff` file format (reference python/flexflow/type.py)."""
    CONV2D = 2011
    EMBEDDING = 2012
    POOL2D = 2013
    LINEAR = 2014
    SOFTMAX = 2015
    CONCAT = 2016
    FLAT = 2017
    MSELOSS = 2020
    BATCH_NORM = 2021
    RELU = 2022
    SIGMOID = 2023
    TANH = 2024
    ELU = 2025
    DROPOUT = 2026
    BATCH_MATMUL = 2027
    SPLIT = 2028
    RESHAPE = 2029
    TRANSPOSE = 2030
    REVERSE = 2031
    EXP = 2040
    ADD = 2041
    SUBTRACT = 2042
    MULTIPLY = 2043
    DIVIDE = 2044
    POW = 2045
    MEAN = 2046
    RSQRT = 2047
    SIN = 2048
    COS = 2049
    INPUT = 2050
    OUTPUT = 2051
    REDUCE_SUM = 2052
    MAX = 2053
    MIN = 2054
    MULTIHEAD_ATTENTION = 2060
    GETITEM = 2070
    GETATTR = 2080
    EXPAND = 2081
    LAYER_NORM = 2082
    FLOOR_DIVIDE = 2083
    IDENTITY = 2084
    GELU = 2085
    PERMUTE = 2086
    SCALAR_MULTIPLY = 2087
    SCALAR_FLOORDIV = 2088
    SCALAR_ADD = 2089
    SCALAR_SUB = 2090
    SCALAR_TRUEDIV = 2091
    INIT_PARAM = 2092
    FLOAT = 2100
    CONTIGUOUS = 2101
    TO = 2102
    UNSQUEEZE = 2103
    TYPE_AS = 2104
    VIEW = 2105
    GATHER = 2106
    ATTRIBUTE = 2200


class PMParameter(IntEnum):
    """Substitution-pattern parameters (reference ffconst.h PMParameter)."""
    PM_OP_TYPE = 0
    PM_NUM_INPUTS = 1
    PM_NUM_OUTPUTS = 2
    PM_GROUP = 3
    PM_KERNEL_H = 4
    PM_KERNEL_W = 5
    PM_STRIDE_H = 6
    PM_STRIDE_W = 7
    PM_PADDING_H = 8
    PM_PADDING_W = 9
    PM_ACTI = 10
    PM_NUMDIM = 11
    PM_AXIS = 12
    PM_PERM = 13
    PM_OUTSHUFFLE = 14
    PM_MERGE_GCONV_COUNT = 15
    PM_AXES = 16
    PM_KEEP_DIMS = 17
    PM_EPSILON = 18
    PM_REPARTITION_DIM = 19
    PM_REPARTITION_DEGREE = 20
    PM_REPLICATE_DIM = 21
    PM_REPLICATE_DEGREE = 22
    PM_COMBINE_DIM = 23
    PM_COMBINE_DEGREE = 24
    PM_REDUCTION_DIM = 25
    PM_REDUCTION_DEGREE = 26
    PM_SOFTMAX_DIM = 27
    PM_NUM_HEADS = 28
    PM_INVALID = 29
    PM_PARALLEL_DIM = 30
    PM_PARALLEL_DEGREE = 31
    PM_PAD = 32


LAYER_GUID_FIRST_VALID = 1000000
OP_GUID_FIRST_VALID = 2000000
TENSOR_GUID_FIRST_VALID = 3000000
PARALLEL_TENSOR_GUID_FIRST_VALID = 4000000
NODE_GUID_FIRST_VALID = 5000000


def enum_to_int(enum, enum_item):
    for item in enum:
        if enum_item == item:
            return item.value
    raise ValueError(f"unknown enum type {enum_item} {enum}")


def int_to_enum(enum, value):
    for item in enum:
        if item.value == value:
            return item
    raise ValueError(f"unknown enum value {value} {enum}")


def enum_to_str(enum, enum_item):
    return enum(enum_item).name


def str_to_enum(enum, value):
    for item in enum:
        if item.name == value:
            return item
    raise ValueError(f"unknown enum value {value} {enum}")


def dtype_size(dt: DataType) -> int:
    return {DataType.DT_BOOLEAN: 1, DataType.DT_INT32: 4, DataType.DT_INT64: 8, DataType.DT_HALF: 2,
            DataType.DT_FLOAT: 4, DataType.DT_DOUBLE: 8, DataType.DT_BF16: 2}.get(dt, 4)
