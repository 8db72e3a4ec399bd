"""Checkpoint key names. These strings ARE the on-disk schema shared with the reference
(deepspeed/checkpoint/constants.py), so they must match it byte for byte."""

# optimizer-file keys
OPTIMIZER_STATE_DICT = "optimizer_state_dict"
ZERO_STAGE = "zero_stage"
PARTITION_COUNT = "partition_count"
LOSS_SCALER = "loss_scaler"
CLIP_GRAD = "clip_grad"
PARAM_GROUPS = "param_groups"
# ZeRO-1/2
BASE_OPTIMIZER_STATE = "base_optimizer_state"
SINGLE_PARTITION_OF_FP32_GROUPS = "single_partition_of_fp32_groups"
GROUP_PADDINGS = "group_paddings"
PARAM_SLICE_MAPPINGS = "param_slice_mappings"
# ZeRO-3
FP32_FLAT_GROUPS = "fp32_flat_groups"

# model-file keys
PARAM_SHAPES = "param_shapes"
BUFFER_NAMES = "buffer_names"
FROZEN_PARAM_SHAPES = "frozen_param_shapes"
FROZEN_PARAM_FRAGMENTS = "frozen_param_fragments"
DS_VERSION = "ds_version"

# universal checkpoint
FP32_WEIGHT_KEY = "fp32"
PARAM = "param"
CAT_DIM = "cat_dim"
VOCAB_TENSOR = "vocab_tensor"
PARAM_N_SUB_PARAMS = "param_n_sub_params"
SUB_PARAM_SHAPE = "sub_param_shape"
UNIVERSAL_CHECKPOINT_INFO = "universal_checkpoint_info"
UNIVERSAL_CHECKPOINT_VERSION_KEY = "universal_checkpoint_version"
UNIVERSAL_CHECKPOINT_VERSION_VALUE = 0.2
ORIGINAL_VOCAB_SIZE = "original_vocab_size"
TP_REPLICATED_PARAMETER_PATTERNS = "tp_replicated_parameter_patterns"
PARAMETER_TO_AVERAGE_PATTERNS = "parameter_to_average_patterns"
PARAMETER_WITH_ROW_PARALLELISM_PATTERNS = "parameter_with_row_parallelism_patterns"
VOCABULARY_PARAMETER_PATTERNS = "vocabulary_parameter_patterns"
PIPELINE_REPLICATED_PARAMETER_PATTERNS = "pipeline_replicated_parameter_patterns"
PARAMETER_WITH_2_SUB_PARAMS_CAT_DIM_0 = "parameter_with_2_sub_params_cat_dim_0"
PARAMETER_WITH_SUB_PARAMS = "parameter_with_sub_params"

# file-name pieces
MODEL_FILE_PREFIX = "mp_rank_"
ZERO_FILE_PREFIX = "zero_pp_rank_"
OPTIM_FILE_SUFFIX = "_optim_states.pt"
MODEL_FILE_SUFFIX = "_model_states.pt"
