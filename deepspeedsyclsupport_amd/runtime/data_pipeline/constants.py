"""Key names of the `data_efficiency` config section and of the curriculum / random-LTD state dicts (reference
`runtime/data_pipeline/constants.py`). One table per constant prefix: NAME suffix -> key string; `...ENABLED` keys
also get an `..._ENABLED_DEFAULT = False`."""

_TABLES = {
    "DATA_EFFICIENCY": ("data_efficiency", {"ENABLED": "enabled", "SEED": "seed"}),
    "DATA_SAMPLING": ("data_sampling", {"ENABLED": "enabled", "NUM_EPOCHS": "num_epochs",
                                        "NUM_WORKERS": "num_workers"}),
    "CURRICULUM_LEARNING": ("curriculum_learning", {
        "ENABLED": "enabled", "CLUSTER_PATH": "data_cluster_path", "METRICS": "curriculum_metrics",
        "SAMPLE_PATH": "index_to_sample_path", "METRIC_PATH": "index_to_metric_path",
        "CLUSTERING_TYPE": "clustering_type", "SINGLE_CLUSTER": "single_cluster", "CLUSTER_PREFIX": "cluster",
        "DIFFICULTY_TYPE": "difficulty_type", "VALUE_BASED": "value", "PERCENTILE_BASED": "percentile",
        "MIN_DIFFICULTY": "min_difficulty", "MAX_DIFFICULTY": "max_difficulty", "SCHEDULE_TYPE": "schedule_type",
        "SCHEDULE_CONFIG": "schedule_config", "SCHEDULE_DIFFICULTY": "difficulty", "SCHEDULE_MAX_STEP": "max_step",
        "SCHEDULE_TOTAL_STEP": "total_curriculum_step", "SCHEDULE_DIFFICULTY_STEP": "difficulty_step",
        "SCHEDULE_ROOT_DEGREE": "root_degree", "SCHEDULE_FIXED_DISCRETE": "fixed_discrete",
        "SCHEDULE_FIXED_ROOT": "fixed_root", "SCHEDULE_FIXED_LINEAR": "fixed_linear", "SCHEDULE_CUSTOM": "custom",
        "CURRENT_DIFFICULTY": "current_difficulty", "BATCH": "batch", "CONSUMED_SAMPLES": "consumed_samples",
        "STEP": "curriculum_step", "CURRENT_DIFFICULTIES": "current_difficulties",
        "DATA_CLUSTER_PATHS": "data_cluster_paths",
        "DATA_CLUSTER_CURRENT_POSITION": "data_cluster_current_position", "NP_RNG_STATE": "np_rng_state"}),
    "DATA_ROUTING": ("data_routing", {"ENABLED": "enabled"}),
    "RANDOM_LTD": ("random_ltd", {
        "ENABLED": "enabled", "MODEL_MASK_NAME": "model_mask_name", "MODEL_TYPE": "model_type",
        "MICRO_BATCH_SIZE": "micro_batch_size", "GLOBAL_BATCH_SIZE": "global_batch_size",
        "SAMPLE_INDEX": "sample_idx", "ATTENTION_MASK": "attention_mask",
        "HIDDEN_STATE_ORDER": "hidden_state_order", "LAYER_NUM": "random_ltd_layer_num",
        "LAYER_ID": "random_ltd_layer_id", "TOTAL_LAYER_NUM": "total_layer_num",
        "CONSUMED_LAYER_TOKENS": "consumed_layer_tokens", "SCHEDULER": "random_ltd_schedule",
        "MAX_VALUE": "max_value", "MIN_VALUE": "min_value", "CURRENT_VALUE": "current_value",
        "SCHEDULE_CONFIG": "schedule_config", "INCREASE_STEP": "seq_per_step", "REQUIRE_STEP": "require_steps",
        "SCHEDULER_TYPE": "schedule_type", "CURR_STEP": "current_steps",
        "LAYER_TOKEN_LR_SCHEDULE": "layer_token_lr_schedule", "LAYER_TOKEN_LR_ENABLED": "enabled",
        "TOTAL_LAYER_TOKENS": "total_layer_tokens", "WARMUP_TYPE": "warmup_type",
        "WARMUP_LAYER_TOKENS": "warmup_layer_tokens"}),
}

for _pre, (_section, _keys) in _TABLES.items():
    globals()[_pre] = _section
    for _name, _key in _keys.items():
        globals()[f"{_pre}_{_name}"] = _key
        if _name.endswith("ENABLED"):
            globals()[f"{_pre}_{_name}_DEFAULT"] = False
del _pre, _section, _keys, _name, _key

DATA_EFFICIENCY_SEED_DEFAULT = 1234
DATA_SAMPLING_NUM_EPOCHS_DEFAULT = 1000
DATA_SAMPLING_NUM_WORKERS_DEFAULT = 0
# the legacy top-level curriculum section
CURRICULUM_LEARNING_LEGACY = "curriculum_learning"
CURRICULUM_ENABLED_LEGACY = "enabled"
CURRICULUM_ENABLED_DEFAULT_LEGACY = False
