"""ZeRO tuning spaces per stage (reference `autotuning/config_templates/template_zero{0..3}.json`), sized for
MI355X: RCCL rings over xGMI are per-link bound, so buckets stay large (>= 200 MB) and the stage-3 prefetch / live
parameter budgets are scaled to 288 GB of HBM. A user `autotuning.tuning_space` overrides these."""

DEFAULT_TUNING_SPACE = {
    0: {"zero_optimization": {"stage": 0}},
    1: {"zero_optimization": {"stage": 1, "reduce_bucket_size": [2e8, 5e8, 1e9], "overlap_comm": [True, False]}},
    2: {"zero_optimization": {"stage": 2, "reduce_bucket_size": [2e8, 5e8, 1e9], "allgather_bucket_size": [5e8, 1e9],
                              "overlap_comm": [True, False], "contiguous_gradients": [True]}},
    3: {"zero_optimization": {"stage": 3, "reduce_bucket_size": [2e8, 5e8, 1e9],
                              "stage3_prefetch_bucket_size": [2e8, 5e8, 1e9],
                              "stage3_max_live_parameters": [1e9, 4e9],
                              "stage3_param_persistence_threshold": [1e5, 1e6], "overlap_comm": [True]}},
}
