from .train_utils import (SnakeActivation, compute_downsample_rate, freeze,
                          linear_warmup_cosine_annealingLR, load_yaml_param_settings, quantize,
                          remove_outliers, set_seed, time_to_timefreq, timefreq_to_time, unfreeze,
                          zero_pad_high_freq, zero_pad_low_freq)

__all__ = [
    "SnakeActivation", "compute_downsample_rate", "freeze", "linear_warmup_cosine_annealingLR",
    "load_yaml_param_settings", "quantize", "remove_outliers", "set_seed", "time_to_timefreq", "timefreq_to_time",
    "unfreeze", "zero_pad_high_freq", "zero_pad_low_freq",
]
