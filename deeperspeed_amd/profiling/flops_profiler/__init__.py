from .profiler import FlopsProfiler, get_model_profile, num_to_string, macs_to_string, flops_to_string, \
    params_to_string, duration_to_string
