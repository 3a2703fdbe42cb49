"""Compat shim: reference import path ``fedml_api/utils/main_flops_counter.py`` -> ``neuroimagedisttraining_amd.utils.flops``."""
from neuroimagedisttraining_amd.utils.flops import (  # noqa: F401
    count_inference_flops, count_model_param_flops, count_training_flops, print_model_param_nums)
