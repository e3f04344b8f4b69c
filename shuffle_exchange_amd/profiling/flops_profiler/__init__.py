from .profiler import FlopsProfiler, get_model_profile  # noqa: F401
