"""Data efficiency pipeline (reference runtime/data_pipeline/)."""
from .curriculum_scheduler import CurriculumScheduler  # noqa: F401
from .data_sampling import CurriculumDataSampler, DataAnalyzer, DistributedDataAnalyzer  # noqa: F401
from .random_ltd import RandomLayerTokenDrop, RandomLTDScheduler, convert_to_random_ltd  # noqa: F401
