"""Configuration: pipeline YAML schema (pipeline.py) and CLI arguments (args.py)."""
from .pipeline import (  # noqa: F401
    C4BadWordsParams,
    C4QualityParams,
    FineWebQualityFilterParams,
    GopherQualityParams,
    GopherRepetitionParams,
    LanguageDetectionParams,
    PipelineConfig,
    StepConfig,
    TokenCounterParams,
    load_pipeline_config,
    load_pipeline_config_str,
)
