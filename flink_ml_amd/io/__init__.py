from . import serialization  # noqa: F401
from .read_write import (  # noqa: F401
    all_registered_stages,
    load_metadata,
    load_model_data,
    load_pipeline,
    load_stage,
    load_stage_param,
    lookup_stage_class,
    register_stage,
    save_metadata,
    save_model_data,
    save_pipeline,
)
