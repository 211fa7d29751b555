"""Benchmark framework (reference ``flink-ml-benchmark``): JSON v1 configs, bit-exact data
generators, runner and results visualiser. ``python -m flink_ml_amd.bench.run conf.json``."""
from . import generators  # noqa: F401
from .runner import load_config, run_benchmark, run_config  # noqa: F401
