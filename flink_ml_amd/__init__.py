"""flink_ml_amd — an MI355X-native machine-learning pipeline engine with Flink ML's API.

Layers (re-designed MI355X-first):
  linalg/    host vector types + BLAS            param/   typed params, JSON
  api/       Stage/Estimator/Model/Pipeline/Graph io/     metadata + binary model data
  table      columnar device-resident tables      parallel/ SPMD context, RCCL collectives, iteration
  ops/       HIP (gfx950) kernels + bindings      models/  the algorithm library
  bench/     benchmark CLI + data generators      utils/   Java-compat RNG/hash, tracing
"""
__version__ = "0.1.0"

from .table import SparseColumn, Table  # noqa: F401,E402
from .linalg import DenseMatrix, DenseVector, SparseVector, Vectors  # noqa: F401,E402
from . import lib as _lib  # noqa: F401,E402  (registers the reference module-path layout)
