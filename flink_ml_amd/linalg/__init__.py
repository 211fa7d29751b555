from .vectors import (  # noqa: F401
    DenseMatrix,
    DenseVector,
    SparseVector,
    Vector,
    Vectors,
    VectorWithNorm,
    as_vector,
    stack_dense,
)
from . import blas as BLAS  # noqa: F401
