"""``stats`` stages (reference ``pyflink.ml.lib.stats``)."""
from .anovatest import ANOVATest  # noqa: F401
from .chisqtest import ChiSqTest  # noqa: F401
from .fvaluetest import FValueTest  # noqa: F401
