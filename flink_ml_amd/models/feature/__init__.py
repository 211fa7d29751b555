"""Feature engineering stages (reference flink-ml-lib ``org.apache.flink.ml.feature``)."""
from . import scalers, text, vector_ops  # noqa: F401
from .scalers import (MaxAbsScaler, MaxAbsScalerModel, MinMaxScaler, MinMaxScalerModel,  # noqa: F401
                      RobustScaler, RobustScalerModel, StandardScaler, StandardScalerModel,
                      VarianceThresholdSelector, VarianceThresholdSelectorModel)
from .text import (IDF, CountVectorizer, CountVectorizerModel, FeatureHasher, HashingTF,  # noqa: F401
                   IDFModel, NGram, RegexTokenizer, StopWordsRemover, Tokenizer)
from .vector_ops import (DCT, Binarizer, Bucketizer, ElementwiseProduct, Interaction,  # noqa: F401
                         Normalizer, PolynomialExpansion, VectorAssembler, VectorSlicer)
from . import encoders  # noqa: F401,E402
from .encoders import (Imputer, ImputerModel, IndexToStringModel, KBinsDiscretizer,  # noqa: F401,E402
                       KBinsDiscretizerModel, OneHotEncoder, OneHotEncoderModel, StringIndexer, StringIndexerModel,
                       VectorIndexer, VectorIndexerModel)
from . import selectors  # noqa: F401,E402
from .selectors import UnivariateFeatureSelector, UnivariateFeatureSelectorModel  # noqa: F401,E402
from . import lsh  # noqa: F401,E402
from .lsh import MinHashLSH, MinHashLSHModel  # noqa: F401,E402
from . import misc  # noqa: F401,E402
from .misc import RandomSplitter, SQLTransformer  # noqa: F401,E402
