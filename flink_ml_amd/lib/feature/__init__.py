"""``feature`` stages (reference ``pyflink.ml.lib.feature``)."""
from .binarizer import Binarizer  # noqa: F401
from .bucketizer import Bucketizer  # noqa: F401
from .countvectorizer import CountVectorizer, CountVectorizerModel  # noqa: F401
from .dct import DCT  # noqa: F401
from .elementwiseproduct import ElementwiseProduct  # noqa: F401
from .featurehasher import FeatureHasher  # noqa: F401
from .hashingtf import HashingTF  # noqa: F401
from .idf import IDF, IDFModel  # noqa: F401
from .imputer import Imputer, ImputerModel  # noqa: F401
from .interaction import Interaction  # noqa: F401
from .kbinsdiscretizer import KBinsDiscretizer, KBinsDiscretizerModel  # noqa: F401
from .lsh import MinHashLSH, MinHashLSHModel  # noqa: F401
from .maxabsscaler import MaxAbsScaler, MaxAbsScalerModel  # noqa: F401
from .minmaxscaler import MinMaxScaler, MinMaxScalerModel  # noqa: F401
from .ngram import NGram  # noqa: F401
from .normalizer import Normalizer  # noqa: F401
from .onehotencoder import OneHotEncoder, OneHotEncoderModel  # noqa: F401
from .polynomialexpansion import PolynomialExpansion  # noqa: F401
from .randomsplitter import RandomSplitter  # noqa: F401
from .regextokenizer import RegexTokenizer  # noqa: F401
from .robustscaler import RobustScaler, RobustScalerModel  # noqa: F401
from .sqltransformer import SQLTransformer  # noqa: F401
from .standardscaler import StandardScaler, StandardScalerModel  # noqa: F401
from .stopwordsremover import StopWordsRemover  # noqa: F401
from .stringindexer import StringIndexer, StringIndexerModel, IndexToStringModel  # noqa: F401
from .tokenizer import Tokenizer  # noqa: F401
from .univariatefeatureselector import UnivariateFeatureSelector, UnivariateFeatureSelectorModel  # noqa: F401
from .variancethresholdselector import VarianceThresholdSelector, VarianceThresholdSelectorModel  # noqa: F401
from .vectorassembler import VectorAssembler  # noqa: F401
from .vectorindexer import VectorIndexer, VectorIndexerModel  # noqa: F401
from .vectorslicer import VectorSlicer  # noqa: F401
