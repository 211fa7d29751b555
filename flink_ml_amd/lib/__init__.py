"""Algorithm modules laid out like the reference Python API (``pyflink.ml.lib.<group>.<algo>``),
so ``from flink_ml_amd.lib.classification.logisticregression import LogisticRegression`` mirrors
``from pyflink.ml.lib.classification.logisticregression import LogisticRegression``.

The layout is a table, not a tree of files: a meta-path finder materialises
``flink_ml_amd.lib.<group>`` and ``flink_ml_amd.lib.<group>.<algo>`` on import, each exposing the
stage classes (from ``flink_ml_amd.models``) that the reference module of the same path defines.
The reference's other Python module paths are aliases of the modules that implement them here
(``ALIASES``: ``core.api`` → ``api.stage``, ``core.builder`` → ``api.pipeline``, ``core.linalg``,
``core.param``, ``core.windows``, ``lib.functions``, ``lib.param``, ``util.read_write_utils``).
"""
from __future__ import annotations

import importlib
import importlib.abc
import importlib.machinery
import sys
import types

# group -> module -> stage classes (reference pyflink/ml/lib/<group>/<module>.py)
LAYOUT = {
    "classification": {
        "knn": ("KNN", "KNNModel"),
        "linearsvc": ("LinearSVC", "LinearSVCModel"),
        "logisticregression": ("LogisticRegression", "LogisticRegressionModel", "OnlineLogisticRegression", "OnlineLogisticRegressionModel"),
        "naivebayes": ("NaiveBayes", "NaiveBayesModel"),
    },
    "clustering": {
        "agglomerativeclustering": ("AgglomerativeClustering",),
        "kmeans": ("KMeans", "KMeansModel", "OnlineKMeans", "OnlineKMeansModel"),
    },
    "evaluation": {
        "binaryclassificationevaluator": ("BinaryClassificationEvaluator",),
    },
    "feature": {
        "binarizer": ("Binarizer",),
        "bucketizer": ("Bucketizer",),
        "countvectorizer": ("CountVectorizer", "CountVectorizerModel"),
        "dct": ("DCT",),
        "elementwiseproduct": ("ElementwiseProduct",),
        "featurehasher": ("FeatureHasher",),
        "hashingtf": ("HashingTF",),
        "idf": ("IDF", "IDFModel"),
        "imputer": ("Imputer", "ImputerModel"),
        "interaction": ("Interaction",),
        "kbinsdiscretizer": ("KBinsDiscretizer", "KBinsDiscretizerModel"),
        "lsh": ("MinHashLSH", "MinHashLSHModel"),
        "maxabsscaler": ("MaxAbsScaler", "MaxAbsScalerModel"),
        "minmaxscaler": ("MinMaxScaler", "MinMaxScalerModel"),
        "ngram": ("NGram",),
        "normalizer": ("Normalizer",),
        "onehotencoder": ("OneHotEncoder", "OneHotEncoderModel"),
        "polynomialexpansion": ("PolynomialExpansion",),
        "randomsplitter": ("RandomSplitter",),
        "regextokenizer": ("RegexTokenizer",),
        "robustscaler": ("RobustScaler", "RobustScalerModel"),
        "sqltransformer": ("SQLTransformer",),
        "standardscaler": ("StandardScaler", "StandardScalerModel"),
        "stopwordsremover": ("StopWordsRemover",),
        "stringindexer": ("StringIndexer", "StringIndexerModel", "IndexToStringModel"),
        "tokenizer": ("Tokenizer",),
        "univariatefeatureselector": ("UnivariateFeatureSelector", "UnivariateFeatureSelectorModel"),
        "variancethresholdselector": ("VarianceThresholdSelector", "VarianceThresholdSelectorModel"),
        "vectorassembler": ("VectorAssembler",),
        "vectorindexer": ("VectorIndexer", "VectorIndexerModel"),
        "vectorslicer": ("VectorSlicer",),
    },
    "regression": {
        "linearregression": ("LinearRegression", "LinearRegressionModel"),
    },
    "stats": {
        "anovatest": ("ANOVATest",),
        "chisqtest": ("ChiSqTest",),
        "fvaluetest": ("FValueTest",),
    },
}


# reference module path (pyflink.ml.<path>) -> implementing module here
ALIASES = {
    "flink_ml_amd.core.api": "flink_ml_amd.api.stage",
    "flink_ml_amd.core.builder": "flink_ml_amd.api.pipeline",
    "flink_ml_amd.core.linalg": "flink_ml_amd.linalg.vectors",
    "flink_ml_amd.core.param": "flink_ml_amd.param.param",
    "flink_ml_amd.core.windows": "flink_ml_amd.common.window",
    "flink_ml_amd.lib.functions": "flink_ml_amd.functions",
    "flink_ml_amd.lib.param": "flink_ml_amd.common.param",
    "flink_ml_amd.util.read_write_utils": "flink_ml_amd.io.read_write",
}
_ALIAS_PACKAGES = {"flink_ml_amd.core", "flink_ml_amd.util"}


class _AliasLoader(importlib.abc.Loader):
    _specs = {}

    def create_module(self, spec):
        if spec.name in ALIASES:
            mod = importlib.import_module(ALIASES[spec.name])
            self._specs[id(mod)] = mod.__spec__  # the import machinery overwrites __spec__
            return mod
        return types.ModuleType(spec.name)

    def exec_module(self, module):
        if id(module) in self._specs:
            module.__spec__ = self._specs.pop(id(module))
            return
        if module.__name__ in _ALIAS_PACKAGES:
            module.__path__ = []
            module.__all__ = sorted(k.rsplit(".", 1)[1] for k in ALIASES if k.startswith(module.__name__ + "."))


class _Loader(importlib.abc.Loader):
    def create_module(self, spec):
        return types.ModuleType(spec.name)

    def exec_module(self, module):
        parts = module.__name__.split(".")[2:]  # flink_ml_amd.lib.<group>[.<algo>]
        models = importlib.import_module("flink_ml_amd.models")
        if len(parts) == 1:
            # a package: its algorithm modules resolve through the finder, and every stage class
            # of the group is also importable from it (``from ...lib.feature import Binarizer``)
            module.__path__ = []
            names = [n for m in sorted(LAYOUT[parts[0]]) for n in LAYOUT[parts[0]][m]]
            for n in names:
                setattr(module, n, getattr(models, n))
            module.__all__ = sorted(LAYOUT[parts[0]]) + names
            module.__doc__ = "``%s`` stages (reference ``pyflink.ml.lib.%s``)." % (parts[0], parts[0])
            return
        names = LAYOUT[parts[0]][parts[1]]
        for n in names:
            setattr(module, n, getattr(models, n))
        module.__all__ = list(names)
        module.__doc__ = "``%s.%s`` stages." % (parts[0], parts[1])


class _Finder(importlib.abc.MetaPathFinder):
    _loader = _Loader()
    _alias_loader = _AliasLoader()

    def find_spec(self, fullname, path=None, target=None):
        if fullname in ALIASES or fullname in _ALIAS_PACKAGES:
            return importlib.machinery.ModuleSpec(fullname, self._alias_loader,
                                                  is_package=fullname in _ALIAS_PACKAGES)
        parts = fullname.split(".")
        if parts[:2] != ["flink_ml_amd", "lib"] or len(parts) not in (3, 4):
            return None
        if parts[2] not in LAYOUT or (len(parts) == 4 and parts[3] not in LAYOUT[parts[2]]):
            return None
        return importlib.machinery.ModuleSpec(fullname, self._loader, is_package=len(parts) == 3)


if not any(isinstance(f, _Finder) for f in sys.meta_path):
    sys.meta_path.insert(0, _Finder())

__all__ = sorted(LAYOUT)
