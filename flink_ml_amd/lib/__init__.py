"""Algorithm modules laid out like the reference Python API (``pyflink.ml.lib.<group>.<algo>``),
so ``from flink_ml_amd.lib.classification.logisticregression import LogisticRegression`` mirrors
``from pyflink.ml.lib.classification.logisticregression import LogisticRegression``."""
