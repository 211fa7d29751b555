"""Stage persistence through filesystem URLs (reference ReadWriteUtilsTest.java:48-83 round-trips
through a non-local Flink FileSystem): ``memory://`` and ``file://`` via fsspec, and plain paths."""
import numpy as np
import pytest
import torch

from flink_ml_amd import Table
from flink_ml_amd.api.pipeline import Pipeline
from flink_ml_amd.models import KMeans, LogisticRegression, StandardScaler


def _data():
    rng = np.random.default_rng(0)
    X = rng.normal(size=(200, 4))
    y = (X[:, 0] + X[:, 1] > 0).astype(np.float64)
    return Table({"features": torch.from_numpy(X), "label": torch.from_numpy(y)}, num_rows=200)


@pytest.mark.parametrize("scheme", ["memory", "file", "plain"])
def test_model_save_load_urls(scheme, tmp_path):
    t = _data()
    base = {"memory": "memory://fmlx-test/%s" % tmp_path.name, "file": "file://%s" % tmp_path,
            "plain": str(tmp_path)}[scheme]
    lr = LogisticRegression().set_max_iter(5).fit(t)
    lr.save(base + "/lr")
    got = type(lr).load(base + "/lr")
    a = lr.transform(t)[0].column("prediction")
    b = got.transform(t)[0].column("prediction")
    assert torch.equal(torch.as_tensor(a), torch.as_tensor(b))
    km = KMeans().set_k(3).set_seed(1).fit(t)
    km.save(base + "/km")
    assert torch.equal(torch.as_tensor(km.transform(t)[0].column("prediction")),
                       torch.as_tensor(type(km).load(base + "/km").transform(t)[0].column("prediction")))
    pm = Pipeline([StandardScaler().set_input_col("features").set_output_col("scaled"), KMeans().set_k(2).set_features_col("scaled")]).fit(t)
    pm.save(base + "/pm")
    out1 = pm.transform(t)[0].column("prediction")
    out2 = type(pm).load(base + "/pm").transform(t)[0].column("prediction")
    assert torch.equal(torch.as_tensor(out1), torch.as_tensor(out2))
    with pytest.raises(IOError):
        lr.save(base + "/lr")  # existing metadata is not overwritten
