"""AgglomerativeClustering against LIBT/clustering/AgglomerativeClusteringTest.java (merge distances
for every linkage/metric, cluster groups, windows, thresholds) and multi-rank windowAll semantics."""
import numpy as np
import pytest
import torch

from flink_ml_amd import Table, Vectors
from flink_ml_amd.common.window import CountTumblingWindows, EventTimeTumblingWindows, GlobalWindows
from flink_ml_amd.models import AgglomerativeClustering
from tests.spmd import run_spmd

PTS = [(1, 1), (1, 4), (1, 0), (4, 4), (4, 1.5), (4, 0)]
MERGE = {
    ("average", "euclidean"): [1, 1.5, 3, 3.1394402, 3.9559706],
    ("average", "cosine"): [0, 1.1102230E-16, 0.0636708, 0.1425070, 0.3664484],
    ("average", "manhattan"): [1, 1.5, 3, 3.75, 4.875],
    ("single", "euclidean"): [1, 1.5, 2.5, 3, 3],
    ("ward", "euclidean"): [1, 1.5, 3, 4.2573465, 5.5113519],
    ("complete", "euclidean"): [1, 1.5, 3, 3.3541019, 5],
}


def _t():
    return Table.from_rows([(Vectors.dense(*p),) for p in PTS], ["features"])


def _groups(out, pred="prediction"):
    g = {}
    for f, p in zip(out.get_list("features"), out.get_list(pred)):
        g.setdefault(int(p), set()).add(tuple(f.values.tolist()))
    return sorted((frozenset(v) for v in g.values()), key=lambda s: sorted(s))


def _exp(*groups):
    return sorted((frozenset(tuple(float(x) for x in p) for p in g) for g in groups), key=lambda s: sorted(s))


def test_params(tmp_path):
    a = AgglomerativeClustering()
    assert a.get_features_col() == "features" and a.get_num_clusters() == 2 and a.get_distance_threshold() is None
    assert a.get_linkage() == "ward" and a.get_distance_measure() == "euclidean" and a.get_compute_full_tree() is False
    assert a.get_prediction_col() == "prediction" and a.get_windows() == GlobalWindows.get_instance()
    a.set_num_clusters(None).set_distance_threshold(0.01).set_linkage("average").set_distance_measure("cosine")
    p = str(tmp_path / "ac")
    a.save(p)
    b = AgglomerativeClustering.load(p)
    assert b.get_num_clusters() is None and b.get_distance_threshold() == 0.01 and b.get_linkage() == "average"


def test_output_schema_and_validation():
    outs = AgglomerativeClustering().set_prediction_col("p").transform(_t())
    assert len(outs) == 2 and outs[0].column_names == ["features", "p"]
    assert outs[1].column_names == ["clusterId1", "clusterId2", "distance", "sizeOfMergedCluster"]
    with pytest.raises(ValueError, match="should be null"):
        AgglomerativeClustering().set_distance_threshold(1.0).transform(_t())
    with pytest.raises(ValueError, match="Ward only works with euclidean"):
        AgglomerativeClustering().set_distance_measure("cosine").transform(_t())


def test_transform_groups():
    ac = AgglomerativeClustering().set_prediction_col("pred")
    two = _exp([(1, 1), (1, 0), (4, 1.5), (4, 0)], [(1, 4), (4, 4)])
    assert _groups(ac.transform(_t())[0], "pred") == two
    assert _groups(ac.set_compute_full_tree(True).transform(_t())[0], "pred") == two
    thr = _exp([(1, 1), (1, 0)], [(1, 4)], [(4, 4)], [(4, 1.5), (4, 0)])
    assert _groups(ac.set_num_clusters(None).set_distance_threshold(2.0).transform(_t())[0], "pred") == thr
    avg = AgglomerativeClustering().set_linkage("average").set_prediction_col("pred")
    assert _groups(avg.transform(_t())[0], "pred") == two
    big = AgglomerativeClustering().set_num_clusters(None).set_distance_threshold(1.7976931348623157e308)
    assert len(set(big.transform(_t())[0].get_list("prediction"))) == 1


@pytest.mark.parametrize("key", list(MERGE))
def test_merge_info(key):
    link, metric = key
    mi = AgglomerativeClustering().set_linkage(link).set_distance_measure(metric).set_compute_full_tree(True) \
        .transform(_t())[1]
    np.testing.assert_allclose(mi.get_list("distance"), MERGE[key], atol=1e-7)
    assert mi.get_list("sizeOfMergedCluster")[-1] == 6


def test_merge_info_partial_tree():
    mi = AgglomerativeClustering().set_linkage("ward").transform(_t())[1]
    np.testing.assert_allclose(mi.get_list("distance"), MERGE[("ward", "euclidean")][:-1], atol=1e-7)


def test_windows():
    out = AgglomerativeClustering().set_prediction_col("pred").set_windows(CountTumblingWindows.of(5)).transform(_t())[0]
    assert out.num_rows == 5
    assert _groups(out, "pred") == _exp([(1, 1), (1, 0)], [(1, 4), (4, 4), (4, 1.5)])
    ts = torch.tensor([1000.0 * p[0] + 1e9 for p in PTS], dtype=torch.float64)
    t = Table({"features": _t().column("features"), "ts": ts}, num_rows=6).with_time_column("ts")
    out = AgglomerativeClustering().set_prediction_col("pred").set_windows(EventTimeTumblingWindows.of(1000)) \
        .transform(t)[0]
    groups = [set(tuple(f.values.tolist()) for f, p, w in zip(out.get_list("features"), out.get_list("pred"),
                                                               out.get_list("ts")) if p == pid and w == wv)
              for pid in (0, 1) for wv in set(out.get_list("ts"))]
    for exp in ({(1.0, 1.0), (1.0, 0.0)}, {(1.0, 4.0)}, {(4.0, 0.0), (4.0, 1.5)}, {(4.0, 4.0)}):
        assert any(exp <= g for g in groups)


def _spmd_ac(rank, world):
    outs = AgglomerativeClustering().transform(_t().partition(rank, world))
    return [(tuple(f.values.tolist()), p) for f, p in zip(outs[0].get_list("features"), outs[0].get_list("prediction"))], \
        outs[1].num_rows


def test_distributed_window_all():
    res = run_spmd(_spmd_ac, 2)
    rows = [r for part, _ in res for r in part]
    assert len(rows) == 6 and sum(n for _, n in res) == 4
    g = {}
    for f, p in rows:
        g.setdefault(p, set()).add(f)
    assert sorted(map(frozenset, g.values()), key=sorted) == _exp([(1, 1), (1, 0), (4, 1.5), (4, 0)], [(1, 4), (4, 4)])


@pytest.mark.gpu
def test_pairwise_euclid_kernel_matches_torch():
    """csrc/blas.hip pairwise_euclid_f64_kernel against the fp64 torch formula: symmetric, zero
    diagonal, tile edges (n not a multiple of 16, d not a multiple of 16)."""
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from flink_ml_amd.models.agglomerative import condensed_distances, pairwise_distances

    g = torch.Generator().manual_seed(4)
    for n, d in ((1, 3), (17, 5), (1000, 100), (333, 37)):
        X = torch.randn(n, d, generator=g, dtype=torch.float64)
        D = pairwise_distances(X.cuda(), "euclidean").cpu()
        sq = (X * X).sum(1)
        ref = torch.sqrt(torch.clamp(sq[:, None] + sq[None, :] - 2.0 * X @ X.t(), min=0.0))
        # off the diagonal (the torch formula's diagonal is sqrt of a rounding residue, up to ~1e-6;
        # the kernel's is exactly 0, checked below)
        off = ~torch.eye(n, dtype=torch.bool)
        torch.testing.assert_close(D[off], ref[off], rtol=1e-12, atol=1e-9)
        assert torch.equal(D, D.t()) and bool((torch.diagonal(D) == 0).all())
        cond = condensed_distances(X.cuda(), "euclidean")  # the kernel's condensed mode
        np.testing.assert_array_equal(cond, D.numpy()[np.triu_indices(n, 1)])


@pytest.mark.gpu
@pytest.mark.parametrize("key", [k for k in MERGE if k[1] == "euclidean"])
def test_merge_info_gpu(key):
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    link, metric = key
    t = Table({"features": torch.tensor(PTS, dtype=torch.float64).cuda()}, num_rows=len(PTS))
    mi = AgglomerativeClustering().set_linkage(link).set_distance_measure(metric).set_compute_full_tree(True) \
        .transform(t)[1]
    np.testing.assert_allclose(mi.get_list("distance"), MERGE[key], atol=1e-7)
