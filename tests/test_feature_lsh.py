"""MinHashLSH against LIBT/feature/MinHashLSHTest.java expectations (signatures for seed 2022,
nearest neighbours, similarity join), plus the MinHash HIP kernel vs the exact int64 path."""
import numpy as np
import pytest
import torch

from flink_ml_amd import Table, Vectors
from flink_ml_amd.models import MinHashLSH, MinHashLSHModel
from flink_ml_amd.models.feature.lsh import generate_model_data
from flink_ml_amd.ops import lsh as lsh_ops
from flink_ml_amd.table import SparseColumn
from flink_ml_amd.utils.java import java_string_hash
from tests.spmd import run_spmd

EXPECTED_5x3 = [
    [[1.73046954E8, 1.57275425E8, 6.90717571E8], [5.02301169E8, 7.967141E8, 4.06089319E8],
     [2.83652171E8, 1.97714719E8, 6.04731316E8], [5.2181506E8, 6.36933726E8, 6.13894128E8],
     [3.04301769E8, 1.113672955E9, 6.1388711E8]],
    [[1.73046954E8, 1.57275425E8, 6.7798584E7], [6.38582806E8, 1.78703694E8, 4.06089319E8],
     [6.232638E8, 9.28867E7, 9.92010642E8], [2.461064E8, 1.12787481E8, 1.92180297E8],
     [2.38162496E8, 1.552933319E9, 2.77995137E8]],
    [[1.73046954E8, 1.57275425E8, 6.90717571E8], [1.453197722E9, 7.967141E8, 4.06089319E8],
     [6.232638E8, 1.97714719E8, 6.04731316E8], [2.461064E8, 1.12787481E8, 1.92180297E8],
     [1.224130231E9, 1.113672955E9, 2.77995137E8]]]
EXPECTED_5x1 = [[[1.73046954E8], [1.57275425E8], [6.7798584E7], [6.38582806E8], [1.78703694E8]],
                [[1.73046954E8], [1.57275425E8], [6.90717571E8], [5.02301169E8], [7.967141E8]],
                [[1.73046954E8], [1.57275425E8], [6.90717571E8], [1.453197722E9], [7.967141E8]]]


def _input():
    return Table.from_rows([(0, Vectors.sparse(6, [0, 1, 2], [1., 1., 1.])), (1, Vectors.sparse(6, [2, 3, 4], [1., 1., 1.])),
                            (2, Vectors.sparse(6, [0, 2, 4], [1., 1., 1.]))], ["id", "vec"])


def _sig_set(out):
    return sorted(tuple(tuple(v.values.tolist()) for v in row) for row in out.get_list("hashes"))


def _exp_set(exp):
    return sorted(tuple(tuple(v) for v in row) for row in exp)


def _lsh(tables=5, funcs=3):
    return MinHashLSH().set_input_col("vec").set_output_col("hashes").set_seed(2022).set_num_hash_tables(tables) \
        .set_num_hash_functions_per_table(funcs)


def test_hash_function():
    md = MinHashLSHModel().set_model_data(MinHashLSHModel.make_model_data_table([(3, 1, [0, 1, 3], [1, 2, 0])]))
    x = SparseColumn.from_vectors([Vectors.sparse(10, [2, 3, 5, 7], [1.] * 4)], 10)
    np.testing.assert_array_equal(md.hash_function(x)[0].reshape(-1).numpy(), [1., 5., 9.])
    md2 = MinHashLSHModel().set_model_data(MinHashLSHModel.make_model_data_table([generate_model_data(3, 1, 10, 2022)]))
    dense = torch.tensor([[0, 0, 1, 1, 0, 1, 0, 1, 0, 0]], dtype=torch.float64)
    assert torch.equal(md2.hash_function(dense), md2.hash_function(x))
    with pytest.raises(ValueError, match="non zero"):
        md.hash_function(SparseColumn.from_vectors([Vectors.sparse(10, [], [])], 10))


def test_params():
    lsh = MinHashLSH()
    assert lsh.get_input_col() == "input" and lsh.get_output_col() == "output"
    assert lsh.get_seed() == java_string_hash("org.apache.flink.ml.feature.lsh.MinHashLSH")
    assert lsh.get_num_hash_tables() == 1 and lsh.get_num_hash_functions_per_table() == 1


def test_fit_transform_save_load(tmp_path):
    lsh = _lsh()
    p = str(tmp_path / "lsh")
    lsh.save(p)
    model = MinHashLSH.load(p).fit(_input())
    md = model.get_model_data()[0]
    assert md.column_names == ["numHashTables", "numHashFunctionsPerTable", "randCoefficientA", "randCoefficientB"]
    nt, nf, a, b = md.rows()[0]
    assert (nt, nf, len(a), len(b)) == (5, 3, 15, 15)
    assert _sig_set(model.transform(_input())[0]) == _exp_set(EXPECTED_5x3)
    pm = str(tmp_path / "lshm")
    model.save(pm)
    assert _sig_set(MinHashLSHModel.load(pm).transform(_input())[0]) == _exp_set(EXPECTED_5x3)
    m2 = MinHashLSHModel().set_model_data(md).set_input_col("vec").set_output_col("hashes")
    assert _sig_set(m2.transform(_input())[0]) == _exp_set(EXPECTED_5x3)
    assert _sig_set(_lsh(5, 1).fit(_input()).transform(_input())[0]) == _exp_set(EXPECTED_5x1)


def test_nearest_neighbors_and_join():
    model = _lsh(5, 1).fit(_input())
    nn = model.approx_nearest_neighbors(_input(), Vectors.sparse(6, [1, 3], [1.0, 1.0]), 2).select("id", "distCol")
    assert sorted(nn.rows()) == [(0, 0.75), (1, 0.75)]
    tb = Table.from_rows([(3, Vectors.sparse(6, [1, 3, 5], [1., 1., 1.])), (4, Vectors.sparse(6, [2, 3, 5], [1., 1., 1.])),
                          (5, Vectors.sparse(6, [1, 2, 4], [1., 1., 1.]))], ["id", "vec"])
    join = model.approx_similarity_join(_input(), tb, 0.6, "id")
    assert join.column_names == ["datasetA.id", "datasetB.id", "distCol"]
    assert sorted(join.rows()) == [(0, 5, 0.5), (1, 4, 0.5), (1, 5, 0.5), (2, 5, 0.5)]


def _spmd_lsh(rank, world):
    model = _lsh(5, 1).fit(_input().partition(rank, world))
    nn = model.approx_nearest_neighbors(_input().partition(rank, world), Vectors.sparse(6, [1, 3], [1.0, 1.0]), 2)
    tb = Table.from_rows([(3, Vectors.sparse(6, [1, 3, 5], [1., 1., 1.])), (4, Vectors.sparse(6, [2, 3, 5], [1., 1., 1.])),
                          (5, Vectors.sparse(6, [1, 2, 4], [1., 1., 1.]))], ["id", "vec"])
    join = model.approx_similarity_join(_input().partition(rank, world), tb.partition(rank, world), 0.6, "id")
    return nn.select("id", "distCol").rows(), join.rows()


def test_lsh_distributed():
    res = run_spmd(_spmd_lsh, 2)
    assert sorted(r for nn, _ in res for r in nn) == [(0, 0.75), (1, 0.75)]
    assert sorted(r for _, j in res for r in j) == [(0, 5, 0.5), (1, 4, 0.5), (1, 5, 0.5), (2, 5, 0.5)]


@pytest.mark.gpu
def test_minhash_kernel_matches_exact():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    rng = np.random.default_rng(5)
    n, d = 20000, 5000
    rows = [np.sort(rng.choice(d, size=rng.integers(1, 60), replace=False)) for _ in range(n)]
    sc = SparseColumn.from_vectors([Vectors.sparse(d, r.tolist(), [1.0] * len(r)) for r in rows], d)
    _, _, a, b = generate_model_data(8, 4, d, 7)
    cpu = lsh_ops.minhash(sc, a, b)
    gpu = lsh_ops.minhash(sc.to("cuda"), a, b)
    assert gpu.is_cuda
    assert torch.equal(gpu.cpu(), cpu)


def _rand_sets(seed, n, d=60):
    rng = np.random.default_rng(seed)
    rows = []
    for i in range(n):
        k = int(rng.integers(1, 8))
        cols = np.sort(rng.choice(d, size=k, replace=False)).tolist()
        rows.append((i + 1000 * seed, Vectors.sparse(d, cols, [1.0] * k)))
    return Table.from_rows(rows, ["id", "vec"])


def _spmd_keyed_join(rank, world):
    a, b = _rand_sets(1, 900), _rand_sets(2, 700)
    model = _lsh(4, 2).fit(a)
    join = model.approx_similarity_join(a.partition(rank, world), b.partition(rank, world), 0.7, "id")
    return join.rows()


def test_lsh_keyed_similarity_join_matches_one_rank():
    """Distributed approxSimilarityJoin (keyed join: signatures to key owners, pairs to A's rank,
    B sets fetched on demand) equals the single-rank join on random sets."""
    a, b = _rand_sets(1, 900), _rand_sets(2, 700)
    ref = sorted(_lsh(4, 2).fit(a).approx_similarity_join(a, b, 0.7, "id").rows())
    assert len(ref) > 50
    got = sorted(r for part in run_spmd(_spmd_keyed_join, 3) for r in part)
    assert got == ref


def _str_sets(seed, n):
    t = _rand_sets(seed, n)
    return Table.from_rows([("s%d" % i, v) for i, v in t.rows()], ["id", "vec"])


def _spmd_mixed_join(rank, world):
    """Rank 0 holds empty partitions (whose ids vote "numeric"), rank 1 all rows with string ids:
    the ranks must agree on the broadcast join, not split between two collective sequences."""
    a, b = _str_sets(1, 300), _str_sets(2, 200)
    model = _lsh(4, 2).fit(a)
    if rank == 0:
        a, b = a.take([]), b.take([])
    return model.approx_similarity_join(a, b, 0.7, "id").rows()


def test_lsh_join_agrees_on_branch_with_empty_partition():
    a, b = _str_sets(1, 300), _str_sets(2, 200)
    ref = sorted(_lsh(4, 2).fit(a).approx_similarity_join(a, b, 0.7, "id").rows())
    assert len(ref) > 10
    part = run_spmd(_spmd_mixed_join, 2)
    assert part[0] == []
    assert sorted(part[1]) == ref


def _big_ids(seed, n):
    t = _rand_sets(seed, n)
    return Table.from_rows([((1 << 60) + 2 * i + 1, v) for i, v in t.rows()], ["id", "vec"])


def _spmd_big_id_join(rank, world):
    a, b = _big_ids(1, 400), _big_ids(2, 300)
    model = _lsh(4, 2).fit(a)
    return model.approx_similarity_join(a.partition(rank, world), b.partition(rank, world), 0.7, "id").rows()


def test_lsh_keyed_join_keeps_int64_ids_above_2p53():
    a, b = _big_ids(1, 400), _big_ids(2, 300)
    ref = sorted(_lsh(4, 2).fit(a).approx_similarity_join(a, b, 0.7, "id").rows())
    assert len(ref) > 10
    got = sorted(r for part in run_spmd(_spmd_big_id_join, 2) for r in part)
    assert got == ref
    assert all(isinstance(r[1], int) and r[1] > (1 << 53) for r in got)
