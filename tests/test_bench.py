"""Benchmark framework: bit-exact generators (vs java.util.Random semantics of RowGenerator), the
JSON v1 runner on the reference demo config and the whole reference suite (scaled down), and a
2-rank run."""
import copy
import json
import os

import numpy as np
import pytest
import torch

from flink_ml_amd.bench.generators import (DenseVectorGenerator, DoubleGenerator, KMeansModelDataGenerator,
                                           LabeledPointWithWeightGenerator, RandomStringGenerator, task_rows, task_seed)
from flink_ml_amd.bench.runner import load_config, run_config
from flink_ml_amd.ops.datagen import java_rows
from flink_ml_amd.utils.java import JavaRandom, java_string_hash
from tests.spmd import run_spmd

CONF = os.path.join(os.path.dirname(__file__), "..", "flink_ml_amd", "bench", "conf")


def _java_rows(seed, n, ops):
    r = JavaRandom(seed)
    return np.array([[r.next_double() if o == 0 else float(r.next_int(o)) for o in ops] for _ in range(n)])


def test_task_seed_and_split():
    # Tuple2.of(2L, 0).hashCode() = 31 * Long.hashCode(2) + 0
    assert task_seed(2, 0) == 62 and task_seed(2, 3) == 65
    assert task_seed(-1, 1) == 1  # Long.hashCode(-1) == 0
    assert [task_rows(10, t, 4) for t in range(4)] == [3, 3, 2, 2]


def test_dense_vector_generator_exact():
    g = DenseVectorGenerator().set_seed(2).set_col_names([["features"]]).set_num_values(50).set_vector_dim(7)
    t = g.get_data()[0]
    got = t.column("features").cpu()
    # exact java.util.Random doubles, stored in the column's dtype (the compute dtype on a GPU host)
    ref = torch.from_numpy(_java_rows(task_seed(2, 0), 50, [0] * 7)).to(got.dtype)
    np.testing.assert_array_equal(got.numpy(), ref.numpy())
    assert DenseVectorGenerator().get_seed() == java_string_hash(
        "org.apache.flink.ml.benchmark.datagenerator.common.DenseVectorGenerator")


def test_labeled_point_and_double_generators_exact():
    g = LabeledPointWithWeightGenerator().set_seed(5).set_col_names([["f", "l", "w"]]).set_num_values(40) \
        .set_vector_dim(4).set_feature_arity(20).set_label_arity(10)
    t = g.get_data()[0]
    ref = _java_rows(task_seed(5, 0), 40, [20] * 4 + [10, 0])
    np.testing.assert_array_equal(t.column("f").cpu().numpy(), ref[:, :4])
    np.testing.assert_array_equal(t.column("l").cpu().numpy(), ref[:, 4])
    np.testing.assert_array_equal(t.column("w").cpu().numpy(), ref[:, 5])
    d = DoubleGenerator().set_seed(1).set_col_names([["a", "b"]]).set_num_values(30).set_arity(3).get_data()[0]
    ref = _java_rows(task_seed(1, 0), 30, [3, 3])
    np.testing.assert_array_equal(np.stack([d.column("a").cpu().numpy(), d.column("b").cpu().numpy()], 1), ref)
    s = RandomStringGenerator().set_seed(9).set_col_names([["s"]]).set_num_values(20).set_num_distinct_values(7)
    ref = _java_rows(task_seed(9, 0), 20, [7])
    assert s.get_data()[0].get_list("s") == [str(int(x)) for x in ref[:, 0]]


def test_rejection_replay_is_exact():
    ops = [0, (1 << 30) + 3, 0]
    vec, sc = java_rows(11, 500, ops, 1)
    ref = _java_rows(11, 500, ops)
    np.testing.assert_array_equal(np.concatenate([vec.numpy(), sc.numpy()], 1), ref)


def test_kmeans_model_data_generator():
    md = KMeansModelDataGenerator().set_seed(1).set_array_size(2).set_vector_dim(10).get_data()[0]
    cents, weights = md.rows()[0]
    assert len(cents) == 2 and list(weights.values) == [0.0, 0.0]
    ref = _java_rows(task_seed(1, 0), 1, [0] * 20).reshape(2, 10)
    np.testing.assert_array_equal(np.stack([c.values for c in cents]), ref)


def test_runner_demo(tmp_path):
    conf = load_config(os.path.join(CONF, "demo.json"))
    res = run_config(conf, verbose=False)
    assert set(res) == {k for k in conf if k != "version"}
    r = res["KMeans-1"]["results"]
    assert r["inputRecordNum"] == 10000 and r["outputRecordNum"] == 1
    assert abs(r["inputThroughput"] - 10000 * 1000.0 / r["totalTimeMs"]) < 1e-6
    assert res["KMeansModel-3"]["results"]["outputRecordNum"] == 30000
    assert "exception" in res["Undefined-Parameter"]["results"]
    assert "exception" in res["Unmatch-Input"]["results"]
    from flink_ml_amd.bench.runner import main

    out = tmp_path / "r.json"
    main([os.path.join(CONF, "demo.json"), "--output-file", str(out), "--pattern", "^KMeansModel-1$"])
    saved = json.load(open(out))
    assert list(saved) == ["KMeansModel-1"] and "results" in saved["KMeansModel-1"]


def _small_suite(n=300):
    conf = load_config(os.path.join(CONF, "reference-suite.json"))
    small = {"version": 1}
    for k, v in conf.items():
        if k == "version":
            continue
        v = copy.deepcopy(v)
        v["inputData"]["paramMap"]["numValues"] = min(v["inputData"]["paramMap"].get("numValues", 10), n)
        small[k] = v
    return small


def test_reference_suite_scaled_down():
    res = run_config(_small_suite(), verbose=False)
    failed = {k: v["results"]["exception"] for k, v in res.items() if "exception" in v["results"]}
    assert not failed, failed
    assert len(res) == 35


def _spmd_bench(rank, world):
    conf = load_config(os.path.join(CONF, "demo.json"))
    res = run_config({"version": 1, "KMeans-1": conf["KMeans-1"], "KMeansModel-2": conf["KMeansModel-2"]},
                     verbose=False)
    g = DenseVectorGenerator().set_seed(2).set_col_names([["f"]]).set_num_values(11).set_vector_dim(3)
    return res["KMeans-1"]["results"]["outputRecordNum"], res["KMeansModel-2"]["results"]["outputRecordNum"], \
        g.get_data()[0].column("f").cpu().numpy().tolist()


def test_runner_distributed():
    res = run_spmd(_spmd_bench, 2)
    for i, (a, b, rows) in enumerate(res):
        assert a == 1 and b == 20000
        np.testing.assert_array_equal(np.array(rows), _java_rows(task_seed(2, i), task_rows(11, i, 2), [0] * 3))


@pytest.mark.gpu
@pytest.mark.parametrize("ops,nvec,n", [([0] * 37, 37, 20000), ([20] * 5 + [10, 0], 5, 20000),
                                        ([0, (1 << 30) + 3, 0, 7], 1, 400)])
def test_java_rows_gpu_matches_cpu(ops, nvec, n):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    cv, cs = java_rows(77, n, ops, nvec)
    gv, gs = java_rows(77, n, ops, nvec, device="cuda", vec_dtype=torch.float64)
    assert torch.equal(gv.cpu(), cv) and torch.equal(gs.cpu(), cs)
    g32, _ = java_rows(77, n, ops, nvec, device="cuda", vec_dtype=torch.float32)
    assert torch.equal(g32.cpu(), cv.float())


class _FakeGraph:
    def __init__(self, log, r):
        self.log, self.r = log, r

    def replay(self):
        self.log.append(("replay", self.r))


class _FakeEvent:
    def __init__(self, **kw):
        pass

    def record(self):
        pass

    def elapsed_time(self, other):
        return 1.0


@pytest.mark.parametrize("defer", [False, True])
@pytest.mark.parametrize("steps,warmup,R", [(20, 5, 10), (7, 0, 10), (200, 20, 10), (3, 1, 1), (25, 5, 10), (13, 3, 4)])
def test_bench_timed_region_only_replays(monkeypatch, steps, warmup, R, defer):
    """bench.py: no hipGraph capture may happen between the timing barriers (round-1 driver run
    captured the 10-round graph inside the timed region). Deferred mode: every replay starts at
    the parity its graph was captured for."""
    import bench
    from flink_ml_amd.common.optimizer import DeviceGlmTrainer

    tr = object.__new__(DeviceGlmTrainer)
    tr.use_graph, tr.rounds_per_graph, tr.graphs, tr.timing = True, R, {}, False
    tr.defer, tr.parity = defer, 0
    tr.csc, tr.bkt, tr._launched, tr._short = None, None, 0, False
    log = []

    class Graph(_FakeGraph):
        def __init__(self, log, key):
            super().__init__(log, key[0] if defer else key)
            self.key = key

        def replay(self):
            if defer:
                assert tr.parity == self.key[1], "graph replayed at the wrong round-number parity"
            super().replay()

    def capture(key):
        assert not tr.timing, "hipGraph captured inside the timed region"
        log.append(("capture", key))
        tr.graphs[key] = Graph(log, key)
        return tr.graphs[key]

    def launch(rounds=1):
        assert not tr.timing, "direct launch inside the timed region"
        log.append(("launch", rounds))
        tr.parity = (tr.parity + rounds) & 1

    tr._capture = capture
    tr._launch_round = launch
    monkeypatch.setattr(bench.torch.cuda, "synchronize", lambda *a: None)
    monkeypatch.setattr(bench.torch.cuda, "Event", _FakeEvent)

    class Ctx:
        def barrier(self):
            log.append(("barrier",))

    elapsed, dev_s = bench.timed_region(tr, Ctx(), warmup, steps)
    assert dev_s == 1e-3 and elapsed >= 0
    first_timed = max(i for i, e in enumerate(log) if e == ("barrier",) and i < len(log) - 1) + 1
    timed = [e for e in log[first_timed:] if e != ("barrier",)]
    assert all(e[0] == "replay" for e in timed)
    assert sum(e[1] for e in timed) == steps  # exactly `steps` rounds timed


@pytest.mark.gpu
@pytest.mark.parametrize("bound,k,n", [(1_000_000, 100, 3000), ((1 << 30) + 3, 3, 5000), (100, 10, 20000), (7, 1, 999),
                                       ((1 << 30) + 3, 3, 100_000)])  # (the last: > 65536 rejections, mask path)
def test_java_uniform_int_rows_gpu_matches_sequential(bound, k, n):
    """Every draw nextInt(b) with one non-power-of-two b: the compacted parallel draws equal the
    sequential java.util.Random rejection loop (bound 2^30+3 rejects ~half of all draws)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from flink_ml_amd.ops.datagen import java_uniform_int_rows

    got = java_uniform_int_rows(77, n, k, bound, torch.device("cuda")).cpu().numpy()
    r = JavaRandom(77)
    ref = np.array([[r.next_int(bound) for _ in range(k)] for _ in range(n)], dtype=np.int64)
    np.testing.assert_array_equal(got.astype(np.int64), ref)
    _, cs = java_rows(77, n, [bound] * k, 0, device="cuda")
    np.testing.assert_array_equal(cs.cpu().numpy(), ref.astype(np.float64))


_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench_cmd(*args, env=None, timeout=240):
    import subprocess
    import sys

    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "FMLX_STORE")}
    e.update({"FMLX_DEVICE": "cpu", "OMP_NUM_THREADS": "1"})
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(_ROOT, "bench.py")] + list(args), env=e, cwd=_ROOT,
                          capture_output=True, text=True, timeout=timeout)


def test_bench_check_world():
    import bench

    assert bench.check_world(1, {}) == "run"
    assert bench.check_world(4, {}) == "launch"
    assert bench.check_world(4, {"WORLD_SIZE": "4"}) == "run"
    with pytest.raises(SystemExit):
        bench.check_world(2, {"WORLD_SIZE": "3"})
    with pytest.raises(SystemExit):
        bench.check_world(1, {"WORLD_SIZE": "8"})


def test_bench_gpus_n_launches_n_ranks():
    """`bench.py --gpus 3` with no WORLD_SIZE: the parent starts 3 rank processes that rendezvous
    on its store and form one process group (the reference's benchmark-run.sh runs the job at the
    cluster's parallelism, BenchmarkUtils.java:131-136)."""
    r = _bench_cmd("--gpus", "3", "--dry-run")
    assert r.returncode == 0, r.stderr
    recs = sorted((json.loads(line) for line in r.stdout.splitlines() if line.startswith("{")), key=lambda d: d["rank"])
    assert [d["rank"] for d in recs] == [0, 1, 2]
    assert all(d["world"] == 3 and d["backend"] == "gloo" and d["rank_sum"] == 6.0 for d in recs)


def test_bench_world_mismatch_and_rank_failure_exit_nonzero():
    r = _bench_cmd("--gpus", "2", "--dry-run", env={"WORLD_SIZE": "3", "RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE=3" in r.stderr
    # without --dry-run every CPU rank fails ("needs a GPU"): the launcher reports the failure
    r = _bench_cmd("--gpus", "2", "--steps", "1", "--warmup", "0")
    assert r.returncode != 0 and "needs a GPU" in r.stderr


class _FakeVerifyTrainer:
    """Stands in for DeviceGlmTrainer in bench.verify_exchange: its coefficients after k rounds
    are a fixed function of k (identical on every rank, as a correct exchange gives)."""

    def __init__(self):
        import types

        self.sgd = types.SimpleNamespace(max_iter=0)
        self.use_graph = True
        self.d_model = 6
        self.coef = torch.zeros(8)
        self.rccl = False

    def use_rccl(self):
        self.rccl = True

    def run_rounds(self, k):
        self.coef += torch.arange(8, dtype=torch.float32) * 0.25 * k

    def flush(self):
        pass


def _verify_worker(rank, world, inject):
    import os

    import bench
    from flink_ml_amd.parallel import comm

    if inject is not None:
        os.environ["FMLX_BENCH_INJECT_EXCHANGE_ERROR"] = str(inject)
    ok, info = bench.verify_exchange(_FakeVerifyTrainer, comm)
    return ok, info["replicas_identical"]


@pytest.mark.parametrize("inject", [None, 0, 1])
def test_bench_verify_exchange_detects_a_corrupted_rank(inject):
    """after the timed region bench.py requires the ranks' replicas to agree bitwise and
    the exchange to equal the process-group sum; a corruption on any one rank makes EVERY rank
    report failure (an agreed verdict), so the run exits non-zero instead of printing a number."""
    from tests.spmd import run_spmd

    res = run_spmd(_verify_worker, 2, inject, timeout=120)
    if inject is None:
        assert res == [(True, True), (True, True)]
    else:
        assert [r[0] for r in res] == [False, False] and not res[0][1]
