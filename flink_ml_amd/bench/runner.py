"""Benchmark runner (reference ``flink-ml-benchmark/.../Benchmark.java`` + ``BenchmarkUtils.java``).

Reads a JSON v1 config (``"version": 1`` plus named benchmarks of ``stage`` / ``inputData`` /
optional ``modelData``, each a ``className`` + ``paramMap``; ``//`` comment lines allowed) and, for
every benchmark, on every rank:

1. instantiates the stage and generators (unknown params fail like the reference);
2. times — between barrier + device synchronisation on both sides, max over ranks — the data
   generation plus ``fit(...).get_model_data()`` for Estimators or ``transform(...)`` for
   AlgoOperators (the reference's ``netRuntime`` also covers its source operators);
3. reports ``totalTimeMs, inputRecordNum, inputThroughput, outputRecordNum, outputThroughput``
   (+ ``stageTimeMs``/``generateTimeMs`` splits), or ``{"exception": ...}`` on failure.

Results are written (rank 0) in the reference's result-file shape: the config entry plus a
``results`` object, keyed by benchmark name.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
import traceback
from typing import Dict, Optional

import torch

from .. import config
from ..api.stage import AlgoOperator, Estimator, Model
from ..io import read_write as rw
from ..parallel import comm
from ..parallel.context import get_context, init_distributed
from . import generators  # noqa: F401  (registers the generator classes)


def load_config(path: str) -> Dict:
    with open(path, encoding="utf-8") as f:
        text = "\n".join(l for l in f.read().split("\n") if not l.strip().startswith("//"))
    conf = json.loads(text)
    if conf.get("version") != 1:
        raise ValueError("Unsupported benchmark config version %s" % conf.get("version"))
    return conf


def _sync():
    if torch.cuda.is_available() and config.compute_device().type == "cuda":
        torch.cuda.synchronize()
    if get_context().is_distributed:
        comm.barrier()


def _count_rows(tables) -> int:
    """Rows the reference's counting sink would see: partitioned tables are summed over ranks,
    replicated ones (model data, statistics) counted once."""
    ctx = get_context()
    part = sum(int(t.num_rows) for t in tables if t is not None and not t.replicated)
    rep = sum(int(t.num_rows) for t in tables if t is not None and t.replicated)
    if ctx.is_distributed:
        part = int(comm.all_reduce_scalar(float(part), "sum"))
    return part + rep


def run_benchmark(name: str, spec: Dict) -> Dict:
    stage = rw.instantiate_with_params(spec["stage"])
    in_gen = rw.instantiate_with_params(spec["inputData"])
    md_gen = rw.instantiate_with_params(spec["modelData"]) if "modelData" in spec else None
    _sync()
    t0 = time.perf_counter()
    inputs = in_gen.get_data()
    if md_gen is not None:
        if not isinstance(stage, Model):
            raise ValueError("modelData given for a non-Model stage %s" % type(stage).__name__)
        stage.set_model_data(*md_gen.get_data())
    _sync()
    t1 = time.perf_counter()
    if isinstance(stage, Estimator):
        outputs = stage.fit(*inputs).get_model_data()
    elif isinstance(stage, AlgoOperator):
        outputs = stage.transform(*inputs)
    else:
        raise ValueError("Unsupported Stage class %s" % type(stage).__name__)
    _sync()
    t2 = time.perf_counter()
    times = torch.tensor([t2 - t0, t1 - t0, t2 - t1], dtype=torch.float64)
    if get_context().is_distributed:
        times = comm.all_reduce(times, "max")
    total_ms, gen_ms, stage_ms = (float(x) * 1000.0 for x in times)
    n_in = int(in_gen.get(in_gen.NUM_VALUES))
    n_out = _count_rows(outputs)
    return {"totalTimeMs": total_ms, "inputRecordNum": n_in, "inputThroughput": n_in * 1000.0 / total_ms,
            "outputRecordNum": n_out, "outputThroughput": n_out * 1000.0 / total_ms, "generateTimeMs": gen_ms,
            "stageTimeMs": stage_ms, "stageInputThroughput": n_in * 1000.0 / stage_ms if stage_ms > 0 else None}


def _cap_values(spec: Dict, max_values: Optional[int]) -> Dict:
    """A copy of ``spec`` whose inputData.numValues is at most ``max_values`` (reduced runs of
    the host-bound string stages; the result records the configured size it stands for)."""
    if not max_values:
        return spec
    spec = json.loads(json.dumps(spec))
    pm = spec.get("inputData", {}).setdefault("paramMap", {})
    if int(pm.get("numValues", 0)) > max_values:
        spec["configuredNumValues"] = int(pm["numValues"])
        pm["numValues"] = int(max_values)
    return spec


def run_config(conf: Dict, pattern: Optional[str] = None, verbose: bool = True, warmup: int = 0,
               max_values: Optional[int] = None) -> Dict:
    import re

    out = {}
    rx = re.compile(pattern) if pattern else None
    for name, spec in conf.items():
        if name == "version" or (rx and not rx.match(name)):
            continue
        spec = _cap_values(spec, max_values)
        entry = dict(spec)
        if verbose and get_context().rank == 0:
            print("running %s ..." % name, flush=True)
        try:
            for _ in range(warmup):  # untimed: first-touch costs (library handles, allocator, caches)
                run_benchmark(name, spec)
            entry["results"] = run_benchmark(name, spec)
        except Exception as e:  # noqa: BLE001 - recorded like the reference's exception results
            entry["results"] = {"exception": "%s: %s" % (type(e).__name__, e)}
            if verbose and get_context().rank == 0:
                traceback.print_exc()
        out[name] = entry
        if verbose and get_context().rank == 0:
            print("%s: %s" % (name, json.dumps(entry["results"])), flush=True)
    return out


def warm_runtime() -> None:
    """Process start-up kept outside every benchmark's clock, as the reference's cluster start-up
    is outside its jobs' net runtime (BenchmarkUtils.java:131): the stage modules (a fresh tree
    byte-compiles ~1,600 functions on import: 1.3 s spread over the first configs that import
    them), the device context and the kernel library with all its code objects (ops/native.py)."""
    import flink_ml_amd.models  # noqa: F401  (every stage class and its helpers)

    if torch.cuda.is_available() and config.compute_device().type == "cuda":
        from ..ops import native

        native.kernels()
        torch.cuda.synchronize()


def main(argv=None):
    ap = argparse.ArgumentParser(description="Runs the benchmarks of a JSON v1 config file.")
    ap.add_argument("config", help="Benchmark JSON config")
    ap.add_argument("--output-file", help="Where to write the results JSON")
    ap.add_argument("--pattern", help="Regex of benchmark names to run", default=None)
    ap.add_argument("--warmup", type=int, default=0, help="untimed runs of each benchmark before the timed one")
    ap.add_argument("--max-values", type=int, default=None,
                    help="cap inputData.numValues (reduced run; results keep configuredNumValues)")
    args = ap.parse_args(argv)
    if "RANK" in os.environ and "WORLD_SIZE" in os.environ and int(os.environ["WORLD_SIZE"]) > 1:
        init_distributed()
    warm_runtime()
    res = run_config(load_config(args.config), args.pattern, warmup=args.warmup, max_values=args.max_values)
    if get_context().rank == 0 and args.output_file:
        with open(args.output_file, "w", encoding="utf-8") as f:
            json.dump(res, f, indent=2)
    return 0


if __name__ == "__main__":
    sys.exit(main())
