"""Scatter plot of benchmark results (reference ``benchmark-results-visualize.py``):
``python -m flink_ml_amd.bench.visualize results.json --pattern '^KMeansModel.*$' --output plot.png``."""
from __future__ import annotations

import argparse
import json
import re


def nested(obj, dotted: str):
    for k in dotted.split("."):
        obj = obj[k]
    return obj


def collect(file_name: str, pattern: str, x_field: str, y_field: str):
    rx = re.compile(pattern)
    xs, ys = [], []
    with open(file_name, encoding="utf-8") as f:
        for name, entry in json.load(f).items():
            if not rx.match(name):
                continue
            try:
                xs.append(nested(entry, x_field))
                ys.append(nested(entry, y_field))
            except (KeyError, TypeError):
                continue
    return xs, ys


def main(argv=None):
    ap = argparse.ArgumentParser(description="Visualizes benchmark results.")
    ap.add_argument("file_name")
    ap.add_argument("--pattern", default=".*")
    ap.add_argument("--x-field", default="inputData.paramMap.numValues")
    ap.add_argument("--y-field", default="results.inputThroughput")
    ap.add_argument("--output", default=None, help="image file (shown interactively if omitted)")
    args = ap.parse_args(argv)
    xs, ys = collect(args.file_name, args.pattern, args.x_field, args.y_field)
    import matplotlib

    if args.output:
        matplotlib.use("Agg")
    import matplotlib.pyplot as plt

    plt.scatter(xs, ys)
    plt.xlabel(args.x_field)
    plt.ylabel(args.y_field)
    plt.title("flink-ml-amd Benchmark Results")
    if args.output:
        plt.savefig(args.output)
    else:
        plt.show()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
