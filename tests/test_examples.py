"""Runs every script under examples/ (the analogue of the reference's python ExamplesTest, which
executes each pyflink example end to end) and checks that it prints results."""
import contextlib
import glob
import io
import os
import runpy

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXAMPLES = sorted(glob.glob(os.path.join(ROOT, "examples", "**", "*_example.py"), recursive=True))


def test_examples_cover_every_stage_group():
    groups = {os.path.basename(os.path.dirname(p)) for p in EXAMPLES}
    assert {"classification", "clustering", "evaluation", "feature", "regression", "stats"} <= groups
    assert len(EXAMPLES) >= 45


@pytest.mark.parametrize("path", EXAMPLES, ids=[os.path.relpath(p, ROOT) for p in EXAMPLES])
def test_example_runs(path):
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        runpy.run_path(path, run_name="__main__")
    out = buf.getvalue()
    assert out.strip(), "example printed nothing"
    assert "nan" not in out.lower() or "imputer" in path  # the imputer example prints its NaN inputs
