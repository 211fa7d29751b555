"""Shared machinery for Models that carry model data.

A Model's model data is exposed as a ``Table`` (``get_model_data()``/``set_model_data()``,
reference ``api/Model.java:38,48``) whose rows are model-data *records*; ``save()`` writes
those records with the reference's binary encoder into ``<path>/data`` so the files are
interchangeable. Subclasses define:

* ``MODEL_DATA_COLUMNS`` — column names of the model-data table;
* ``encode_record(out, row)`` / ``decode_record(inp) -> row`` — the binary codec;
* optionally ``_on_model_data()`` to build device-resident state (cached per table).
"""
from __future__ import annotations

from typing import List, Sequence

from ..api.stage import Model
from ..io import read_write as rw
from ..table import Table


class ModelWithData(Model):
    MODEL_DATA_COLUMNS: Sequence[str] = ()

    def __init__(self):
        super().__init__()
        self._md_table: Table = None
        self._md_cache = None

    # -- model data ----------------------------------------------------------------------------
    def set_model_data(self, *inputs: Table):
        self._md_table = inputs[0]
        self._md_cache = None
        return self

    def get_model_data(self) -> List[Table]:
        if self._md_table is not None:
            self._md_table.replicated = True  # every rank holds the full model data
        return [self._md_table]

    def model_data_rows(self) -> List[tuple]:
        if self._md_table is None:
            raise RuntimeError("Model data of %s is not set" % type(self).__name__)
        return self._md_table.rows()

    def _model_state(self):
        """Lazily-built (device) state derived from the model-data table."""
        if self._md_cache is None:
            self._md_cache = self._build_state(self.model_data_rows())
        return self._md_cache

    def _build_state(self, rows):  # pragma: no cover - overridden
        return rows

    @classmethod
    def make_model_data_table(cls, rows: Sequence[tuple]) -> Table:
        return Table.from_rows(rows, list(cls.MODEL_DATA_COLUMNS))

    # -- persistence ---------------------------------------------------------------------------
    @staticmethod
    def encode_record(out, row):  # pragma: no cover - overridden
        raise NotImplementedError

    @staticmethod
    def decode_record(inp):  # pragma: no cover - overridden
        raise NotImplementedError

    def save(self, path: str) -> None:
        rw.save_metadata(self, path)
        rw.save_model_data(path, self.model_data_rows(), type(self).encode_record)

    @classmethod
    def load(cls, path: str):
        model = rw.load_stage_param(path)
        rows = rw.load_model_data(path, cls.decode_record)
        model.set_model_data(cls.make_model_data_table(rows))
        return model
