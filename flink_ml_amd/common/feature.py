"""``LabeledPointWithWeight`` (reference ``CORE/common/feature/LabeledPointWithWeight.java:24``).

The reference converts every training Row into this object before SGD (features are a
DenseVector there). The engine trains on columnar device tensors, so this class is the row-level
view used at API boundaries (``to_table`` / ``from_table``), not the training representation.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Iterable, List

from ..linalg.vectors import DenseVector, Vector


@dataclass
class LabeledPointWithWeight:
    features: Vector
    label: float
    weight: float = 1.0

    def get_features(self) -> Vector:
        return self.features

    def get_label(self) -> float:
        return self.label

    def get_weight(self) -> float:
        return self.weight

    @staticmethod
    def to_table(points: Iterable["LabeledPointWithWeight"], features_col: str = "features",
                 label_col: str = "label", weight_col: str = "weight"):
        from ..table import Table

        rows = [(p.features, float(p.label), float(p.weight)) for p in points]
        return Table.from_rows(rows, [features_col, label_col, weight_col])

    @staticmethod
    def from_table(table, features_col: str = "features", label_col: str = "label",
                   weight_col: str = None) -> List["LabeledPointWithWeight"]:
        rows = table.rows()
        names = list(table.column_names)
        fi, li = names.index(features_col), names.index(label_col)
        wi = names.index(weight_col) if weight_col else None
        out = []
        for r in rows:
            f = r[fi] if isinstance(r[fi], Vector) else DenseVector(r[fi])
            out.append(LabeledPointWithWeight(f, float(r[li]), float(r[wi]) if wi is not None else 1.0))
        return out
