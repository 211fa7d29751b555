"""Stage persistence (reference ``flink-ml-core/.../util/ReadWriteUtils.java``).

Layout on disk (identical to the reference):

    <path>/metadata                 JSON {className, timestamp, paramMap, ...extra}
    <path>/data/part-<rank>-<n>     model-data records, big-endian Flink encoding
    <path>/stages/<zero-padded i>/  pipeline / pipeline-model members

``className`` is the *Java* class name of the equivalent reference stage, so metadata files
are interchangeable; ``load_stage`` dispatches on it through the stage registry.
Only rank 0 writes (model data is replicated across ranks in this engine).

Paths: plain paths use the local filesystem; a URL (``scheme://...``: ``file://``,
``memory://``, and any remote filesystem fsspec has a driver for — the reference round-trips
through any Flink FileSystem, ``ReadWriteUtilsTest.java:48-83``) goes through fsspec.
"""
from __future__ import annotations

import json
import os
import posixpath
import re
import time
from typing import Any, Callable, Dict, Iterable, List, Optional

from .serialization import DataInput, DataOutput

_REGISTRY: Dict[str, type] = {}


def register_stage(cls: type) -> type:
    """Class decorator: registers a stage under its Java and Python names."""
    java = getattr(cls, "JAVA_CLASS_NAME", None)
    if java:
        _REGISTRY[java] = cls
    _REGISTRY[cls.__module__ + "." + cls.__qualname__] = cls
    _REGISTRY[cls.__name__] = cls
    return cls


def lookup_stage_class(class_name: str) -> type:
    if class_name in _REGISTRY:
        return _REGISTRY[class_name]
    # make sure the whole library is imported (registers every stage)
    import flink_ml_amd.models  # noqa: F401
    if class_name in _REGISTRY:
        return _REGISTRY[class_name]
    short = class_name.rsplit(".", 1)[-1]
    if short in _REGISTRY:
        return _REGISTRY[short]
    raise ValueError("Unknown stage class %s" % class_name)


def all_registered_stages() -> Dict[str, type]:
    import flink_ml_amd.models  # noqa: F401
    return {k: v for k, v in _REGISTRY.items() if k.startswith("org.apache.flink")}


_URL = re.compile(r"^[A-Za-z][A-Za-z0-9+.-]*://")


class _LocalFS:
    join = staticmethod(os.path.join)
    exists = staticmethod(os.path.exists)
    open = staticmethod(open)

    @staticmethod
    def makedirs(p):
        os.makedirs(p, exist_ok=True)

    @staticmethod
    def walk(p):
        return os.walk(p)


class _FsspecFS:
    def __init__(self, path):
        import fsspec

        self.fs, _ = fsspec.core.url_to_fs(path)
        self.proto = path.split("://", 1)[0]

    def _p(self, p):
        return self.fs._strip_protocol(p)

    @staticmethod
    def join(*parts):
        return posixpath.join(*parts)

    def exists(self, p):
        return self.fs.exists(self._p(p))

    def open(self, p, mode="r"):
        return self.fs.open(self._p(p), mode)

    def makedirs(self, p):
        self.fs.makedirs(self._p(p), exist_ok=True)

    def walk(self, p):
        for root, dirs, names in self.fs.walk(self._p(p)):
            yield root, dirs, names


def fs_for(path: str):
    """The filesystem behind ``path``: local for plain paths, fsspec for URLs."""
    return _FsspecFS(path) if _URL.match(str(path)) else _LocalFS


def path_join(path: str, *parts: str) -> str:
    return fs_for(path).join(path, *parts)


def _is_writer() -> bool:
    from ..parallel.context import get_context

    return get_context().rank == 0


def _barrier():
    from ..parallel.context import get_context

    get_context().barrier()


def save_to_file(path: str, content: str, overwrite: bool = False) -> None:
    fs = fs_for(path)
    if not overwrite and fs.exists(path):
        raise IOError("File %s already exists." % path)
    parent = (posixpath.dirname(path) if fs is not _LocalFS else os.path.dirname(path)) or "."
    fs.makedirs(parent)
    with fs.open(path, "w") as f:
        f.write(content)


def param_map_to_json(stage) -> Dict[str, Any]:
    return {p.name: p.json_encode(v) for p, v in stage.get_param_map().items()}


def save_metadata(stage, path: str, extra: Optional[Dict[str, Any]] = None) -> None:
    meta = dict(extra or {})
    meta["className"] = getattr(type(stage), "JAVA_CLASS_NAME", None) or (
        type(stage).__module__ + "." + type(stage).__qualname__)
    meta["timestamp"] = int(time.time() * 1000)
    meta["paramMap"] = param_map_to_json(stage)
    if _is_writer():
        save_to_file(path_join(path, "metadata"), json.dumps(meta), overwrite=False)
    _barrier()


def _strip_comments(text: str) -> str:
    # Jackson ALLOW_COMMENTS: // line and /* block */ comments
    out, i, n = [], 0, len(text)
    in_str = False
    while i < n:
        c = text[i]
        if in_str:
            out.append(c)
            if c == "\\" and i + 1 < n:
                out.append(text[i + 1])
                i += 2
                continue
            if c == '"':
                in_str = False
            i += 1
            continue
        if c == '"':
            in_str = True
            out.append(c)
            i += 1
        elif text.startswith("//", i):
            j = text.find("\n", i)
            i = n if j < 0 else j
        elif text.startswith("/*", i):
            j = text.find("*/", i + 2)
            i = n if j < 0 else j + 2
        else:
            out.append(c)
            i += 1
    return "".join(out)


def loads_json_with_comments(text: str):
    return json.loads(_strip_comments(text))


def load_metadata(path: str, expected_class_name: str = "") -> Dict[str, Any]:
    with fs_for(path).open(path_join(path, "metadata"), "r") as f:
        lines = [l for l in f.read().splitlines() if not l.startswith("#")]
    meta = loads_json_with_comments("".join(lines))
    cls = meta.get("className")
    if expected_class_name and expected_class_name != cls:
        raise RuntimeError("Class name %s does not match the expected class name %s." % (cls, expected_class_name))
    return meta


def instantiate_with_params(meta: Dict[str, Any], strict: bool = True):
    cls = lookup_stage_class(meta["className"])
    stage = cls()
    pm = meta.get("paramMap", {}) or {}
    by_name = {p.name: p for p in stage.get_param_map().keys()}
    for name, value in pm.items():
        p = by_name.get(name)
        if p is None and not strict:
            continue
        if p is None:  # the reference dereferences a null Param here (NPE)
            raise ValueError("Parameter %s is not defined on the class %s" % (name, cls.__name__))
        stage.set(p, p.json_decode(value))
    return stage


def load_stage_param(path: str):
    """Instantiates the stage recorded in ``<path>/metadata`` and restores its params."""
    return instantiate_with_params(load_metadata(path), strict=False)


def load_stage(path: str):
    meta = load_metadata(path)
    cls = lookup_stage_class(meta["className"])
    return cls.load(path)


def stage_path(parent: str, idx: int, num: int) -> str:
    return path_join(parent, "stages", str(idx).zfill(len(str(num))))


def save_pipeline(pipeline, stages: List, path: str) -> None:
    save_metadata(pipeline, path, {"numStages": len(stages)})
    for i, s in enumerate(stages):
        s.save(stage_path(path, i, len(stages)))


def load_pipeline(path: str, expected_class_name: str) -> List:
    meta = load_metadata(path, expected_class_name)
    n = int(meta["numStages"])
    return [load_stage(stage_path(path, i, n)) for i in range(n)]


def data_path(path: str) -> str:
    return path_join(path, "data")


def save_model_data(path: str, records: Iterable[Any], encode: Callable[[DataOutput, Any], None]) -> None:
    """Writes model-data records (one FileSink part file, rank 0 only)."""
    if _is_writer():
        fs = fs_for(path)
        d = data_path(path)
        fs.makedirs(d)
        out = DataOutput()
        for r in records:
            encode(out, r)
        with fs.open(path_join(d, "part-0-0"), "wb") as f:
            f.write(out.getvalue())
    _barrier()


def _data_files(path: str) -> List[str]:
    fs = fs_for(path)
    files = []
    d = data_path(path)
    if fs is not _LocalFS and not fs.exists(d):
        return files
    for root, dirs, names in fs.walk(d):
        if isinstance(dirs, list):
            dirs[:] = sorted(x for x in dirs if not x.startswith((".", "_")))
        for n in sorted(names):
            if not n.startswith((".", "_")):
                files.append(fs.join(root, n) if fs is _LocalFS else "%s://%s" % (fs.proto, posixpath.join(root, n)))
    return sorted(files)


def load_model_data(path: str, decode: Callable[[DataInput], Any]) -> List[Any]:
    """Reads every record of every part file under ``<path>/data`` (FileSource semantics)."""
    out = []
    fs = fs_for(path)
    for fn in _data_files(path):
        with fs.open(fn, "rb") as f:
            inp = DataInput(f.read())
        while not inp.eof():
            out.append(decode(inp))
    return out
