"""Window descriptors (reference ``flink-ml-core/.../common/window/*.java``).

In the engine a window is a rule for cutting a (possibly unbounded) input into bounded
chunks that an AlgoOperator processes independently (``DataStreamUtils.windowAllAndProcess``,
``common/datastream/DataStreamUtils.java:262-303``). ``GlobalWindows`` = the whole bounded
input; ``CountTumblingWindows(n)`` = consecutive n-row chunks (the trailing partial chunk is
dropped, matching Flink's count trigger); time windows cut on a timestamp column.
"""
from __future__ import annotations

_JPKG = "org.apache.flink.ml.common.window."


class Windows:
    java_class = None

    def to_json(self):
        return {"class": _JPKG + type(self).__name__}

    @staticmethod
    def from_json(obj):
        cls = obj["class"].rsplit(".", 1)[-1]
        if cls == "GlobalWindows":
            return GlobalWindows.get_instance()
        if cls == "CountTumblingWindows":
            return CountTumblingWindows.of(int(obj["size"]))
        if cls == "ProcessingTimeTumblingWindows":
            return ProcessingTimeTumblingWindows.of(int(obj["size"]))
        if cls == "EventTimeTumblingWindows":
            return EventTimeTumblingWindows.of(int(obj["size"]))
        if cls == "ProcessingTimeSessionWindows":
            return ProcessingTimeSessionWindows.with_gap(int(obj["gap"]))
        if cls == "EventTimeSessionWindows":
            return EventTimeSessionWindows.with_gap(int(obj["gap"]))
        raise ValueError("Unsupported Windows subclass: %s" % obj["class"])

    def __eq__(self, other):
        return type(self) is type(other) and self.__dict__ == other.__dict__

    def __hash__(self):
        return hash((type(self).__name__, tuple(sorted(self.__dict__.items()))))

    def __repr__(self):
        return "%s(%s)" % (type(self).__name__, ", ".join("%s=%s" % kv for kv in self.__dict__.items()))


class GlobalWindows(Windows):
    _INSTANCE = None

    @classmethod
    def get_instance(cls):
        if cls._INSTANCE is None:
            cls._INSTANCE = GlobalWindows()
        return cls._INSTANCE

    getInstance = get_instance


class CountTumblingWindows(Windows):
    def __init__(self, size: int):
        self.size = int(size)

    @staticmethod
    def of(size: int):
        return CountTumblingWindows(size)


class _TimeTumbling(Windows):
    def __init__(self, size_ms: int):
        self.size = int(size_ms)

    @classmethod
    def of(cls, size_ms: int):
        return cls(size_ms)

    def to_json(self):
        d = super().to_json()
        d["size"] = self.size
        return d


class _TimeSession(Windows):
    def __init__(self, gap_ms: int):
        self.gap = int(gap_ms)

    @classmethod
    def with_gap(cls, gap_ms: int):
        return cls(gap_ms)

    withGap = with_gap

    def to_json(self):
        d = super().to_json()
        d["gap"] = self.gap
        return d


class ProcessingTimeTumblingWindows(_TimeTumbling):
    pass


class EventTimeTumblingWindows(_TimeTumbling):
    pass


class ProcessingTimeSessionWindows(_TimeSession):
    pass


class EventTimeSessionWindows(_TimeSession):
    pass


def _count_to_json(self):
    d = Windows.to_json(self)
    d["size"] = self.size
    return d


CountTumblingWindows.to_json = _count_to_json


class EndOfStreamWindows(Windows):
    """A single window covering the whole bounded input, fired at end of input
    (``CORE/common/datastream/EndOfStreamWindows.java:36-74``). For the bounded partitions
    processed here it cuts the same single chunk as ``GlobalWindows``."""

    _INSTANCE = None

    @classmethod
    def get(cls):
        if cls._INSTANCE is None:
            cls._INSTANCE = EndOfStreamWindows()
        return cls._INSTANCE

