"""DAG of stages: GraphBuilder / Graph / GraphModel.

Reference: ``flink-ml-core/.../builder/{GraphBuilder,Graph,GraphModel,GraphNode,GraphData,
GraphExecutionHelper,TableId}.java``. Nodes execute in ready order (a node is ready once all
its input tables exist, ``GraphExecutionHelper.java:74-127``); per node the executor runs
``fit`` (estimators, when fitting) → ``set_model_data`` → ``transform`` → ``get_model_data``
(``Graph.java:93-127``). Saved as ``metadata`` with a ``graphData`` map plus one stage
directory per node id, exactly like the reference.
"""
from __future__ import annotations

from collections import deque
from typing import Dict, List, Optional, Sequence

from ..io import read_write as rw
from ..table import Table
from .stage import AlgoOperator, Estimator, Model, Stage

ESTIMATOR = "ESTIMATOR"
ALGO_OPERATOR = "ALGO_OPERATOR"


class TableId:
    __slots__ = ("id",)

    def __init__(self, id: int):
        self.id = int(id)

    def __eq__(self, other):
        return isinstance(other, TableId) and other.id == self.id

    def __hash__(self):
        return hash(self.id)

    def __repr__(self):
        return "TableId(%d)" % self.id

    @staticmethod
    def to_list(ids):
        return [t.id for t in ids]

    @staticmethod
    def from_list(lst):
        return [TableId(i) for i in lst]


class GraphNode:
    def __init__(self, node_id: int, stage: Optional[Stage], stage_type: str,
                 estimator_input_ids, algo_op_input_ids, output_ids,
                 input_model_data_ids=None, output_model_data_ids=None):
        self.node_id = node_id
        self.stage = stage
        self.stage_type = stage_type
        self.estimator_input_ids = estimator_input_ids
        self.algo_op_input_ids = algo_op_input_ids
        self.output_ids = output_ids
        self.input_model_data_ids = input_model_data_ids
        self.output_model_data_ids = output_model_data_ids

    def to_map(self):
        m = {"nodeId": self.node_id, "stageType": self.stage_type,
             "algoOpInputIds": TableId.to_list(self.algo_op_input_ids),
             "outputIds": TableId.to_list(self.output_ids)}
        if self.estimator_input_ids is not None:
            m["estimatorInputIds"] = TableId.to_list(self.estimator_input_ids)
        if self.input_model_data_ids is not None:
            m["inputModelDataIds"] = TableId.to_list(self.input_model_data_ids)
        if self.output_model_data_ids is not None:
            m["outputModelDataIds"] = TableId.to_list(self.output_model_data_ids)
        return m

    @staticmethod
    def from_map(m):
        g = lambda k: TableId.from_list(m[k]) if k in m else None  # noqa: E731
        return GraphNode(int(m["nodeId"]), None, m["stageType"], g("estimatorInputIds"),
                         TableId.from_list(m["algoOpInputIds"]), TableId.from_list(m["outputIds"]),
                         g("inputModelDataIds"), g("outputModelDataIds"))


class GraphData:
    def __init__(self, nodes, estimator_input_ids, model_input_ids, output_ids,
                 input_model_data_ids, output_model_data_ids):
        self.nodes = nodes
        self.estimator_input_ids = estimator_input_ids
        self.model_input_ids = model_input_ids
        self.output_ids = output_ids
        self.input_model_data_ids = input_model_data_ids
        self.output_model_data_ids = output_model_data_ids

    def to_map(self):
        m = {"nodes": [n.to_map() for n in self.nodes],
             "modelInputIds": TableId.to_list(self.model_input_ids),
             "outputIds": TableId.to_list(self.output_ids)}
        if self.estimator_input_ids is not None:
            m["estimatorInputIds"] = TableId.to_list(self.estimator_input_ids)
        if self.input_model_data_ids is not None:
            m["inputModelDataIds"] = TableId.to_list(self.input_model_data_ids)
        if self.output_model_data_ids is not None:
            m["outputModelDataIds"] = TableId.to_list(self.output_model_data_ids)
        return m

    @staticmethod
    def from_map(m):
        g = lambda k: TableId.from_list(m[k]) if k in m else None  # noqa: E731
        return GraphData([GraphNode.from_map(x) for x in m["nodes"]], g("estimatorInputIds"),
                         TableId.from_list(m["modelInputIds"]), TableId.from_list(m["outputIds"]),
                         g("inputModelDataIds"), g("outputModelDataIds"))


class _ExecutionHelper:
    def __init__(self, nodes: Sequence[GraphNode]):
        self.tables: Dict[TableId, Table] = {}
        self.consumers: Dict[TableId, List[GraphNode]] = {}
        self.pending: Dict[int, int] = {}
        self.ready: deque = deque()
        self.nodes = {n.node_id: n for n in nodes}
        for n in nodes:
            inputs = set(n.algo_op_input_ids)
            if n.stage_type == ESTIMATOR and n.estimator_input_ids is not None:
                inputs |= set(n.estimator_input_ids)
            if n.input_model_data_ids is not None:
                inputs |= set(n.input_model_data_ids)
            for t in inputs:
                self.consumers.setdefault(t, []).append(n)
            self.pending[n.node_id] = len(inputs)
            if not inputs:
                self.ready.append(n)
                del self.pending[n.node_id]

    def set_tables(self, ids, tables):
        if len(ids) < len(tables):
            raise ValueError("the length of tablesIds %d is less than the length of tables %d" % (len(ids), len(tables)))
        for tid, t in zip(ids, tables):
            if tid in self.tables:
                raise ValueError("the table with id=%s has already been constructed" % tid)
            self.tables[tid] = t
            for n in self.consumers.get(tid, []):
                c = self.pending.get(n.node_id)
                if c is None:
                    continue
                if c == 1:
                    self.ready.append(n)
                    del self.pending[n.node_id]
                else:
                    self.pending[n.node_id] = c - 1

    def get_tables(self, ids):
        out = []
        for t in ids:
            if t not in self.tables:
                raise ValueError("the table with id=%s has not been constructed yet" % t)
            out.append(self.tables[t])
        return out

    def poll(self) -> Optional[GraphNode]:
        if not self.ready and self.pending:
            raise RuntimeError("there exists node whose input can not be constructed")
        return self.ready.popleft() if self.ready else None


def _run_node(helper: _ExecutionHelper, node: GraphNode, fit_estimators: bool):
    stage = node.stage
    if node.stage_type == ESTIMATOR and fit_estimators:
        stage = stage.fit(*helper.get_tables(node.estimator_input_ids))
    elif node.stage_type == ESTIMATOR:
        stage = stage.fit(*helper.get_tables(node.estimator_input_ids))
    if node.input_model_data_ids is not None:
        stage.set_model_data(*helper.get_tables(node.input_model_data_ids))
    outs = stage.transform(*helper.get_tables(node.algo_op_input_ids))
    helper.set_tables(node.output_ids, outs)
    if node.output_model_data_ids is not None:
        helper.set_tables(node.output_model_data_ids, stage.get_model_data())
    return stage


def _save_graph(stage, data: GraphData, path: str):
    rw.save_metadata(stage, path, {"graphData": data.to_map()})
    max_id = max((n.node_id for n in data.nodes), default=-1)
    for n in data.nodes:
        n.stage.save(rw.stage_path(path, n.node_id, max_id + 1))


def _load_graph_data(path: str, expected: str) -> GraphData:
    meta = rw.load_metadata(path, expected)
    data = GraphData.from_map(meta["graphData"])
    max_id = max((n.node_id for n in data.nodes), default=-1)
    for n in data.nodes:
        n.stage = rw.load_stage(rw.stage_path(path, n.node_id, max_id + 1))
    return data


@rw.register_stage
class GraphModel(Model):
    JAVA_CLASS_NAME = "org.apache.flink.ml.builder.GraphModel"

    def __init__(self, nodes=(), input_ids=(), output_ids=(), input_model_data_ids=None,
                 output_model_data_ids=None):
        super().__init__()
        self.nodes = list(nodes)
        self.input_ids = list(input_ids)
        self.output_ids = list(output_ids)
        self.input_model_data_ids = input_model_data_ids
        self.output_model_data_ids = output_model_data_ids
        self._helper = _ExecutionHelper(self.nodes)

    def transform(self, *inputs: Table) -> List[Table]:
        if len(inputs) != len(self.input_ids):
            raise ValueError("number of provided tables %d does not match the expected number of tables %d"
                             % (len(inputs), len(self.input_ids)))
        helper = self._helper
        helper.set_tables(self.input_ids, inputs)
        while True:
            node = helper.poll()
            if node is None:
                break
            _run_node(helper, node, fit_estimators=False)
        out = helper.get_tables(self.output_ids)
        self._last_helper = helper
        self._helper = _ExecutionHelper(self.nodes)
        if self.input_model_data_ids is not None and hasattr(self, "_model_data_tables"):
            self._helper.set_tables(self.input_model_data_ids, self._model_data_tables)
        return out

    def set_model_data(self, *inputs: Table):
        if self.input_model_data_ids is None:
            raise ValueError("setModelData() is not supported")
        self._model_data_tables = list(inputs)
        self._helper.set_tables(self.input_model_data_ids, inputs)
        return self

    def get_model_data(self) -> List[Table]:
        if self.output_model_data_ids is None:
            raise ValueError("getModelData() is not supported")
        return getattr(self, "_last_helper", self._helper).get_tables(self.output_model_data_ids)

    def save(self, path: str) -> None:
        _save_graph(self, GraphData(self.nodes, None, self.input_ids, self.output_ids,
                                    self.input_model_data_ids, self.output_model_data_ids), path)

    @classmethod
    def load(cls, path: str) -> "GraphModel":
        d = _load_graph_data(path, cls.JAVA_CLASS_NAME)
        return GraphModel(d.nodes, d.model_input_ids, d.output_ids, d.input_model_data_ids, d.output_model_data_ids)


@rw.register_stage
class Graph(Estimator):
    JAVA_CLASS_NAME = "org.apache.flink.ml.builder.Graph"

    def __init__(self, nodes=(), estimator_input_ids=(), model_input_ids=(), output_ids=(),
                 input_model_data_ids=None, output_model_data_ids=None):
        super().__init__()
        self.nodes = list(nodes)
        self.estimator_input_ids = list(estimator_input_ids)
        self.model_input_ids = list(model_input_ids)
        self.output_ids = list(output_ids)
        self.input_model_data_ids = input_model_data_ids
        self.output_model_data_ids = output_model_data_ids

    def fit(self, *inputs: Table) -> GraphModel:
        if len(inputs) != len(self.estimator_input_ids):
            raise ValueError("number of provided tables %d does not match the expected number of tables %d"
                             % (len(inputs), len(self.estimator_input_ids)))
        helper = _ExecutionHelper(self.nodes)
        helper.set_tables(self.estimator_input_ids, inputs)
        model_nodes = []
        while True:
            node = helper.poll()
            if node is None:
                break
            stage = _run_node(helper, node, fit_estimators=True)
            model_nodes.append(GraphNode(node.node_id, stage, ALGO_OPERATOR, None, node.algo_op_input_ids,
                                         node.output_ids, node.input_model_data_ids, node.output_model_data_ids))
        return GraphModel(model_nodes, self.model_input_ids, self.output_ids, self.input_model_data_ids,
                          self.output_model_data_ids)

    def save(self, path: str) -> None:
        _save_graph(self, GraphData(self.nodes, self.estimator_input_ids, self.model_input_ids, self.output_ids,
                                    self.input_model_data_ids, self.output_model_data_ids), path)

    @classmethod
    def load(cls, path: str) -> "Graph":
        d = _load_graph_data(path, cls.JAVA_CLASS_NAME)
        return Graph(d.nodes, d.estimator_input_ids, d.model_input_ids, d.output_ids, d.input_model_data_ids,
                     d.output_model_data_ids)


class GraphBuilder:
    """Builds Graph / GraphModel / AlgoOperator DAGs (``builder/GraphBuilder.java:40-434``)."""

    def __init__(self):
        self.max_output_length = 20
        self.next_table_id = 0
        self.next_node_id = 0
        self.nodes: List[GraphNode] = []
        self.existing: Dict[int, GraphNode] = {}

    def set_max_output_table_num(self, n: int) -> "GraphBuilder":
        self.max_output_length = n
        return self

    def create_table_id(self) -> TableId:
        t = TableId(self.next_table_id)
        self.next_table_id += 1
        return t

    def _ids(self, n):
        return [self.create_table_id() for _ in range(n)]

    def _add(self, stage, stype, est_inputs, model_inputs):
        if id(stage) in self.existing:
            raise RuntimeError("The stage %s has already been added." % stage)
        outs = self._ids(self.max_output_length)
        node = GraphNode(self.next_node_id, stage, stype, est_inputs, list(model_inputs), outs)
        self.next_node_id += 1
        self.nodes.append(node)
        self.existing[id(stage)] = node
        return outs

    def add_algo_operator(self, algo_op: AlgoOperator, *inputs: TableId) -> List[TableId]:
        return self._add(algo_op, ALGO_OPERATOR, None, inputs)

    def add_estimator(self, estimator: Estimator, *inputs, model_inputs=None) -> List[TableId]:
        if len(inputs) == 2 and isinstance(inputs[0], (list, tuple)):
            est_in, mod_in = list(inputs[0]), list(inputs[1])
        else:
            est_in = list(inputs)
            mod_in = list(model_inputs) if model_inputs is not None else list(inputs)
        return self._add(estimator, ESTIMATOR, est_in, mod_in)

    def _node(self, stage, stype, what):
        node = self.existing.get(id(stage))
        if node is None:
            raise RuntimeError("the %s has not been added to the graph" % what)
        if node.stage_type != stype:
            raise RuntimeError("the %s was previously added as %s" % (what, node.stage_type))
        return node

    def set_model_data_on_estimator(self, estimator, *inputs):
        node = self._node(estimator, ESTIMATOR, "Estimator")
        if node.input_model_data_ids is not None:
            raise RuntimeError("the model data of this Estimator has already been set")
        node.input_model_data_ids = list(inputs)

    def set_model_data_on_model(self, model, *inputs):
        node = self._node(model, ALGO_OPERATOR, "Model")
        if node.input_model_data_ids is not None:
            raise RuntimeError("the model data of this Model has already been set")
        node.input_model_data_ids = list(inputs)

    def get_model_data_from_estimator(self, estimator) -> List[TableId]:
        node = self._node(estimator, ESTIMATOR, "Estimator")
        if node.output_model_data_ids is not None:
            raise RuntimeError("the model data of this Estimator has already been fetched")
        node.output_model_data_ids = self._ids(self.max_output_length)
        return node.output_model_data_ids

    def get_model_data_from_model(self, model) -> List[TableId]:
        node = self._node(model, ALGO_OPERATOR, "Model")
        if node.output_model_data_ids is not None:
            raise RuntimeError("the model data of this Model has already been fetched")
        node.output_model_data_ids = self._ids(self.max_output_length)
        return node.output_model_data_ids

    def build_estimator(self, inputs, outputs, input_model_data=None, output_model_data=None,
                        model_inputs=None) -> Graph:
        return Graph(self.nodes, list(inputs), list(model_inputs if model_inputs is not None else inputs),
                     list(outputs), input_model_data, output_model_data)

    def build_algo_operator(self, inputs, outputs) -> GraphModel:
        return self.build_model(inputs, outputs)

    def build_model(self, inputs, outputs, input_model_data=None, output_model_data=None) -> GraphModel:
        return GraphModel(self.nodes, list(inputs), list(outputs), input_model_data, output_model_data)
