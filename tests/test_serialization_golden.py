"""Golden byte layouts of the model-data serializers, derived by hand from the reference's Java
serializer code (no serialized model ships with the reference, so these hex strings pin the
format instead):
  DenseVectorSerializer.java:78-93   int32 n, then n big-endian f64 (Bits.putDouble)
  SparseVectorSerializer.java:77-90  int32 size, int32 nnz, then (int32 index, f64 value) pairs
  VectorSerializer.java:80-88        byte tag (0 dense, 1 sparse) + the vector
  DenseMatrixSerializer.java:76-86   int32 rows, int32 cols, column-major f64
  Flink MapSerializer                int32 size, then key, bool isNull, value (if not null)
  Flink StringSerializer             StringValue.writeString: varint (length + 1), then the
                                     chars as varints (0 = null)."""
from flink_ml_amd.io import serialization as ser
from flink_ml_amd.linalg import DenseMatrix, Vectors

ONE, MINUS_2_5, HALF, TWO = "3ff0000000000000", "c004000000000000", "3fe0000000000000", "4000000000000000"


def _hex(fn, *args) -> str:
    out = ser.DataOutput()
    fn(out, *args)
    return out.getvalue().hex()


def test_dense_vector_golden():
    h = _hex(ser.write_dense_vector, Vectors.dense(1.0, -2.5))
    assert h == "00000002" + ONE + MINUS_2_5
    assert ser.read_dense_vector(ser.DataInput(bytes.fromhex(h))).values.tolist() == [1.0, -2.5]


def test_sparse_vector_golden():
    h = _hex(ser.write_sparse_vector, Vectors.sparse(5, [1, 3], [0.5, 2.0]))
    assert h == "00000005" + "00000002" + "00000001" + HALF + "00000003" + TWO
    v = ser.read_sparse_vector(ser.DataInput(bytes.fromhex(h)))
    assert v.size() == 5 and list(v.indices) == [1, 3] and list(v.values) == [0.5, 2.0]


def test_tagged_vector_golden():
    assert _hex(ser.write_vector, Vectors.dense(1.0)) == "00" + "00000001" + ONE
    assert _hex(ser.write_vector, Vectors.sparse(2, [0], [2.0])) == "01" + "00000002" + "00000001" + "00000000" + TWO


def test_dense_matrix_golden():
    m = DenseMatrix(2, 2, [1.0, 2.0, 3.0, 4.0])  # column-major values, as the reference stores them
    h = _hex(ser.write_dense_matrix, m)
    assert h == "00000002" + "00000002" + ONE + TWO + "4008000000000000" + "4010000000000000"


def test_map_golden():
    h = _hex(ser.write_map, {1.5: 2.0, 3.0: None}, lambda o, k: o.write_double(k), lambda o, v: o.write_double(v))
    assert h == "00000002" + "3ff8000000000000" + "00" + TWO + "4008000000000000" + "01"
    m = ser.read_map(ser.DataInput(bytes.fromhex(h)), lambda i: i.read_double(), lambda i: i.read_double())
    assert m == {1.5: 2.0, 3.0: None}


def test_string_golden():
    assert _hex(ser.DataOutput.write_string, "ab") == "036162"
    assert _hex(ser.DataOutput.write_string, None) == "00"
    # a char >= 0x80 is a varint of 7-bit groups, low group first, high bit = more
    assert _hex(ser.DataOutput.write_string, "é") == "02" + "e901"
