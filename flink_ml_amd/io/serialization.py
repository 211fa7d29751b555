"""Big-endian binary codecs compatible with Flink's ``DataOutputView`` serializers.

Model data written by ``save()`` must be byte-identical to the reference's FileSink output
 so a model saved by one framework loads in the other. Covered encodings:

* ``DenseVectorSerializer`` — int32 len + f64[len]  (``linalg/typeinfo/DenseVectorSerializer.java:78-93``)
* ``SparseVectorSerializer`` — int32 n, int32 nnz, (int32 idx, f64 val)*  (``…/SparseVectorSerializer.java:77-90``)
* ``VectorSerializer`` — byte tag 0 dense / 1 sparse + payload  (``…/VectorSerializer.java:80-88``)
* ``DenseMatrixSerializer`` — int32 rows, int32 cols, f64 col-major  (``…/DenseMatrixSerializer.java:76-86``)
* Flink ``StringValue`` strings (varint length+1, varint UTF-16 code units), ``StringArraySerializer``,
  ``MapSerializer`` (int32 size, key, bool isNull, value), primitive-array serializers.
"""
from __future__ import annotations

import io
import struct
from typing import BinaryIO, Callable, Dict, List, Optional

import numpy as np

from ..linalg.vectors import DenseMatrix, DenseVector, SparseVector, Vector

_HIGH_BIT = 0x80


class DataOutput:
    def __init__(self, stream: Optional[BinaryIO] = None):
        self.stream = stream if stream is not None else io.BytesIO()

    def write(self, b: bytes):
        self.stream.write(b)

    def write_byte(self, v: int):
        self.stream.write(struct.pack(">b", v if v < 128 else v - 256))

    def write_ubyte(self, v: int):
        self.stream.write(bytes([v & 0xFF]))

    def write_bool(self, v: bool):
        self.stream.write(b"\x01" if v else b"\x00")

    def write_int(self, v: int):
        self.stream.write(struct.pack(">i", int(v)))

    def write_long(self, v: int):
        self.stream.write(struct.pack(">q", int(v)))

    def write_double(self, v: float):
        self.stream.write(struct.pack(">d", float(v)))

    def write_float(self, v: float):
        self.stream.write(struct.pack(">f", float(v)))

    def write_doubles(self, arr):
        self.stream.write(np.asarray(arr, dtype=">f8").tobytes())

    def write_string(self, s: Optional[str]):
        """Flink ``StringValue.writeString``."""
        if s is None:
            self.write_ubyte(0)
            return
        units = s.encode("utf-16-be")
        n = len(units) // 2
        out = bytearray()
        ln = n + 1
        while ln >= _HIGH_BIT:
            out.append((ln | _HIGH_BIT) & 0xFF)
            ln >>= 7
        out.append(ln)
        for k in range(n):
            c = (units[2 * k] << 8) | units[2 * k + 1]
            while c >= _HIGH_BIT:
                out.append((c | _HIGH_BIT) & 0xFF)
                c >>= 7
            out.append(c)
        self.stream.write(bytes(out))

    def getvalue(self) -> bytes:
        return self.stream.getvalue()


class DataInput:
    def __init__(self, data):
        if isinstance(data, (bytes, bytearray, memoryview)):
            self.buf = memoryview(bytes(data))
        else:
            self.buf = memoryview(data.read())
        self.pos = 0

    def remaining(self) -> int:
        return len(self.buf) - self.pos

    def eof(self) -> bool:
        return self.pos >= len(self.buf)

    def _take(self, n: int) -> memoryview:
        if self.pos + n > len(self.buf):
            raise EOFError("unexpected end of data")
        b = self.buf[self.pos:self.pos + n]
        self.pos += n
        return b

    def read_ubyte(self) -> int:
        return self._take(1)[0]

    def read_byte(self) -> int:
        v = self.read_ubyte()
        return v - 256 if v >= 128 else v

    def read_bool(self) -> bool:
        return self.read_ubyte() != 0

    def read_int(self) -> int:
        return struct.unpack(">i", self._take(4))[0]

    def read_long(self) -> int:
        return struct.unpack(">q", self._take(8))[0]

    def read_double(self) -> float:
        return struct.unpack(">d", self._take(8))[0]

    def read_float(self) -> float:
        return struct.unpack(">f", self._take(4))[0]

    def read_doubles(self, n: int) -> np.ndarray:
        return np.frombuffer(self._take(8 * n), dtype=">f8").astype(np.float64)

    def read_string(self) -> Optional[str]:
        ln = self.read_ubyte()
        if ln >= _HIGH_BIT:
            shift = 7
            ln &= 0x7F
            while True:
                b = self.read_ubyte()
                if b >= _HIGH_BIT:
                    ln |= (b & 0x7F) << shift
                    shift += 7
                else:
                    ln |= b << shift
                    break
        if ln == 0:
            return None
        n = ln - 1
        units = bytearray()
        for _ in range(n):
            c = self.read_ubyte()
            if c >= _HIGH_BIT:
                shift = 7
                c &= 0x7F
                while True:
                    b = self.read_ubyte()
                    if b >= _HIGH_BIT:
                        c |= (b & 0x7F) << shift
                        shift += 7
                    else:
                        c |= b << shift
                        break
            units += bytes([(c >> 8) & 0xFF, c & 0xFF])
        return bytes(units).decode("utf-16-be", errors="surrogatepass")


# -- vector / matrix serializers --------------------------------------------------------------
def write_dense_vector(out: DataOutput, v: DenseVector):
    vals = v.values if isinstance(v, DenseVector) else np.asarray(v, dtype=np.float64)
    out.write_int(vals.shape[0])
    out.write_doubles(vals)


def read_dense_vector(inp: DataInput) -> DenseVector:
    n = inp.read_int()
    return DenseVector(inp.read_doubles(n))


def write_sparse_vector(out: DataOutput, v: SparseVector):
    out.write_int(v.n)
    nnz = v.indices.shape[0]
    out.write_int(nnz)
    rec = np.empty(nnz, dtype=[("i", ">i4"), ("v", ">f8")])
    rec["i"] = v.indices
    rec["v"] = v.values
    out.write(rec.tobytes())


def read_sparse_vector(inp: DataInput) -> SparseVector:
    n = inp.read_int()
    nnz = inp.read_int()
    rec = np.frombuffer(inp._take(12 * nnz), dtype=[("i", ">i4"), ("v", ">f8")])
    return SparseVector(n, rec["i"].astype(np.int32), rec["v"].astype(np.float64))


def write_vector(out: DataOutput, v: Vector):
    if isinstance(v, SparseVector):
        out.write_ubyte(1)
        write_sparse_vector(out, v)
    else:
        out.write_ubyte(0)
        write_dense_vector(out, v)


def read_vector(inp: DataInput) -> Vector:
    tag = inp.read_ubyte()
    return read_sparse_vector(inp) if tag == 1 else read_dense_vector(inp)


def write_dense_matrix(out: DataOutput, m: DenseMatrix):
    out.write_int(m.num_rows)
    out.write_int(m.num_cols)
    out.write_doubles(m.values)


def read_dense_matrix(inp: DataInput) -> DenseMatrix:
    r = inp.read_int()
    c = inp.read_int()
    return DenseMatrix(r, c, inp.read_doubles(r * c))


def write_double_array(out: DataOutput, arr):
    arr = np.asarray(arr, dtype=np.float64)
    out.write_int(arr.shape[0])
    out.write_doubles(arr)


def read_double_array(inp: DataInput) -> np.ndarray:
    return inp.read_doubles(inp.read_int())


def write_int_array(out: DataOutput, arr):
    arr = np.asarray(arr, dtype=np.int64)
    out.write_int(arr.shape[0])
    out.write(arr.astype(">i4").tobytes())


def read_int_array(inp: DataInput) -> np.ndarray:
    n = inp.read_int()
    return np.frombuffer(inp._take(4 * n), dtype=">i4").astype(np.int64)


def write_long_array(out: DataOutput, arr):
    arr = np.asarray(arr, dtype=np.int64)
    out.write_int(arr.shape[0])
    out.write(arr.astype(">i8").tobytes())


def read_long_array(inp: DataInput) -> np.ndarray:
    n = inp.read_int()
    return np.frombuffer(inp._take(8 * n), dtype=">i8").astype(np.int64)


def write_string_array(out: DataOutput, arr):
    out.write_int(len(arr))
    for s in arr:
        out.write_string(s)


def read_string_array(inp: DataInput) -> List[str]:
    return [inp.read_string() for _ in range(inp.read_int())]


def write_map(out: DataOutput, m: Dict, write_key: Callable, write_value: Callable):
    out.write_int(len(m))
    for k, v in m.items():
        write_key(out, k)
        if v is None:
            out.write_bool(True)
        else:
            out.write_bool(False)
            write_value(out, v)


def read_map(inp: DataInput, read_key: Callable, read_value: Callable) -> Dict:
    n = inp.read_int()
    res = {}
    for _ in range(n):
        k = read_key(inp)
        is_null = inp.read_bool()
        res[k] = None if is_null else read_value(inp)
    return res
