"""Text / hashing feature stages (reference ``LIB/feature/{tokenizer,regextokenizer,ngram,
stopwordsremover,hashingtf,featurehasher,countvectorizer,idf}``).

String handling is host-side (columns of Python lists); the hashing (Guava murmur3_32, K18) runs in
the native host library or, for large batches, in the device kernel (``hash.hip``). Numeric
outputs (term-frequency vectors, IDF weighting) are device-resident sparse/dense columns.
"""
from __future__ import annotations

import functools
import json
import math
import os
import re
from collections import Counter
from typing import Dict, List, Sequence

import numpy as np
import torch

from ... import config
from ...api.stage import Estimator, Transformer
from ...common.param import (HasCategoricalCols, HasInputCol, HasInputCols, HasNumFeatures, HasOutputCol,
                             HasOutputCols)
from ...io import read_write as rw
from ...io import serialization as ser
from ...linalg.vectors import DenseVector, SparseVector, Vector
from ...ops import hashing, native
from ...param.param import (BooleanParam, FloatParam, IntParam, ParamValidators, StringArrayParam, StringParam)
from ...parallel import comm
from ...parallel import datastream as ds
from ...table import SparseColumn, StringArrayColumn, StringColumn, Table
from ...utils.java import java_hashmap_order as _java_hashmap_order
from ...utils.java import java_number_to_string, java_string_hash
from ...utils.strtable import StrTable, hashmap_order_from_hashes
from ..base import ModelWithData
from ..linear import rw_update
from .common import dec_dense, enc_dense, get_world_distributed, vector_input

ENGLISH_STOP_WORDS = (
    'a', 'about', 'above', 'after', 'again', 'against', 'all', 'am', 'an', 'and', 'any', 'are', "aren't",
    'as', 'at', 'be', 'because', 'been', 'before', 'being', 'below', 'between', 'both', 'but', 'by', 'can',
    "can't", 'cannot', 'could', "couldn't", 'did', "didn't", 'do', 'does', "doesn't", 'doing', 'don',
    "don't", 'down', 'during', 'each', 'few', 'for', 'from', 'further', 'had', "hadn't", 'has', "hasn't",
    'have', "haven't", 'having', 'he', "he'd", "he'll", "he's", 'her', 'here', "here's", 'hers', 'herself',
    'him', 'himself', 'his', 'how', "how's", 'i', "i'd", "i'll", "i'm", "i've", 'if', 'in', 'into', 'is',
    "isn't", 'it', "it's", 'its', 'itself', 'just', "let's", 'me', 'more', 'most', "mustn't", 'my', 'myself',
    'no', 'nor', 'not', 'now', 'of', 'off', 'on', 'once', 'only', 'or', 'other', 'ought', 'our', 'ours',
    'ourselves', 'out', 'over', 'own', 's', 'same', "shan't", 'she', "she'd", "she'll", "she's", 'should',
    "shouldn't", 'so', 'some', 'such', 't', 'than', 'that', "that's", 'the', 'their', 'theirs', 'them',
    'themselves', 'then', 'there', "there's", 'these', 'they', "they'd", "they'll", "they're", "they've",
    'this', 'those', 'through', 'to', 'too', 'under', 'until', 'up', 'very', 'was', "wasn't", 'we', "we'd",
    "we'll", "we're", "we've", 'were', "weren't", 'what', "what's", 'when', "when's", 'where', "where's",
    'which', 'while', 'who', "who's", 'whom', 'why', "why's", 'will', 'with', "won't", 'would', "wouldn't",
    'you', "you'd", "you'll", "you're", "you've", 'your', 'yours', 'yourself', 'yourselves',
)


def java_split(pattern: str, s: str) -> List[str]:
    """``String.split(regex)``: trailing empty strings removed, no leading empty string for a
    zero-width match at position 0, ``"".split(x) == [""]``."""
    if s == "":
        return [""]
    parts = re.split(pattern, s)
    m = re.match(pattern, s)
    if m is not None and m.end() == 0 and parts and parts[0] == "":
        parts = parts[1:]
    while parts and parts[-1] == "":
        parts.pop()
    return parts


_ZERO_WIDTH = ("^", "$", "\\b", "\\B", "\\A", "\\Z", "\\G", "(?=", "(?!", "(?<")


def batched_java_split(strings: List[str], pat: "re.Pattern", lower: bool):
    """``java_split`` of many strings with ONE regex pass over their concatenation: the strings
    are joined by a separator the pattern cannot match, the pattern splits the whole text, and
    the pieces are cut back per string with C-level splits and numpy (no Python call per string).
    Returns (tokens per string [n] int64, flat token object array) or None when the pattern is not
    safe to run across string boundaries (groups, anchors, lookarounds, empty matches) or the
    data holds the separator characters — the per-string path applies then."""
    if pat.groups or any(z in pat.pattern for z in _ZERO_WIDTH) or pat.search("") is not None:
        return None
    seps = [c for c in ("\x00", "\x01", "\x02", "\ue000", "\ue001", "\ue002") if pat.search(c) is None]
    if len(seps) < 3:
        return None
    text = seps[0].join(strings)
    if lower:
        text = text.lower()
    sep, mark, end = seps[0], seps[1], seps[2]
    if text.count(sep) != max(len(strings) - 1, 0) or mark in text or end in text:
        return None
    pieces = pat.split(text)
    # every string ends with the `end` token; pieces of one string are joined by `mark`
    flat = np.array(mark.join(pieces).replace(sep, mark + end + mark).split(mark) + [end], dtype=object)
    is_end = flat == end
    if int(is_end.sum()) != len(strings):
        return None
    sid = np.cumsum(is_end) - is_end  # string id of every token (the end token: its own string)
    ntok_raw = np.bincount(sid[~is_end], minlength=len(strings))
    tok = flat[~is_end]
    tsid = sid[~is_end]
    # Java removes trailing empty strings when the string had a match (> 1 piece); a string
    # without a match is returned whole (also "")
    nonempty = np.fromiter(map(len, tok), dtype=np.int64, count=tok.shape[0]) > 0
    pos = np.arange(tok.shape[0])
    last = np.full(len(strings), -1, dtype=np.int64)
    np.maximum.at(last, tsid[nonempty], pos[nonempty])
    keep = (pos <= last[tsid]) | (ntok_raw[tsid] == 1)
    tok, tsid = tok[keep], tsid[keep]
    return np.bincount(tsid, minlength=len(strings)).astype(np.int64), tok


def java_hashmap_order(keys: Sequence[str]) -> List[str]:
    """Iteration order of a ``java.util.HashMap<String, _>`` filled in ``keys`` order."""
    return _java_hashmap_order(keys, java_string_hash)


def _strings_col(t: Table, col: str) -> list:
    return t.get_list(col)


def _dict_col(t: Table, col: str):
    """The column as a dictionary-encoded ``StringArrayColumn`` on the compute device (codes stay
    in HBM), or None when it is a plain list column (the per-row host path then applies)."""
    c = t.column(col)
    if isinstance(c, StringArrayColumn) and len(c) > 0:
        return c.to(config.compute_device()).rebased()
    return None


def _register_textops():
    import ctypes

    from ...ops import native

    vp, i64 = ctypes.c_void_p, ctypes.c_int64
    native.register_host_sigs({"fmlx_tokenize_ws_lower": ([vp, vp, i64, vp, vp, i64, vp, vp, vp], i64),
                               "fmlx_tokenize_class": ([vp, vp, i64, vp, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                        vp, vp, i64, vp, vp, vp], i64)})


_register_textops()


def simple_class_pattern(pattern: str):
    """(delimiter table over ASCII [128] uint8, plus) when ``pattern`` is ONE character atom (a
    literal, an escape, ``.``, a ``[...]`` class, ``\\s``/``\\d``/``\\w``) optionally followed by
    ``+`` — the split the native class tokenizer does; None otherwise."""
    try:
        import re._parser as sre_parse  # Python >= 3.11
    except ImportError:  # pragma: no cover - Python 3.10
        import sre_parse
    try:
        parsed = list(sre_parse.parse(pattern))
    except Exception:
        return None
    if len(parsed) != 1:
        return None
    op, av = parsed[0]
    plus = False
    atom = pattern
    if op is sre_parse.MAX_REPEAT or op is sre_parse.MIN_REPEAT:
        lo, hi, sub = av
        if op is not sre_parse.MAX_REPEAT or lo != 1 or hi != sre_parse.MAXREPEAT or len(sub) != 1:
            return None
        op = list(sub)[0][0]
        plus = True
        atom = pattern[:-1]
        if not pattern.endswith("+"):
            return None
    if op not in (sre_parse.LITERAL, sre_parse.IN, sre_parse.ANY, sre_parse.NOT_LITERAL):
        return None
    try:
        rx = re.compile(atom)
    except re.error:
        return None
    table = np.array([1 if rx.fullmatch(chr(c)) else 0 for c in range(128)], dtype=np.uint8)
    return table, plus


def native_class_tokens(strings: List[str], table: np.ndarray, plus: bool, lower: bool, min_len: int):
    """RegexTokenizer's split (gaps) on a one-character pattern in native code for ASCII strings:
    (tokens per string, flat token ids, token vocabulary), or None for non-ASCII input."""
    from ...ops import native

    try:
        raw = "".join(strings).encode("ascii")
    except UnicodeEncodeError:
        return None
    n = len(strings)
    offs = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(np.fromiter(map(len, strings), dtype=np.int64, count=n), out=offs[1:])
    cap = int(offs[-1]) + n + 1
    ntok = np.zeros(n, dtype=np.int32)
    ids = np.zeros(cap, dtype=np.int32)
    vbytes = np.zeros(int(offs[-1]) + cap, dtype=np.uint8)
    voffs = np.zeros(cap + 1, dtype=np.int64)
    nv = np.zeros(1, dtype=np.int64)
    buf = np.frombuffer(raw, dtype=np.uint8) if raw else np.zeros(1, dtype=np.uint8)
    tab = np.ascontiguousarray(table, dtype=np.uint8)
    nt = native.host().fmlx_tokenize_class(buf.ctypes.data, offs.ctypes.data, n, tab.ctypes.data, int(plus),
                                           int(lower), int(min_len), ntok.ctypes.data, ids.ctypes.data, cap,
                                           vbytes.ctypes.data, voffs.ctypes.data, nv.ctypes.data)
    if nt < 0:
        return None
    nvoc = int(nv[0])
    vocab = vbytes[: int(voffs[nvoc])].tobytes().decode("ascii").split("\n")[:nvoc] if nvoc else []
    return ntok.astype(np.int64), ids[:nt], vocab


def _native_ws_lower_tokens(strings: List[str]):
    """Tokenizer's lowercase + ``split("\\s")`` over distinct strings in native code
    (``csrc/host/textops.cpp``): (tokens per string, flat token ids, token vocabulary), or None
    when a string is not ASCII (the Unicode-aware Python path then applies)."""
    from ...ops import native

    try:
        raw = "".join(strings).encode("ascii")
    except UnicodeEncodeError:
        return None
    n = len(strings)
    offs = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(np.fromiter(map(len, strings), dtype=np.int64, count=n), out=offs[1:])
    cap = int(offs[-1]) + n + 1
    ntok = np.zeros(n, dtype=np.int32)
    ids = np.zeros(cap, dtype=np.int32)
    vbytes = np.zeros(int(offs[-1]) + cap, dtype=np.uint8)
    voffs = np.zeros(cap + 1, dtype=np.int64)
    nv = np.zeros(1, dtype=np.int64)
    buf = np.frombuffer(raw, dtype=np.uint8) if raw else np.zeros(1, dtype=np.uint8)
    nt = native.host().fmlx_tokenize_ws_lower(buf.ctypes.data, offs.ctypes.data, n, ntok.ctypes.data, ids.ctypes.data,
                                              cap, vbytes.ctypes.data, voffs.ctypes.data, nv.ctypes.data)
    if nt < 0:
        return None
    nvoc = int(nv[0])
    vocab = vbytes[: int(voffs[nvoc])].tobytes().decode("ascii").split("\n")[:nvoc] if nvoc else []
    return ntok.astype(np.int64), ids[:nt], vocab


def _all_str(values) -> bool:
    """Whether every element is a str (one C-level join instead of a Python loop)."""
    try:
        "".join(values)
        return True
    except TypeError:
        return False


def _per_string_arrays(t: Table, col: str, fn, native_kind: str = "", batched=None):
    """``fn`` (str -> list of str) applied once per distinct string of a dictionary-encoded
    ``StringColumn``, expanded to every row by code on the device → ``StringArrayColumn``; None for
    a plain list column. ``native_kind="ws_lower"``: ``fn`` is Tokenizer's lowercase + ``\\s``
    split, done for all distinct strings at once in native code when they are ASCII. ``batched``
    (list of str -> (tokens per string, flat tokens) or None): a whole-batch version of ``fn``."""
    c = t.column(col)
    if not isinstance(c, StringColumn) or len(c) == 0 or not _all_str(c.vocab):
        return None
    dev = config.compute_device()
    codes = c.codes.to(dev).long()
    nat = _native_ws_lower_tokens(c.vocab) if native_kind == "ws_lower" else None
    if nat is None and callable(native_kind):
        nat = native_kind(c.vocab)
    if nat is None and batched is not None:
        # one regex pass over all distinct strings, the token dictionary by a native hash join
        res = batched(c.vocab)
        if res is not None:
            ntok, tok = res
            tab = StrTable.from_strings(tok.tolist())
            rep = tab.first_of_equal()
            uniq, inv = np.unique(rep, return_inverse=True)
            nat = ntok, inv.astype(np.int32), tab.take_strings(uniq)
    if nat is not None:
        vlen_np, flat_np, vocab = nat
        vlen_t = torch.from_numpy(vlen_np).to(dev)
        vflat = torch.from_numpy(flat_np).to(dev)
    else:
        index, vocab, flat, vlen = {}, [], [], []
        for w in c.vocab:
            toks = fn(w)
            vlen.append(len(toks))
            for x in toks:
                k = index.get(x)
                if k is None:
                    k = index[x] = len(vocab)
                    vocab.append(x)
                flat.append(k)
        vlen_t = torch.tensor(vlen, dtype=torch.int64, device=dev)
        vflat = torch.tensor(flat, dtype=torch.int32, device=dev)
    voff = torch.zeros(vlen_t.shape[0] + 1, dtype=torch.int64, device=dev)
    voff[1:] = torch.cumsum(vlen_t, 0)
    lens = vlen_t[codes]
    off = torch.zeros(codes.shape[0] + 1, dtype=torch.int64, device=dev)
    off[1:] = torch.cumsum(lens, 0)
    total = int(off[-1])
    rid = torch.repeat_interleave(torch.arange(codes.shape[0], device=dev), lens, output_size=total)
    local = torch.arange(total, device=dev) - off[rid]
    return StringArrayColumn(off, vflat[voff[codes[rid]] + local] if total else vflat[:0], vocab)


TF_ROWS_MAX_LEN = 32  # longest document the per-row device count takes (csrc/hash.hip fmlx_tf_rows)
native.register_kernel_sigs({
    "fmlx_tf_rows": [native.c_void_p, native.c_void_p, native.c_int, native.c_long, native.c_int, native.c_int,
                     native.c_void_p, native.c_void_p, native.c_void_p, native.c_void_p, native.c_void_p, native.c_int,
                     native.c_void_p],
})


def _tf_rows(off: torch.Tensor, idx: torch.Tensor, n: int, maxlen: int, binary: bool, nf: int):
    """HashingTF's per-document bucket counts on the GPU with one thread per document (the
    document's buckets sorted and counted in registers, csrc/hash.hip tf_rows_kernel) — instead of
    a sort-unique over all (document, bucket) keys. None when not on the GPU or a document is
    longer than ``maxlen`` (<= TF_ROWS_MAX_LEN): the caller takes the general path."""
    if idx.device.type != "cuda" or n == 0 or maxlen > TF_ROWS_MAX_LEN or TF_ROWS_MAX_LEN <= 0:
        return None
    dev = idx.device
    off = off.to(dev, torch.int64).contiguous()
    if idx.dtype not in (torch.int32, torch.int64):
        idx = idx.to(torch.int64)
    idx = idx.contiguous()
    key64, stream = int(idx.dtype == torch.int64), native.stream_ptr(dev)
    indptr = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    flag = torch.zeros(1, dtype=torch.int32, device=dev)
    native.call("fmlx_tf_rows", native.ptr(off), native.ptr(idx) if idx.numel() else None, key64, n, maxlen, 0,
                native.ptr(indptr[1:]), native.ptr(flag), None, None, None, int(binary), stream)
    if int(flag.item()):
        return None
    indptr[1:] = torch.cumsum(indptr[1:], 0)
    nnz = int(indptr[-1])
    oi = torch.empty(nnz, dtype=torch.int32, device=dev)
    ov = torch.empty(nnz, dtype=torch.float64, device=dev)
    native.call("fmlx_tf_rows", native.ptr(off), native.ptr(idx) if idx.numel() else None, key64, n, maxlen, 1,
                None, None, native.ptr(indptr), native.ptr(oi), native.ptr(ov), int(binary), stream)
    return SparseColumn(indptr, oi, ov, nf)


def _count_csr(rows: torch.Tensor, idx: torch.Tensor, n: int, width: int):
    """Per-row term counts of (row, index) pairs as one sort-unique → (indptr, indices, counts)."""
    keys, cnt = torch.unique(rows * width + idx, return_counts=True)
    r = torch.div(keys, width, rounding_mode="floor")
    indptr = torch.zeros(n + 1, dtype=torch.int64, device=rows.device)
    indptr[1:] = torch.cumsum(torch.bincount(r, minlength=n), 0)
    return indptr, (keys - r * width), cnt, r


# ------------------------------------------------------------------------------------ Tokenizer
@rw.register_stage
class Tokenizer(Transformer, HasInputCol, HasOutputCol):
    JAVA_CLASS_NAME = "org.apache.flink.ml.feature.tokenizer.Tokenizer"

    def transform(self, *inputs):
        t = inputs[0]
        out = _per_string_arrays(t, self.get(self.INPUT_COL), lambda s: java_split(r"\s", s.lower()), "ws_lower")
        if out is None:
            out = [java_split(r"\s", s.lower()) for s in _strings_col(t, self.get(self.INPUT_COL))]
        return [t.with_column(self.get(self.OUTPUT_COL), out)]


@rw.register_stage
class RegexTokenizer(Transformer, HasInputCol, HasOutputCol):
    JAVA_CLASS_NAME = "org.apache.flink.ml.feature.regextokenizer.RegexTokenizer"
    MIN_TOKEN_LENGTH = IntParam("minTokenLength", "Minimum token length", 1, ParamValidators.gt_eq(0))
    GAPS = BooleanParam("gaps", "Set regex to match gaps or tokens", True)
    PATTERN = StringParam("pattern", "Regex pattern used for tokenizing", "\\s+")
    TO_LOWERCASE = BooleanParam("toLowercase", "Whether to convert all characters to lowercase before tokenizing",
                                True)

    def transform(self, *inputs):
        t = inputs[0]
        pat = re.compile(self.get(self.PATTERN))
        gaps, low, mn = self.get(self.GAPS), self.get(self.TO_LOWERCASE), self.get(self.MIN_TOKEN_LENGTH)
        def tokenize(s):
            s = s.lower() if low else s
            toks = java_split(pat.pattern, s) if gaps else [m.group(0) for m in pat.finditer(s)]
            return [x for x in toks if len(x) >= mn]

        def batched(strings):
            res = batched_java_split(strings, pat, low) if gaps else None
            if res is None or mn <= 0:
                return res
            ntok, tok = res
            ok = np.fromiter(map(len, tok), dtype=np.int64, count=tok.shape[0]) >= mn
            sid = np.repeat(np.arange(ntok.shape[0]), ntok)
            return np.bincount(sid[ok], minlength=ntok.shape[0]).astype(np.int64), tok[ok]

        simple = simple_class_pattern(pat.pattern) if gaps else None
        nat = (lambda strings: native_class_tokens(strings, simple[0], simple[1], low, mn)) if simple else ""
        out = _per_string_arrays(t, self.get(self.INPUT_COL), tokenize, native_kind=nat, batched=batched)
        if out is None:
            out = [tokenize(s) for s in _strings_col(t, self.get(self.INPUT_COL))]
        return [t.with_column(self.get(self.OUTPUT_COL), out)]


NGRAM_DENSE_MAX = 1 << 26  # possible grams (V^n) up to which NGram uses the presence-table kernels
native.register_kernel_sigs({
    "fmlx_ngram_codes": [native.c_void_p, native.c_void_p, native.c_long, native.c_int, native.c_long, native.c_int,
                         native.c_void_p, native.c_void_p, native.c_void_p, native.c_void_p, native.c_void_p,
                         native.c_void_p],
})


def _ngram_device(dc, n: int, V: int) -> StringArrayColumn:
    """NGram on a device dictionary column with few possible grams (V^n <= NGRAM_DENSE_MAX): a
    presence table and its prefix sum replace the sort-unique of all grams (csrc/hash.hip
    ngram_mark_kernel / ngram_emit_kernel); the distinct grams come out sorted, as before."""
    dev = dc.codes.device
    codes = dc.codes.to(torch.int32).contiguous()
    off = dc.offsets.to(dev, torch.int64).contiguous()
    nd, G, stream = len(dc), V ** n, native.stream_ptr(dev)
    present = torch.zeros(G, dtype=torch.uint8, device=dev)
    noff = torch.zeros(nd + 1, dtype=torch.int64, device=dev)
    native.call("fmlx_ngram_codes", native.ptr(codes) if codes.numel() else None, native.ptr(off), nd, n, V, 0,
                native.ptr(present), native.ptr(noff[1:]), None, None, None, stream)
    noff[1:] = torch.cumsum(noff[1:], 0)
    rank = torch.cumsum(present, 0, dtype=torch.int32)
    total = int(noff[-1])
    out = torch.empty(total, dtype=torch.int32, device=dev)
    if total:
        native.call("fmlx_ngram_codes", native.ptr(codes), native.ptr(off), nd, n, V, 1, None, None, native.ptr(rank),
                    native.ptr(noff), native.ptr(out), stream)
    # (a small table is read back whole: cheaper than a device nonzero, and no torch kernel to load)
    u = np.nonzero(present.cpu().numpy())[0] if G <= (1 << 22) else torch.nonzero(present).view(-1).cpu().numpy()
    digits = []
    for _ in range(n):
        digits.append(u % V)
        u = u // V
    words = dc.vocab
    vocab = [" ".join(words[digits[n - 1 - j][i]] for j in range(n)) for i in range(len(digits[0]))]
    return StringArrayColumn(noff, out, vocab)


@rw.register_stage
class NGram(Transformer, HasInputCol, HasOutputCol):
    JAVA_CLASS_NAME = "org.apache.flink.ml.feature.ngram.NGram"
    N = IntParam("n", "Number of elements per n-gram (>=1).", 2, ParamValidators.gt_eq(1))

    def transform(self, *inputs):
        t = inputs[0]
        n = self.get(self.N)
        dc = _dict_col(t, self.get(self.INPUT_COL))
        V = len(dc.vocab) if dc is not None else 0
        if dc is not None and all(isinstance(w, str) for w in dc.vocab) and V > 0 and (V + 1) ** n < (1 << 62):
            # grams as base-V integers over consecutive codes of a row, dictionary-encoded again;
            # only the distinct grams are joined into strings on the host
            if dc.codes.is_cuda and V ** n <= NGRAM_DENSE_MAX:
                out = _ngram_device(dc, n, V)
                return [t.with_column(self.get(self.OUTPUT_COL), out)]
            codes = dc.codes.long()
            N = codes.shape[0]
            pos = torch.arange(N, device=codes.device)
            rid = dc.row_ids()
            valid = (pos - dc.offsets[rid] + n) <= dc.offsets[rid + 1] - dc.offsets[rid]
            gram = torch.zeros(N, dtype=torch.int64, device=codes.device)
            for j in range(n):
                shifted = torch.zeros_like(codes)
                shifted[: N - j] = codes[j:]
                gram = gram * V + shifted
            uniq, inv = torch.unique(gram[valid], return_inverse=True)
            digits, u = [], uniq.cpu().numpy()
            for _ in range(n):
                digits.append(u % V)
                u = u // V
            words = dc.vocab
            vocab = [" ".join(words[digits[n - 1 - j][i]] for j in range(n)) for i in range(len(uniq))]
            csum = torch.zeros(N + 1, dtype=torch.int64, device=codes.device)
            csum[1:] = torch.cumsum(valid, 0)
            out = StringArrayColumn(csum[dc.offsets], inv.to(torch.int32), vocab)
            return [t.with_column(self.get(self.OUTPUT_COL), out)]
        out = [[" ".join(toks[i:i + n]) for i in range(len(toks) - n + 1)]
               for toks in _strings_col(t, self.get(self.INPUT_COL))]
        return [t.with_column(self.get(self.OUTPUT_COL), out)]


# ------------------------------------------------------------------------------------ StopWordsRemover
_AVAILABLE_LOCALES = ("en_US", "en", "en_GB", "fr_FR", "de_DE", "es_ES", "it_IT", "pt_PT", "nl_NL", "sv_SE",
                      "da_DK", "fi_FI", "hu_HU", "nb_NO", "ru_RU", "tr_TR", "zh_CN", "ja_JP")


def _default_locale() -> str:
    return "en_US"


@functools.lru_cache(maxsize=1)
def _stopword_corpus() -> dict:
    path = os.path.join(os.path.dirname(__file__), "..", "..", "resources", "stopwords.json")
    with open(path, encoding="utf-8") as f:
        return json.load(f)["languages"]


@rw.register_stage
class StopWordsRemover(Transformer, HasInputCols, HasOutputCols):
    JAVA_CLASS_NAME = "org.apache.flink.ml.feature.stopwordsremover.StopWordsRemover"
    STOP_WORDS = StringArrayParam("stopWords", "The words to be filtered out.", ENGLISH_STOP_WORDS,
                                  ParamValidators.non_empty_array())
    CASE_SENSITIVE = BooleanParam("caseSensitive", "Whether to do a case-sensitive comparison over the stop words.",
                                  False)
    LOCALE = StringParam("locale", "Locale of the input for case insensitive matching. Ignored when caseSensitive is "
                         "true.", _default_locale(), ParamValidators.in_array(_AVAILABLE_LOCALES))
    SUPPORTED_LANGUAGES = ("danish", "dutch", "english", "finnish", "french", "german", "hungarian", "italian",
                           "norwegian", "portuguese", "russian", "spanish", "swedish", "turkish")

    @staticmethod
    def load_default_stop_words(language: str):
        """Default stop words of ``language`` (StopWordsRemover.java loadDefaultStopWords); the
        lists are the Snowball corpus bundled in ``resources/stopwords.json``."""
        lang = language.lower()
        if lang not in StopWordsRemover.SUPPORTED_LANGUAGES:
            raise ValueError("%s is not in the supported language list: %s."
                             % (language, list(StopWordsRemover.SUPPORTED_LANGUAGES)))
        if lang == "english":
            return list(ENGLISH_STOP_WORDS)
        return list(_stopword_corpus()[lang])

    @staticmethod
    def get_default_or_us() -> str:
        return _default_locale()

    @staticmethod
    def get_available_locales():
        return set(_AVAILABLE_LOCALES)

    @staticmethod
    def load_stop_words_file(path: str):
        with open(path, encoding="utf-8") as f:
            return [l.strip() for l in f if l.strip()]

    def transform(self, *inputs):
        t = inputs[0]
        ins, outs = self.get(self.INPUT_COLS), self.get(self.OUTPUT_COLS)
        if len(ins) != len(outs):
            raise ValueError("The number of input columns and output columns must be equal.")
        cs = self.get(self.CASE_SENSITIVE)
        sw = set(self.get(self.STOP_WORDS)) if cs else {w.lower() for w in self.get(self.STOP_WORDS)}
        res = {}
        for c, o in zip(ins, outs):
            dc = _dict_col(t, c)
            if dc is not None:
                # filter the codes on the device: one vocabulary-sized keep mask, a gather and a
                # prefix sum for the new row offsets
                keep = torch.tensor([(w if cs else (w.lower() if w is not None else w)) not in sw for w in dc.vocab],
                                    dtype=torch.bool, device=dc.device)
                m = keep[dc.codes.long()]
                csum = torch.zeros(m.shape[0] + 1, dtype=torch.int64, device=dc.device)
                csum[1:] = torch.cumsum(m, 0)
                res[o] = StringArrayColumn(csum[dc.offsets], dc.codes[m], dc.vocab)
                continue
            res[o] = [[w for w in toks if (w if cs else (w.lower() if w is not None else w)) not in sw]
                      for toks in _strings_col(t, c)]
        return [t.with_columns(res)]


# ------------------------------------------------------------------------------------ HashingTF
@rw.register_stage
class HashingTF(Transformer, HasInputCol, HasOutputCol, HasNumFeatures):
    JAVA_CLASS_NAME = "org.apache.flink.ml.feature.hashingtf.HashingTF"
    BINARY = BooleanParam("binary", "Whether each dimension of the output vector is binary or not.", False)

    def transform(self, *inputs):
        t = inputs[0]
        nf, binary = self.get(self.NUM_FEATURES), self.get(self.BINARY)
        dc = _dict_col(t, self.get(self.INPUT_COL))
        if dc is not None and all(isinstance(w, str) for w in dc.vocab):
            # hash each distinct string once, then gather the buckets by code on the device
            vb = hashing.non_negative_mod(hashing.hash_strings(dc.vocab), nf).astype(np.int64)
            idx = torch.from_numpy(vb).to(dc.device)[dc.codes.long()]
            got = _tf_rows(dc.offsets, idx, len(dc), TF_ROWS_MAX_LEN, binary, nf)
            if got is not None:
                return [t.with_column(self.get(self.OUTPUT_COL), got)]
            indptr, ind, cnt, _ = _count_csr(dc.row_ids(), idx, len(dc), nf)
            vals = torch.ones_like(cnt, dtype=torch.float64) if binary else cnt.to(torch.float64)
            return [t.with_column(self.get(self.OUTPUT_COL), SparseColumn(indptr, ind.to(torch.int32), vals, nf))]
        docs = _strings_col(t, self.get(self.INPUT_COL))
        flat, lens = [], []
        for d in docs:
            if isinstance(d, str) or not hasattr(d, "__iter__"):
                raise ValueError("Input format %s is not supported for input column %s. Supported options are "
                                 "Array and Iterable." % (type(d).__name__, self.get(self.INPUT_COL)))
            d = list(d)
            flat.extend(d)
            lens.append(len(d))
        dev = config.compute_device()
        all_str = bool(flat) and all(isinstance(x, str) for x in flat)
        if all_str and dev.type == "cuda":
            idx = hashing.hash_strings_device(flat, nf, 0, dev).to(torch.int64)
        else:
            h = hashing.hash_strings(flat) if all_str else np.array([hashing.hash_object(x) for x in flat],
                                                                    dtype=np.int32)
            idx = torch.from_numpy(hashing.non_negative_mod(h, nf).astype(np.int64)).to(dev)
        n = len(lens)
        if n and max(lens) <= TF_ROWS_MAX_LEN:
            off = torch.from_numpy(np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)).to(dev)
            got = _tf_rows(off, idx, n, max(lens), binary, nf)
            if got is not None:
                return [t.with_column(self.get(self.OUTPUT_COL), got)]
        # term counts per document as one sort-unique over (doc, bucket) keys -> CSR column
        doc = torch.repeat_interleave(torch.arange(n, device=dev), torch.tensor(lens, dtype=torch.int64, device=dev))
        keys, cnt = torch.unique(doc * nf + idx, return_counts=True)
        rows = torch.div(keys, nf, rounding_mode="floor")
        indptr = torch.zeros(n + 1, dtype=torch.int64, device=dev)
        indptr[1:] = torch.cumsum(torch.bincount(rows, minlength=n), 0)
        vals = torch.ones_like(cnt, dtype=torch.float64) if binary else cnt.to(torch.float64)
        col = SparseColumn(indptr, (keys - rows * nf).to(torch.int32), vals, nf)
        return [t.with_column(self.get(self.OUTPUT_COL), col)]


# ------------------------------------------------------------------------------------ FeatureHasher
FH_ROWS_MAX_COLS = 16  # input columns the per-row device assembly takes (csrc/hash.hip fmlx_fh_rows)
native.register_kernel_sigs({
    "fmlx_fh_rows": [native.c_void_p, native.c_int, native.c_long, native.c_int, native.c_void_p, native.c_void_p,
                     native.c_void_p, native.c_void_p, native.c_void_p],
})


@rw.register_stage
class FeatureHasher(Transformer, HasInputCols, HasOutputCol, HasCategoricalCols, HasNumFeatures):
    JAVA_CLASS_NAME = "org.apache.flink.ml.feature.featurehasher.FeatureHasher"

    def transform(self, *inputs):
        t = inputs[0]
        nf = self.get(self.NUM_FEATURES)
        ins = list(self.get(self.INPUT_COLS))
        cats = list(self.get(self.CATEGORICAL_COLS))
        if cats and not set(cats) <= set(ins):
            raise ValueError("CategoricalCols must be included in inputCols!")
        dev = config.compute_device()

        def is_cat(c):
            if c in cats:
                return True
            col = t.column(c)
            if isinstance(col, torch.Tensor):
                return col.dtype == torch.bool
            vals = [v for v in col if v is not None]
            return bool(vals) and all(isinstance(v, (str, bool, np.bool_)) for v in vals)

        def bucket(strings):
            h = hashing.hash_strings(list(strings)).astype(np.int64)
            h = np.where(h == -(1 << 31), h, np.abs(h))  # Math.abs(Integer.MIN_VALUE) stays negative
            return np.mod(h, nf)

        n = t.num_rows
        if (dev.type == "cuda" and n and 0 < len(ins) <= FH_ROWS_MAX_COLS
                and all(isinstance(t.column(c), torch.Tensor) for c in ins)):
            out = self._device_rows(t, ins, is_cat, bucket, nf, dev, n)
            return [t.with_column(self.get(self.OUTPUT_COL), out)]
        rows_l, idx_l, val_l = [], [], []
        ar = torch.arange(n, device=dev)
        for c in [c for c in ins if not is_cat(c)]:
            col = t.column(c)
            if isinstance(col, torch.Tensor):
                x, ok = col.to(dev, torch.float64), None
            else:
                ok = torch.tensor([v is not None for v in col], device=dev)
                x = torch.tensor([float(v) if v is not None else 0.0 for v in col], dtype=torch.float64, device=dev)
            i = torch.full((n,), int(bucket([c])[0]), dtype=torch.int64, device=dev)
            rows_l.append(ar if ok is None else ar[ok])
            idx_l.append(i if ok is None else i[ok])
            val_l.append(x if ok is None else x[ok])
        for c in [c for c in ins if is_cat(c)]:
            col = t.column(c)
            if isinstance(col, torch.Tensor) and col.dtype.is_floating_point:
                if col.device.type == "cuda":
                    # Double.toString + murmur3 of every value on the device (csrc/javastr.hip)
                    h = hashing.hash_prefixed_doubles_device(c + "=", col.detach()).to(torch.int64)
                    h = torch.where(h == -(1 << 31), h, h.abs())  # Math.abs(Integer.MIN_VALUE) stays negative
                    idx_l.append(torch.remainder(h, nf).to(dev))
                else:
                    # the same in native multi-threaded host code
                    h = hashing.hash_prefixed_doubles(c + "=", col.detach().to("cpu", torch.float64).numpy())
                    h = np.where(h == -(1 << 31), h.astype(np.int64), np.abs(h.astype(np.int64)))
                    idx_l.append(torch.from_numpy(np.mod(h, nf)).to(dev))
                rows_l.append(ar)
                val_l.append(torch.ones(n, dtype=torch.float64, device=dev))
            elif isinstance(col, torch.Tensor):
                u, inv = torch.unique(col, return_inverse=True)
                if col.dtype == torch.bool:
                    names = ["true" if v else "false" for v in u.tolist()]
                elif col.dtype.is_floating_point:
                    names = [java_number_to_string(v) for v in u.tolist()]
                else:
                    names = [str(int(v)) for v in u.tolist()]
                lut = torch.from_numpy(bucket(c + "=" + x for x in names)).to(dev)
                rows_l.append(ar)
                idx_l.append(lut[inv.to(dev)])
                val_l.append(torch.ones(n, dtype=torch.float64, device=dev))
            else:
                keep = [r for r, v in enumerate(col) if v is not None]
                strs = [c + "=" + (("true" if col[r] else "false") if isinstance(col[r], (bool, np.bool_)) else
                                   (col[r] if isinstance(col[r], str) else java_number_to_string(col[r])))
                        for r in keep]
                rows_l.append(torch.tensor(keep, dtype=torch.int64, device=dev))
                idx_l.append(torch.from_numpy(bucket(strs)).to(dev))
                val_l.append(torch.ones(len(keep), dtype=torch.float64, device=dev))
        # TreeMap<Integer, Double> per row: sum duplicates, ascending indices -> one sort-unique
        rows = torch.cat(rows_l) if rows_l else torch.zeros(0, dtype=torch.int64, device=dev)
        keys = rows * nf + (torch.cat(idx_l) if idx_l else rows)
        vals = torch.cat(val_l) if val_l else torch.zeros(0, dtype=torch.float64, device=dev)
        ukeys, inv = torch.unique(keys, return_inverse=True)
        sums = torch.zeros(ukeys.numel(), dtype=torch.float64, device=dev).index_add_(0, inv, vals)
        urows = torch.div(ukeys, nf, rounding_mode="floor")
        indptr = torch.zeros(n + 1, dtype=torch.int64, device=dev)
        indptr[1:] = torch.cumsum(torch.bincount(urows, minlength=n), 0)
        col_out = SparseColumn(indptr, (ukeys - urows * nf).to(torch.int32), sums, nf)
        return [t.with_column(self.get(self.OUTPUT_COL), col_out)]

    @staticmethod
    def _device_rows(t, ins, is_cat, bucket, nf, dev, n):
        """Every input a tensor on the GPU: each row's (index, value) pairs — numeric columns
        (constant index, the value), categorical ones (the murmur3 of "col=value", 1.0) — go to
        one kernel (csrc/hash.hip fh_rows_kernel) that sorts and merges them per row in registers,
        instead of a sort-unique + index_add over all n·W pairs."""
        keep, desc = [], []
        for c in [c for c in ins if not is_cat(c)]:
            x = t.column(c).to(dev, torch.float64).contiguous()
            keep.append(x)
            desc.append((0, x.data_ptr(), 2, int(bucket([c])[0])))
        for c in [c for c in ins if is_cat(c)]:
            col = t.column(c)
            if col.dtype.is_floating_point:
                # Double.toString + murmur3 of every value on the device (csrc/javastr.hip)
                h = hashing.hash_prefixed_doubles_device(c + "=", col.detach().to(dev))
                keep.append(h)
                desc.append((h.data_ptr(), 0, 1, nf))
            else:
                u, inv = torch.unique(col, return_inverse=True)
                names = (["true" if v else "false" for v in u.tolist()] if col.dtype == torch.bool
                         else [str(int(v)) for v in u.tolist()])
                lut = torch.from_numpy(bucket(c + "=" + x for x in names)).to(dev)
                ix = lut[inv.to(dev)].contiguous()
                keep.append(ix)
                desc.append((ix.data_ptr(), 0, 3, 0))
        d = torch.tensor(desc, dtype=torch.int64).to(dev)
        W, stream = len(desc), native.stream_ptr(dev)
        indptr = torch.zeros(n + 1, dtype=torch.int64, device=dev)
        native.call("fmlx_fh_rows", native.ptr(d), W, n, 0, native.ptr(indptr[1:]), None, None, None, stream)
        indptr[1:] = torch.cumsum(indptr[1:], 0)
        nnz = int(indptr[-1])
        oi = torch.empty(nnz, dtype=torch.int32, device=dev)
        ov = torch.empty(nnz, dtype=torch.float64, device=dev)
        native.call("fmlx_fh_rows", native.ptr(d), W, n, 1, None, native.ptr(indptr), native.ptr(oi), native.ptr(ov),
                    stream)
        del keep
        return SparseColumn(indptr, oi, ov, nf)


# ------------------------------------------------------------------------------------ CountVectorizer
class CountVectorizerModelParams(HasInputCol, HasOutputCol):
    MIN_TF = FloatParam("minTF", "Filter to ignore rare words in a document.", 1.0, ParamValidators.gt_eq(0.0))
    BINARY = BooleanParam("binary", "Binary toggle to control the output vector values.", False)


class CountVectorizerParams(CountVectorizerModelParams):
    VOCABULARY_SIZE = IntParam("vocabularySize", "Max size of the vocabulary.", 1 << 18, ParamValidators.gt(0))
    MIN_DF = FloatParam("minDF", "Minimum number of different documents a term must appear in.", 1.0,
                        ParamValidators.gt_eq(0.0))
    MAX_DF = FloatParam("maxDF", "Maximum number of different documents a term could appear in.", float(2 ** 63 - 1),
                        ParamValidators.gt_eq(0.0))


@rw.register_stage
class CountVectorizerModel(ModelWithData, CountVectorizerModelParams):
    JAVA_CLASS_NAME = "org.apache.flink.ml.feature.countvectorizer.CountVectorizerModel"
    MODEL_DATA_COLUMNS = ("vocabulary",)

    @staticmethod
    def encode_record(out, row):
        ser.write_string_array(out, list(row[0]))

    @staticmethod
    def decode_record(inp):
        return (ser.read_string_array(inp),)

    @classmethod
    def make_model_data_table(cls, rows):
        return Table({"vocabulary": [list(r[0]) for r in rows]}, num_rows=len(rows))

    def transform(self, *inputs):
        t = inputs[0]
        vocab = self.model_data_rows()[0][0]
        index = {w: i for i, w in enumerate(vocab)}
        min_tf, binary = self.get(self.MIN_TF), self.get(self.BINARY)
        dc = _dict_col(t, self.get(self.INPUT_COL))
        if dc is not None:
            vmap = torch.tensor([index.get(w, -1) for w in dc.vocab], dtype=torch.int64, device=dc.device)
            mi = vmap[dc.codes.long()]
            ok = mi >= 0
            n = len(dc)
            indptr, ind, cnt, r = _count_csr(dc.row_ids()[ok], mi[ok], n, max(1, len(vocab)))
            thr = (torch.full_like(cnt, 0, dtype=torch.float64) + min_tf if min_tf >= 1.0
                   else dc.row_lengths().to(torch.float64)[r] * min_tf)
            keep = cnt.to(torch.float64) >= thr
            if not bool(keep.all()):
                r, ind, cnt = r[keep], ind[keep], cnt[keep]
                indptr = torch.zeros(n + 1, dtype=torch.int64, device=dc.device)
                indptr[1:] = torch.cumsum(torch.bincount(r, minlength=n), 0)
            vals = torch.ones_like(cnt, dtype=torch.float64) if binary else cnt.to(torch.float64)
            col = SparseColumn(indptr, ind.to(torch.int32), vals, len(vocab))
            return [t.with_column(self.get(self.OUTPUT_COL), col)]
        out = []
        for doc in _strings_col(t, self.get(self.INPUT_COL)):
            cnt = Counter(index[w] for w in doc if w in index)
            thr = min_tf if min_tf >= 1.0 else len(doc) * min_tf
            keys = sorted(k for k, c in cnt.items() if c >= thr)
            out.append(SparseVector(len(vocab), keys, [1.0 if binary else float(cnt[k]) for k in keys]))
        return [t.with_column(self.get(self.OUTPUT_COL), SparseColumn.from_vectors(out, len(vocab)) if out else out)]


# document frequencies: a (doc, term) presence bitmap up to this many bits, else a per-document
# segmented sort (equal-length documents), else one global unique of (doc, term) keys
DF_BITMAP_MAX = 1 << 32
DF_SEGMENTED_SORT = True
CV_TFDF_MAX_V = 4096  # dictionary sizes the one-pass tf / df kernel takes (csrc/hash.hip cv_tfdf_kernel)
native.register_kernel_sigs({
    "fmlx_cv_tfdf": [native.c_void_p, native.c_void_p, native.c_long, native.c_int, native.c_void_p, native.c_void_p,
                     native.c_void_p, native.c_void_p],
})


def _cv_counts_device(dc, tab, V: int, N: int):
    """(vocabulary table in first-seen order, [tf, df] per term, first positions) of a device
    dictionary column in one kernel pass over its codes (csrc/hash.hip cv_tfdf_kernel); the [V]
    results are ordered on the host."""
    dev = dc.codes.device
    codes = dc.codes if dc.codes.dtype == torch.int32 else dc.codes.to(torch.int32)
    off = dc.offsets.to(dev, torch.int64).contiguous()
    out = torch.zeros(3 * V, dtype=torch.int64, device=dev)  # tf | df | first
    out[2 * V:] = N
    native.call("fmlx_cv_tfdf", native.ptr(codes.contiguous()), native.ptr(off), len(dc), V, native.ptr(out),
                native.ptr(out[V:]), native.ptr(out[2 * V:]), native.stream_ptr(dev))
    h = out.cpu().numpy().reshape(3, V)
    present = np.nonzero(h[0] > 0)[0]
    present = present[np.argsort(h[2][present], kind="stable")]  # first-seen order
    sums = np.stack([h[0][present], h[1][present]], 1).astype(np.float64)
    return tab.take(present), sums, h[2][present].copy()


@rw.register_stage
class CountVectorizer(Estimator, CountVectorizerParams):
    JAVA_CLASS_NAME = "org.apache.flink.ml.feature.countvectorizer.CountVectorizer"

    def fit(self, *inputs):
        dc = _dict_col(inputs[0], self.get(self.INPUT_COL))
        tab = None
        if dc is not None:
            try:
                tab = StrTable.from_strings(dc.vocab)
            except TypeError:
                tab = None
            if tab is not None and not np.array_equal(tab.first_of_equal(), np.arange(len(tab))):
                tab = None  # repeated dictionary entries: per-document counting on the host path
        if tab is not None:
            # term and document frequencies per distinct string from the codes on the device; the
            # first-occurrence order (it decides HashMap bucket-collision order) via a scatter-min
            V = len(dc.vocab)
            N, nd = dc.codes.shape[0], len(dc)
            if dc.codes.is_cuda and 0 < V <= CV_TFDF_MAX_V and N < (1 << 32) and nd:
                tab, sums, firsts = _cv_counts_device(dc, tab, V, N)
            else:
                codes = dc.codes.long()
                tf_t = torch.bincount(codes, minlength=V)
                lens = dc.offsets[1:] - dc.offsets[:-1]
                L = int(lens[0]) if nd else 0
                if nd * V <= DF_BITMAP_MAX:  # (doc, term) presence bitmap: a scatter instead of a sort
                    pres = torch.zeros(nd * V, dtype=torch.bool, device=codes.device)
                    pres[dc.row_ids() * V + codes] = True
                    df_t = pres.view(nd, V).sum(0)
                    del pres
                elif 0 < L <= 4096 and DF_SEGMENTED_SORT and bool((lens == L).all()):
                    # equal-length documents: sort each document's codes (a segmented sort along
                    # dim 1), count every term once per document
                    S = torch.sort(dc.codes.view(nd, L), dim=1).values
                    first_in_doc = torch.ones_like(S, dtype=torch.bool)
                    first_in_doc[:, 1:] = S[:, 1:] != S[:, :-1]
                    df_t = torch.bincount(S[first_in_doc].long(), minlength=V)
                    del S, first_in_doc
                else:
                    df_t = torch.bincount(torch.unique(dc.row_ids() * V + codes) % V, minlength=V)
                present = torch.nonzero(tf_t > 0).reshape(-1)
                # first occurrences over a geometrically growing prefix: every term usually shows up
                # early, so the scatter-min does not run over (and contend on) all N codes
                first = torch.full((V,), N, dtype=torch.int64, device=codes.device)
                s0, step = 0, 1 << 20
                while s0 < N:
                    e0 = min(N, s0 + step)
                    first.scatter_reduce_(0, codes[s0:e0], torch.arange(s0, e0, device=codes.device), reduce="amin")
                    if not bool((first[present] == N).any()):
                        break
                    s0, step = e0, step * 4
                present = present[torch.argsort(first[present])]  # first-seen order, sorted on the device
                pres_h = present.cpu().numpy()
                tab = tab.take(pres_h)
                sums = torch.stack([tf_t[present], df_t[present]], 1).cpu().numpy().astype(np.float64)
                firsts = first[present].cpu().numpy()
            ndocs = len(dc)
        else:
            docs = _strings_col(inputs[0], self.get(self.INPUT_COL))
            order, tf, df = [], {}, {}
            for doc in docs:
                for w, c in Counter(doc).items():
                    if w not in tf:
                        order.append(w)
                        tf[w], df[w] = 0, 0
                    tf[w] += c
                    df[w] += 1
            ndocs = len(docs)
            tab = StrTable.from_strings(order)
            sums = np.array([[tf[w], df[w]] for w in order], dtype=np.float64).reshape(-1, 2)
            firsts = np.arange(len(order), dtype=np.int64)
        # the per-rank vocabularies merged by a keyed shuffle of the strings (first-seen order:
        # rank, then position), document counts summed
        tab, sums, _ = ds.reduce_strings_by_key(tab, sums, firsts)
        rows = int(comm.all_reduce_scalar(float(ndocs), "sum")) if get_world_distributed() else ndocs
        if rows == 0:
            raise RuntimeError("The training set is empty.")
        g_df = sums[:, 1]
        min_df, max_df = self.get(self.MIN_DF), self.get(self.MAX_DF)
        keys = hashmap_order_from_hashes(tab.java_hashes())
        if min_df != self.MIN_DF.default_value or max_df != self.MAX_DF.default_value:
            amin = min_df if min_df >= 1.0 else min_df * rows
            amax = max_df if max_df >= 1.0 else max_df * rows
            if amax < amin:
                raise RuntimeError("maxDF must be >= minDF.")
            kept = keys[(g_df[keys] >= amin) & (g_df[keys] <= amax)]
            keys = kept[hashmap_order_from_hashes(tab.java_hashes()[kept])]
        keys = keys[np.argsort(-g_df[keys], kind="stable")]  # stable, like List.sort
        vocab = tab.take_strings(keys[: self.get(self.VOCABULARY_SIZE)])
        m = CountVectorizerModel().set_model_data(CountVectorizerModel.make_model_data_table([(vocab,)]))
        rw_update(m, self)
        return m


# ------------------------------------------------------------------------------------ IDF
class IDFModelParams(HasInputCol, HasOutputCol):
    pass


@rw.register_stage
class IDFModel(ModelWithData, IDFModelParams):
    JAVA_CLASS_NAME = "org.apache.flink.ml.feature.idf.IDFModel"
    MODEL_DATA_COLUMNS = ("idf", "docFreq", "numDocs")

    @staticmethod
    def encode_record(out, row):
        enc_dense(out, row[0])
        ser.write_long_array(out, row[1])
        out.write_long(int(row[2]))

    @staticmethod
    def decode_record(inp):
        return (dec_dense(inp), list(ser.read_long_array(inp)), inp.read_long())

    @classmethod
    def make_model_data_table(cls, rows):
        return Table({"idf": [r[0] for r in rows], "docFreq": [list(r[1]) for r in rows],
                      "numDocs": torch.tensor([int(r[2]) for r in rows])}, num_rows=len(rows))

    def transform(self, *inputs):
        t = inputs[0]
        idf = self.model_data_rows()[0][0]
        X = vector_input(t, self.get(self.INPUT_COL))
        if isinstance(X, SparseColumn):
            w = torch.as_tensor(idf.values, dtype=torch.float64, device=X.values.device)
            out = SparseColumn(X.indptr, X.indices, X.values.to(torch.float64) * w[X.indices.long()], X.size)
        else:
            w = torch.as_tensor(idf.values, dtype=torch.float64, device=X.device)
            out = X.to(torch.float64) * w if X.device.type == "cpu" else X.float() * w.float()
        return [t.with_column(self.get(self.OUTPUT_COL), out)]


@rw.register_stage
class IDF(Estimator, IDFModelParams):
    JAVA_CLASS_NAME = "org.apache.flink.ml.feature.idf.IDF"
    MIN_DOC_FREQ = IntParam("minDocFreq", "Minimum number of documents that a term should appear for filtering.", 0,
                            ParamValidators.gt_eq(0))

    def fit(self, *inputs):
        t = inputs[0]
        X = vector_input(t, self.get(self.INPUT_COL))
        if isinstance(X, SparseColumn):
            n = len(X)
            df = torch.zeros(X.size, dtype=torch.float64, device=X.values.device)
            df.index_add_(0, X.indices.long(), (X.values > 0).to(torch.float64))
        else:
            n = X.shape[0]
            df = (X > 0).to(torch.float64).sum(0)
        df = comm.all_reduce_sum(df)
        n = int(comm.all_reduce_scalar(float(n), "sum"))
        if n == 0:
            raise RuntimeError("The training set is empty.")
        df = df.cpu()  # the [d] finalisation on the host (no first-use torch kernel loads on the GPU)
        keep = df >= self.get(self.MIN_DOC_FREQ)
        idf = torch.where(keep, torch.log((n + 1) / (df + 1)), torch.zeros_like(df))
        dfl = torch.where(keep, df, torch.zeros_like(df)).to(torch.int64)
        m = IDFModel().set_model_data(IDFModel.make_model_data_table(
            [(DenseVector(idf.numpy()), dfl.tolist(), n)]))
        rw_update(m, self)
        return m
