"""The segmented stable LSD radix sort (csrc/radix.hip ``seg_sort``) that replaced hipCUB's
DeviceRadixSort in the sparse trainer's column-major copies and KMeans' many-cluster grouping:
exact agreement with ``torch.sort(stable=True)`` per segment — keys AND payload order — over one
and several segments (key offsets per segment, empty / one-element / partial-tile segments,
1–24 key bits = 1–3 digit passes), int32 and int64 payloads."""
import pytest
import torch

from flink_ml_amd.ops import glm as gk

pytestmark = pytest.mark.gpu


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")


def _reference(keys, vals, bounds, kbase, bits):
    ko, vo = keys.clone(), vals.clone()
    mask = (1 << bits) - 1
    for s in range(len(bounds) - 1):
        a, b = bounds[s], bounds[s + 1]
        if b <= a:
            continue
        dig = ((keys[a:b].long() - kbase[s]) & mask)
        o = torch.sort(dig, stable=True).indices
        ko[a:b] = keys[a:b][o]
        vo[a:b] = vals[a:b][o]
    return ko, vo


@pytest.mark.parametrize("n,bits,vdtype", [(1, 1, torch.int32), (8191, 4, torch.int32), (8193, 11, torch.int64),
                                           (300_001, 17, torch.int32), (1_000_003, 20, torch.int64),
                                           (2_000_000, 24, torch.int32)])
def test_single_segment_matches_torch_stable_sort(n, bits, vdtype):
    _need_gpu()
    g = torch.Generator(device="cuda").manual_seed(n + bits)
    keys = torch.randint(0, 1 << bits, (n,), generator=g, device="cuda", dtype=torch.int32)
    if bits > 6:  # many duplicates too: stability must hold inside long equal-key runs
        keys[: n // 3] = keys[: n // 3] % 37
    vals = torch.arange(n, device="cuda", dtype=vdtype) * 3 + 1
    if vdtype == torch.int64:
        vals = vals | (torch.randint(0, 1 << 30, (n,), generator=g, device="cuda", dtype=torch.int64) << 33)
    ref_k, ref_v = _reference(keys, vals, [0, n], [0], bits)
    got_k, got_v = gk.seg_sort(keys.clone(), vals.clone(), [0, n], [0], bits)
    assert torch.equal(got_k, ref_k)
    assert torch.equal(got_v, ref_v)


@pytest.mark.parametrize("vdtype", [torch.int32, torch.int64])
def test_segments_with_key_offsets_match_per_segment_sort(vdtype):
    """The column-major copy layout: key = slot·d + column, segments = batches of a run."""
    _need_gpu()
    d = 1_000_000
    lens = [0, 1, 8191, 8192, 8193, 250_000, 0, 77, 640_000, 3, 0, 100_000, 9000, 1, 2, 65_536]
    bounds = [0]
    for x in lens:
        bounds.append(bounds[-1] + x)
    n = bounds[-1]
    g = torch.Generator(device="cuda").manual_seed(5)
    keys = torch.empty(n, dtype=torch.int32, device="cuda")
    for s in range(len(lens)):
        a, b = bounds[s], bounds[s + 1]
        keys[a:b] = s * d + torch.randint(0, d, (b - a,), generator=g, device="cuda", dtype=torch.int32)
    vals = torch.arange(n, device="cuda", dtype=vdtype)
    kbase = [s * d for s in range(len(lens))]
    bits = (d - 1).bit_length()
    ref_k, ref_v = _reference(keys, vals, bounds, kbase, bits)
    got_k, got_v = gk.seg_sort(keys.clone(), vals.clone(), bounds, kbase, bits)
    assert torch.equal(got_k, ref_k)
    assert torch.equal(got_v, ref_v)
    # preallocated buffers (the hipGraph-capturable form) give the same result
    k2, v2 = torch.empty_like(keys), torch.empty_like(vals)
    sc = torch.empty(gk.seg_sort_scratch(bounds, bits), dtype=torch.int32, device="cuda")
    got_k2, got_v2 = gk.seg_sort(keys.clone(), vals.clone(), bounds, kbase, bits, k2, v2, sc)
    assert torch.equal(got_k2, ref_k) and torch.equal(got_v2, ref_v)
    assert (got_k2.data_ptr() == k2.data_ptr()) == bool(gk.seg_sort_passes(bits) & 1)


def test_split_output_writes_payload_halves():
    """Last pass with split output: keys sorted, payload low words → lo[off + i], high words →
    hi[off + i] (the column-major copy's rows / value bits), bit-exact against the unsplit sort."""
    _need_gpu()
    g = torch.Generator(device="cuda").manual_seed(9)
    bounds = [0, 70_000, 70_001, 200_000]
    d = 50_000
    n = bounds[-1]
    keys = torch.empty(n, dtype=torch.int32, device="cuda")
    for s in range(3):
        a, b = bounds[s], bounds[s + 1]
        keys[a:b] = s * d + torch.randint(0, d, (b - a,), generator=g, device="cuda", dtype=torch.int32)
    rows = torch.randint(0, 1 << 20, (n,), generator=g, device="cuda", dtype=torch.int64)
    vals = torch.rand(n, generator=g, device="cuda", dtype=torch.float32)
    pay = (vals.view(torch.int32).to(torch.int64) << 32) | rows
    kbase = [s * d for s in range(3)]
    bits = (d - 1).bit_length()
    ref_k, ref_p = _reference(keys, pay, bounds, kbase, bits)
    off = 123
    lo = torch.zeros(n + off, dtype=torch.int32, device="cuda")
    hi = torch.zeros(n + off, dtype=torch.float32, device="cuda")
    got_k, _ = gk.seg_sort(keys.clone(), pay.clone(), bounds, kbase, bits, split=(lo, hi, off))
    assert torch.equal(got_k, ref_k)
    assert torch.equal(lo[off:], (ref_p & 0xFFFFFFFF).to(torch.int32))
    assert torch.equal(hi[off:].view(torch.int32), (ref_p >> 32).to(torch.int32))
