"""Device → host reads without a blocking HIP wait.

A blocking copy (``tensor.cpu()``, ``.item()``, ``.tolist()``) waits inside the HIP runtime on
an HSA completion signal; in the sparse SVC whole-fit traces those waits sat in 4-ms
``hsa_signal_wait_scacquire`` timeouts with the GPU idle (profiles/r4/svc_stall_systrace_summary.json).
Here the copy is stream-ordered into pinned host memory (torch's caching host allocator: no
hipHostMalloc after the first use of a size) and the host polls the completion event
(``hipEventQuery``: a load of the signal value, no wait), yielding the CPU between polls only
after a spin budget.
"""
from __future__ import annotations

import time

import torch

SPIN_POLLS = 20000  # ≈ tens of µs of busy polling before the poll loop starts yielding


def wait_event(ev: "torch.cuda.Event") -> None:
    """Returns once ``ev`` has completed, by polling (never a blocking runtime wait)."""
    i = 0
    while not ev.query():
        i += 1
        if i > SPIN_POLLS:
            time.sleep(0)  # yield; still a poll, not a runtime wait


def wait_stream(device=None) -> None:
    """Completion of everything queued so far on the current stream of ``device``, polled."""
    ev = torch.cuda.Event()
    ev.record(torch.cuda.current_stream(device))
    wait_event(ev)


def to_host(t: torch.Tensor) -> torch.Tensor:
    """A pinned host copy of a device tensor, stream-ordered after the work that produces it."""
    if t.device.type != "cuda":
        return t
    out = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
    out.copy_(t, non_blocking=True)
    wait_stream(t.device)
    return out


WARM_PINNED_BYTES = 64 << 20  # (plus one block of each smaller power-of-two size, see warm)


def warm(device=None) -> None:
    """One-time set-up of the read-back path, done at library load instead of inside the first
    fit: a pinned block in torch's caching host allocator (later read-backs up to its size reuse
    it instead of a hipHostMalloc each), and one large copy each way (the runtime brings up its
    copy engine queues on the first large copy: ~2 ms per copy inside the first sparse-SVC fit),
    plus the event machinery's first-use imports."""
    dev = torch.device(device if device is not None else "cuda")
    buf = torch.empty(WARM_PINNED_BYTES, dtype=torch.uint8, pin_memory=True)
    big = 8 << 20
    d = torch.empty(big, dtype=torch.uint8, device=dev)
    d.copy_(buf[:big], non_blocking=True)
    buf[:big].copy_(d, non_blocking=True)
    buf[:16].copy_(d[:16], non_blocking=True)
    wait_stream(dev)
    del buf, d
    # torch's caching host allocator keeps freed pinned blocks per power-of-two size and does not
    # split a larger one for a smaller request: one block of every read-back size up to 64 MiB
    # (a 1M-wide fp64 coefficient vector is 8 MiB: its first read-back paid a ~1 ms hipHostMalloc
    # inside the first fit, profiles/r6 svc fit timeline)
    keep = [torch.empty(1 << b, dtype=torch.uint8, pin_memory=True) for b in range(5, 27)]
    del keep
