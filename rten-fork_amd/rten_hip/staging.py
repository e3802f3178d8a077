"""Host-resident inputs and outputs for the device graph: ``Model::run`` as the
reference's callers use it.

RTen's ``Model::run`` takes host tensors and returns host tensors
(src/model.rs:580-592), and rten-cli times exactly that call
(rten-cli/src/main.rs:296-317).  The device graph (librten_hip.so) takes
device buffers, so a drop-in caller has to move a batch over PCIe before the
forward and the outputs back after it: 38.5 MB in and 256 KB out per
ResNet-50 batch of 64.  Done naively (copy, run, copy, wait) every step pays
the upload on top of the forward.

``HostStaging`` pipelines it instead.  Inputs come from pinned host memory
(DMA straight from the pages, no bounce copy) into one of ``slots`` device
buffers; the forward of step k runs on the compute stream as soon as its slot
has landed, while step k+1's upload is already in flight; step k's outputs go
back to pinned host memory while step k+1 computes.  ONE copy stream carries
both directions, in the order upload(k), download(k - 1): the upload of step k
only waits for the forward that last read its slot (k - 2), so it runs during
forward k - 1, and the download of step k - 1 follows it.  Events order the
streams per slot, so nothing waits on the host:

    copy    : wait in_free[s]   -> H2D host_in(k) -> dev_in[s]   -> in_ready[s]
              wait out_ready[s'] -> D2H out(k - 1) -> host_out    -> out_free[s']
    compute : wait in_ready[s], out_free[s] -> forward(dev_in[s]) -> in_free[s], out_ready[s]

The copy stream is created at high priority: a process gets few hardware
queues (GPU_MAX_HW_QUEUES, 4 by default) and a normal-priority stream can land
on the queue of the graph executor's stream, where the copies would wait
behind the forwards they are meant to overlap.  The graph keeps one captured
hipGraph per (input, output) binding (``Plan::captures``, up to four), so
alternating slots replay without re-capturing.  With the batch sharded over
ranks (parallel.py) each rank stages its own slice.
"""
from __future__ import annotations

from typing import Callable, List


class HostStaging:
    """Pipelined host -> device -> host execution of ``forward``.

    forward(dev_in, slot) runs one step on torch's current stream and returns
    the device tensor to download (it may be a slot-owned buffer or a fresh
    tensor, e.g. gathered logits)."""

    def __init__(self, forward: Callable, in_shape, device, slots: int = 2, dtype=None):
        import torch

        self.torch = torch
        self.forward = forward
        self.slots = int(slots)
        if self.slots < 1:
            raise ValueError("slots must be >= 1")
        self.device = torch.device(device)
        dtype = dtype or torch.float32
        self.compute = torch.cuda.current_stream(self.device)
        self.copy = torch.cuda.Stream(self.device, priority=-1)
        self.dev_in = [torch.empty(tuple(in_shape), dtype=dtype, device=self.device) for _ in range(self.slots)]
        E = torch.cuda.Event
        self.in_ready = [E() for _ in range(self.slots)]
        self.in_free = [E() for _ in range(self.slots)]
        self.out_ready = [E() for _ in range(self.slots)]
        self.out_free = [E() for _ in range(self.slots)]
        self.k = 0
        self.pending = None  # (slot, device output, host output) of the last step

    @staticmethod
    def pinned(shape, dtype=None):
        """A page-locked host tensor (the form the upload DMA reads directly)."""
        import torch

        return torch.empty(tuple(shape), dtype=dtype or torch.float32, pin_memory=True)

    def _download(self):
        s, out, host_out = self.pending
        self.pending = None
        with self.torch.cuda.stream(self.copy):
            self.copy.wait_event(self.out_ready[s])
            out.record_stream(self.copy)  # the allocator must not reuse it before the copy
            host_out.copy_(out, non_blocking=True)
            self.out_free[s].record(self.copy)

    def submit(self, host_in, host_out) -> None:
        """Queue one step: host_in (pinned, in_shape) -> forward -> host_out
        (pinned, the forward's output shape).  Returns without waiting; the
        host buffers must stay untouched until synchronize()."""
        torch = self.torch
        if tuple(host_in.shape) != tuple(self.dev_in[0].shape):
            raise ValueError(f"input shape {tuple(host_in.shape)} != staged {tuple(self.dev_in[0].shape)}")
        s = self.k % self.slots
        self.k += 1
        with torch.cuda.stream(self.copy):
            self.copy.wait_event(self.in_free[s])  # the forward that read this slot is done
            self.dev_in[s].copy_(host_in, non_blocking=True)
            self.in_ready[s].record(self.copy)
        if self.pending is not None:
            self._download()  # the previous step's outputs, behind this upload
        with torch.cuda.stream(self.compute):
            self.compute.wait_event(self.in_ready[s])
            self.compute.wait_event(self.out_free[s])  # this slot's last outputs are downloaded
            out = self.forward(self.dev_in[s], s)
            self.in_free[s].record(self.compute)
            self.out_ready[s].record(self.compute)
        self.pending = (s, out, host_out)

    def synchronize(self) -> None:
        if self.pending is not None:
            self._download()
        for st in (self.copy, self.compute):
            st.synchronize()


def pcie_rates(nbytes_in: int, nbytes_out: int, device, reps: int = 10) -> dict:
    """Measured pinned-host <-> device copy rates (GB/s) at the staging sizes:
    the PCIe figures the host-input throughput is judged against."""
    import time

    import torch

    dev = torch.device(device)
    hin = torch.empty(nbytes_in // 4, dtype=torch.float32, pin_memory=True)
    din = torch.empty(nbytes_in // 4, dtype=torch.float32, device=dev)
    dout = torch.empty(max(1, nbytes_out // 4), dtype=torch.float32, device=dev)
    hout = torch.empty(max(1, nbytes_out // 4), dtype=torch.float32, pin_memory=True)
    res: dict = {}
    for name, dst, src, nb in (("h2d", din, hin, nbytes_in), ("d2h", hout, dout, nbytes_out)):
        dst.copy_(src, non_blocking=True)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(reps):
            dst.copy_(src, non_blocking=True)
        torch.cuda.synchronize(dev)
        dt = (time.perf_counter() - t0) / reps
        res[f"{name}_gbps"] = round(nb / dt / 1e9, 2)
        res[f"{name}_us"] = round(dt * 1e6, 1)
    return res


__all__: List[str] = ["HostStaging", "pcie_rates"]
