"""Batch-sharded multi-GPU inference.

Batch items are independent in every configuration, so the path shards by
contiguous slices of the batch: rank r of G runs the whole graph on items
[r*B/G, (r+1)*B/G) with its own replica of the weights.  The only exchange is
one all-gather of the per-rank outputs (RCCL over xGMI on the GPUs, gloo in
the CPU tests).  There is no cross-rank dependency inside the graph, so no
collective runs on the data path before the outputs exist.
"""
from __future__ import annotations

from typing import Callable, Sequence, Tuple


def shard_bounds(total: int, rank: int, world: int) -> Tuple[int, int]:
    """[start, end) of rank's contiguous slice; earlier ranks take the
    remainder one item each, so sizes differ by at most one."""
    if world <= 0 or not (0 <= rank < world):
        raise ValueError("invalid rank/world")
    base, rem = divmod(total, world)
    start = rank * base + min(rank, rem)
    return start, start + base + (1 if rank < rem else 0)


def shard_sizes(total: int, world: int) -> Sequence[int]:
    return [shard_bounds(total, r, world)[1] - shard_bounds(total, r, world)[0]
            for r in range(world)]


class BatchShardRunner:
    """Runs ``fn`` (local batch -> local output, both torch tensors whose
    first dim is the batch) on this rank's slice and all-gathers the outputs
    in rank order, so every rank ends with the full [B, ...] result."""

    def __init__(self, fn: Callable, group=None):
        import torch.distributed as dist

        self.fn = fn
        self.group = group
        self.dist = dist if dist.is_available() and dist.is_initialized() else None

    @property
    def world(self) -> int:
        return self.dist.get_world_size(self.group) if self.dist else 1

    @property
    def rank(self) -> int:
        return self.dist.get_rank(self.group) if self.dist else 0

    def local_slice(self, total: int) -> Tuple[int, int]:
        return shard_bounds(total, self.rank, self.world)

    def run(self, full_batch_local_view, total: int):
        """full_batch_local_view: this rank's slice of the inputs (already
        resident on its device).  Returns the gathered [total, ...] output."""
        return self.gather(self.fn(full_batch_local_view), total)

    def gather(self, out, total: int):
        """All-gather this rank's output slice in rank order (identity with
        one rank)."""
        if self.dist is None:
            return out
        if out.is_cuda and self.dist.get_backend(self.group) == "gloo":
            # gloo moves host tensors only (the CPU tests and the one-GPU
            # multi-rank rehearsal); RCCL gathers device tensors directly.
            return self._gather(out.cpu(), total).to(out.device)
        return self._gather(out, total)

    def _gather(self, out, total: int):
        import torch

        sizes = shard_sizes(total, self.world)
        if len(set(sizes)) == 1:
            gathered = torch.empty((total,) + tuple(out.shape[1:]), dtype=out.dtype,
                                   device=out.device)
            self.dist.all_gather_into_tensor(gathered, out.contiguous(), group=self.group)
            return gathered
        # Ragged shards: pad to the largest slice, gather, then drop padding.
        m = max(sizes)
        pad = torch.zeros((m,) + tuple(out.shape[1:]), dtype=out.dtype, device=out.device)
        pad[: out.shape[0]] = out
        parts = [torch.empty_like(pad) for _ in range(self.world)]
        self.dist.all_gather(parts, pad, group=self.group)
        return torch.cat([p[:s] for p, s in zip(parts, sizes)], dim=0)
