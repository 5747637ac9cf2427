"""Signature sharding across GPUs: one process per GPU,
contiguous index ranges, and the one real exchange of the path — gathering
every rank's validity vector as a packed bitmap (n/8 bytes) over RCCL
(torch.distributed "nccl") or gloo on CPU tensors.

Signatures are independent, so there is no data-path collective; the
all-gather only assembles the Add-order vector the host needs (the
reference's verifyCommitBatch walks it for the first failure,
types/validation.go:244-251).
"""
from __future__ import annotations

from typing import List, Tuple

import torch
import torch.distributed as dist

_WEIGHTS = {}


def shard_range(n: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous, size-balanced [lo, hi) of n entries for this rank."""
    return n * rank // world, n * (rank + 1) // world


def pack_bits(valid: torch.Tensor) -> torch.Tensor:
    """Status vector -> little-endian bit-packed uint8 (8 entries per byte),
    bit set iff the status is 1 (sr25519 Add-error statuses are negative)."""
    n = valid.numel()
    pad = (-n) % 8
    key = valid.device
    w = _WEIGHTS.get(key)
    if w is None:
        w = torch.tensor([1, 2, 4, 8, 16, 32, 64, 128], dtype=torch.int32, device=valid.device)
        _WEIGHTS[key] = w
    v = torch.nn.functional.pad((valid.reshape(-1) == 1).to(torch.int32), (0, pad)).view(-1, 8)
    return (v * w).sum(1).to(torch.uint8)


def unpack_bits(bits: torch.Tensor, n: int) -> torch.Tensor:
    shifts = torch.arange(8, device=bits.device, dtype=torch.int32)
    v = (bits.to(torch.int32).unsqueeze(1) >> shifts) & 1
    return v.reshape(-1)[:n].to(torch.uint8)


def all_gather_statuses(status_local: torch.Tensor, counts: List[int], group=None) -> torch.Tensor:
    """Gather every rank's int8 status vector unpacked (n bytes): sr25519 and
    mixed batches, whose statuses -1 / -2 are deferred BatchVerifier.Add
    errors (crypto/sr25519/batch.go:30-37) that verifyCommitBatch returns
    verbatim (types/validation.go:211-213) — a bitmap would turn them into
    plain invalid signatures."""
    world = len(counts)
    m = max(counts)
    st = status_local.reshape(-1).to(torch.int8)
    if st.numel() < m:
        st = torch.nn.functional.pad(st, (0, m - st.numel()))
    out = [torch.empty(m, dtype=torch.int8, device=st.device) for _ in range(world)]
    dist.all_gather(out, st, group=group)
    return torch.cat([out[r][:counts[r]] for r in range(world)])


def all_gather_validity(valid_local: torch.Tensor, counts: List[int], group=None) -> torch.Tensor:
    """Gather every rank's validity vector (counts[r] entries on rank r) as
    packed bitmaps (n/8 bytes) and return the full Add-order 0/1 vector on
    every rank.  ed25519 batches only: use all_gather_statuses where an entry
    can carry a negative (Add-error) status."""
    world = len(counts)
    nbytes = (max(counts) + 7) // 8
    bits = pack_bits(valid_local)
    if bits.numel() < nbytes:
        bits = torch.nn.functional.pad(bits, (0, nbytes - bits.numel()))
    out = [torch.empty(nbytes, dtype=torch.uint8, device=bits.device) for _ in range(world)]
    dist.all_gather(out, bits, group=group)
    return torch.cat([unpack_bits(out[r], counts[r]) for r in range(world)])
