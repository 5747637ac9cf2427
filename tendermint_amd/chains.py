"""Callers of the commit verifier, driven with cross-commit batching
 — the two reference loops that feed the
signature path one commit at a time:

  * light.Client.verifySequential (light/client.go:554-634) ->
    light.VerifyAdjacent (light/verifier.go:106-155) -> VerifyCommitLight
  * blocksync Reactor.poolRoutine (internal/blocksync/reactor.go:549-645):
    state.Validators.VerifyCommitLight(second.LastCommit) and then
    ValidateBlock(first) -> state.LastValidators.VerifyCommit(first.LastCommit)

Here every commit check of a window of headers/blocks is planned on the host
and all their signatures go to the GPU in ONE tmv_verify_commits call; the
per-header / per-block results are then walked in order, so the first error
returned is the one the sequential reference loop would return.  The
ValidatorSet.Hash of every supplied set of a window (light/verifier.go:266,
SURVEY §8(f) rank 4) is computed on the GPU in one tmv_validator_set_hashes
call; the header hash itself is not (headers carry it as opaque bytes).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional, Tuple

import numpy as np

from . import host as H


@dataclass
class SignedHeader:
    chain_id: str
    height: int
    time: Tuple[int, int]
    validators_hash: bytes
    next_validators_hash: bytes
    commit: H.Commit


@dataclass
class LightBlock:
    header: SignedHeader
    vals: H.ValidatorSet


def _after(a: Tuple[int, int], b: Tuple[int, int]) -> bool:
    return a > b


def validator_set_arrays(sets: List[H.ValidatorSet]):
    """Column arrays of tmv_validator_set_hashes for `sets` (set order kept)."""
    vals = [v for vs in sets for v in vs.validators]
    n = len(vals)
    pk = np.frombuffer(b"".join(v.pub_key for v in vals), np.uint8) if n else np.zeros(0, np.uint8)
    kind = np.fromiter((v.key_kind for v in vals), np.uint8, count=n)
    power = np.fromiter((v.voting_power for v in vals), np.int64, count=n)
    off = np.zeros(len(sets) + 1, np.uint32)
    off[1:] = np.cumsum([len(vs.validators) for vs in sets])
    return pk, kind, power, off


def validator_set_hashes(ctx, sets: List[H.ValidatorSet]) -> List[bytes]:
    """ValidatorSet.Hash (types/validator_set.go:344-350) of each set, one GPU call."""
    if not sets:
        return []
    out = ctx.validator_set_hashes(*validator_set_arrays(sets))
    return [bytes(r) for r in out]


def verify_adjacent_checks(trusted: SignedHeader, untrusted: SignedHeader,
                           untrusted_vals_hash: Optional[bytes] = None) -> Optional[str]:
    """The non-signature checks of light.VerifyAdjacent (light/verifier.go:115-150)
    that this engine's callers need, in the reference's order and text;
    `untrusted_vals_hash` = Hash() of the supplied set (verifier.go:266)."""
    if trusted.height == 0:
        return "height in trusted header must be set (non zero"
    if not trusted.chain_id:
        return "chain ID in trusted header must be set"
    if len(trusted.next_validators_hash) == 0:
        return "next validators hash in trusted header is empty"
    if untrusted.height != trusted.height + 1:
        return "headers must be adjacent in height"
    if not _after(untrusted.time, trusted.time):
        return "invalid header: expected new header time to be after old header time"
    if untrusted_vals_hash is not None and untrusted.validators_hash != untrusted_vals_hash:
        return ("invalid header: expected new header validators (%s) to match those that were supplied (%s) "
                "at height %d" % (untrusted.validators_hash.hex().upper(), untrusted_vals_hash.hex().upper(),
                                  untrusted.height))
    if untrusted.validators_hash != trusted.next_validators_hash:
        return ("invalid header: expected old header's next validators (%s) to match those from new header (%s)"
                % (trusted.next_validators_hash.hex().upper(), untrusted.validators_hash.hex().upper()))
    return None


def verify_sequential(ctx, trusted: SignedHeader, blocks: List[LightBlock], window: int = 1000
                      ) -> Tuple[int, Optional[str]]:
    """light.Client.verifySequential over `blocks` (heights trusted+1 ...).
    Returns (number of headers verified, first error or None).  `window`
    headers share one GPU batch (the light client's prefetch depth)."""
    done = 0
    for lo in range(0, len(blocks), window):
        chunk = blocks[lo:lo + window]
        jobs = [H.CommitJob(H.MODE_LIGHT, trusted.chain_id, lb.vals, lb.header.commit.block_id, lb.header.height,
                            lb.header.commit) for lb in chunk]
        res = H.verify_commits(ctx, jobs)
        vhash = validator_set_hashes(ctx, [lb.vals for lb in chunk])
        for lb, err, vh in zip(chunk, res, vhash):
            e = verify_adjacent_checks(trusted, lb.header, vh)
            if e is None and err is not None:
                e = "invalid header: " + err
            if e is not None:
                return done, e
            trusted = lb.header
            done += 1
    return done, None


@dataclass
class Block:
    height: int
    block_id: H.BlockID
    last_commit: Optional[H.Commit]   # commit for height-1 (None at the first height)
    commit: H.Commit                  # the commit for this block (= next block's LastCommit)


def blocksync_replay(ctx, chain_id: str, vals: H.ValidatorSet, blocks: List[Block], window: int = 600
                     ) -> Tuple[int, Optional[Tuple[int, str]]]:
    """poolRoutine's two checks per block pair (first, second):
      light: vals.VerifyCommitLight(chainID, first.BlockID, first.Height, second.LastCommit)
      full:  vals.VerifyCommit(chainID, prev.BlockID, first.Height-1, first.LastCommit)
    over a static validator set, `window` blocks per GPU batch (the pool
    buffers up to 600 blocks, internal/blocksync/pool.go:32-35).  A commit
    checked light at height H and full at H+1 is one tmv_commit, so its
    signatures are verified once.  Returns (blocks applied, (height, error))."""
    applied = 0
    for lo in range(0, len(blocks) - 1, window):
        chunk = blocks[lo:lo + window + 1]
        jobs, where = [], []
        for i in range(len(chunk) - 1):
            first, second = chunk[i], chunk[i + 1]
            jobs.append(H.CommitJob(H.MODE_LIGHT, chain_id, vals, first.block_id, first.height, first.commit))
            where.append((first.height, "light"))
            if first.last_commit is not None:
                prev = blocks[lo + i - 1] if lo + i >= 1 else None
                pbid = prev.block_id if prev is not None else first.last_commit.block_id
                jobs.append(H.CommitJob(H.MODE_FULL, chain_id, vals, pbid, first.height - 1, first.last_commit))
                where.append((first.height, "full"))
        res = H.verify_commits(ctx, jobs)
        for (height, _kind), err in zip(where, res):
            if err is not None:
                return applied + (height - chunk[0].height), (height, err)
        applied += len(chunk) - 1
    return applied, None
