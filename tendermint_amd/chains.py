"""Callers of the verification engine, driven with cross-commit batching
 — the reference loops that feed the
signature path one header / block at a time:

  * light.Client.verifySequential (light/client.go:554-634): VerifyAdjacent
    per height (light/verifier.go:106-155)
  * light.Client.verifySkipping (light/client.go:647-727): light.Verify
    (light/verifier.go:158-177) against a bisection cache of pivots
  * blocksync Reactor.poolRoutine (internal/blocksync/reactor.go:549-645):
    state.Validators.VerifyCommitLight(firstID, second.LastCommit), then
    ValidateBlock(first) -> state.LastValidators.VerifyCommit(
    state.LastBlockID, first.Height-1, first.LastCommit)
    (internal/state/validation.go:86-96)

The light checks run entirely in the engine's C++ host layer
(tmv_light_verify_many: Header.Hash and ValidatorSet.Hash of a whole window
on the device, SignedHeader.ValidateBasic, the trusting period / clock drift
checks and every commit check of the window in one signature batch); the
drivers here only decide which checks form a window and walk the results in
the reference's order, so the first error returned is the one the
one-at-a-time loop returns.  Primary/witness handling (provider I/O,
detector) is out of scope (networking).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, Dict, List, Optional, Tuple

from . import host as H
from .host import LightBlock, LightJob, SignedHeader  # noqa: F401  (re-exported)

# light/client.go:45-46
SKIPPING_NUM, SKIPPING_DEN = 9, 16


@dataclass
class VerificationFailed:
    """light.ErrVerificationFailed (light/errors.go:53-66): the class and text
    of the wrapped error (TMV_LIGHT_*), the heights it failed between."""
    from_height: int
    to_height: int
    kind: int
    reason: str

    def __str__(self) -> str:
        return "verify from #%d to #%d failed: %s" % (self.from_height, self.to_height, self.reason)


def validator_set_arrays(sets: List[H.ValidatorSet]):
    """Column arrays of tmv_validator_set_hashes for `sets` (set order kept)."""
    import numpy as np
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


def in_order(windows, run, depth: int):
    """run(w) for each window with up to `depth` windows in flight on caller
    threads, results yielded in window order.  The engine calls release the
    GIL, so one window's conversion and engine call overlap another's.
    Windows are independent (each is built from inputs only, never from an
    earlier window's result), so a later window verified before an earlier
    one fails only costs work: the consumer stops at the first error and
    what ran past it is discarded -- the results equal one window at a
    time.  A consumer that stops early cancels the windows not yet started
    and waits for the running ones."""
    if depth <= 1:
        for w in windows:
            yield run(w)
        return
    from collections import deque
    from concurrent.futures import ThreadPoolExecutor
    q = deque()
    with ThreadPoolExecutor(depth) as ex:
        try:
            for w in windows:
                q.append(ex.submit(run, w))
                if len(q) >= depth:
                    yield q.popleft().result()
            while q:
                yield q.popleft().result()
        finally:
            for f in q:
                f.cancel()


def verify_sequential(ctx, trusted: LightBlock, blocks: List[LightBlock], trusting_period_ns: int,
                      now: Tuple[int, int], max_clock_drift_ns: int = 10 * 10**9, window: int = 1000,
                      verify_many=None, depth: Optional[int] = None) -> Tuple[int, Optional[VerificationFailed]]:
    """Client.verifySequential over `blocks` (heights trusted+1, ...) with a
    single primary: VerifyAdjacent(verified, interim) per height, `window`
    headers per engine call (the light client's prefetch), `depth` windows in
    flight (default 2 on the engine, 1 with a caller's `verify_many`; see
    in_order).  Returns (headers verified, first ErrVerificationFailed or
    None)."""
    if depth is None:
        depth = 1 if verify_many else 2
    if verify_many:
        run, prepare = verify_many, (lambda jobs: jobs)
    else:
        # the C structs are built on this thread (Python, under the GIL),
        # the engine calls on the in_order threads (GIL released)
        fn = H._setup_light(H._setup(H._native.lib())).tmv_light_verify_many
        run = lambda pj: H.run_light_jobs(fn, ctx.handle, pj)
        prepare = H.PreparedLightJobs

    def windows():
        for lo in range(0, len(blocks), window):
            p = trusted if lo == 0 else blocks[lo - 1]
            jobs = []
            for lb in blocks[lo:lo + window]:
                jobs.append(LightJob(p.signed_header, None, lb.signed_header, lb.vals, trusting_period_ns, now,
                                     max_clock_drift_ns, mode=H.LIGHT_ADJACENT))
                p = lb
            yield prepare(jobs)

    done = 0
    prev = trusted
    for lo, res in zip(range(0, len(blocks), window), in_order(windows(), run, depth)):
        chunk = blocks[lo:lo + window]
        for lb, (kind, text) in zip(chunk, res):
            if kind != H.LIGHT_OK:
                return done, VerificationFailed(prev.height, lb.height, kind, text)
            prev = lb
            done += 1
    return done, None


def schedule(last_verified: int, last_failed: int) -> int:
    """Client.schedule (light/client.go:721-725)."""
    return last_verified + (last_failed - last_verified) * SKIPPING_NUM // SKIPPING_DEN


def verify_skipping(ctx, trusted: LightBlock, target: LightBlock, provider: Callable[[int], LightBlock],
                    trusting_period_ns: int, now: Tuple[int, int], max_clock_drift_ns: int = 10 * 10**9,
                    trust: Tuple[int, int] = (1, 3), speculate: int = 8, verify_many=None
                    ) -> Tuple[Optional[List[int]], Optional[VerificationFailed]]:
    """Client.verifySkipping (light/client.go:647-727): bisection from the
    trusted block towards `target`, pivots from `provider(height)`.  The
    reference verifies one candidate per step; here every step verifies the
    current candidate, the rest of the cache and up to `speculate` further
    pivots (the heights schedule() would request next) in ONE engine call, and
    the results are consumed in the reference's order, so the trace and the
    error equal the reference's.  A provider error on a speculative pivot
    only stops the speculation; on a pivot the reference requests it is
    returned as ErrVerificationFailed{verified, pivot, err}
    (light/client.go:706-709).  Returns (trace heights, None) or
    (None, ErrVerificationFailed)."""
    run = verify_many or (lambda jobs: H.light_verify_many(ctx, jobs))
    cache = [target]
    fetched: Dict[int, LightBlock] = {}
    refused: Dict[int, Exception] = {}  # speculative fetches that failed (asked again only when needed)
    depth = 0
    verified = trusted
    trace = [trusted.height]
    results: Dict[Tuple[int, int], Tuple[int, Optional[str]]] = {}

    def block_at(h: int) -> LightBlock:
        if h not in fetched:
            fetched[h] = provider(h)
        return fetched[h]

    def speculative(h: int) -> Optional[LightBlock]:
        """A pivot the reference may never request: a provider error only
        ends the speculation (the reference would not have seen it)."""
        if h in refused:
            return None
        try:
            return block_at(h)
        except Exception as e:  # noqa: BLE001 -- any provider failure
            refused[h] = e
            return None

    while True:
        cand = cache[depth]
        key = (id(verified), id(cand))
        if key not in results:
            batch = list(cache[depth:])
            last = cache[-1].height
            for _ in range(speculate):
                p = schedule(verified.height, last)
                if p <= verified.height or p >= last:
                    break
                b = speculative(p)
                if b is None:
                    break
                batch.append(b)
                last = p
            # the client passes the verified block's own validator set
            # (light/client.go:680-681)
            jobs = [LightJob(verified.signed_header, verified.vals, b.signed_header, b.vals,
                             trusting_period_ns, now, max_clock_drift_ns, trust) for b in batch]
            for b, r in zip(batch, run(jobs)):
                results[(id(verified), id(b))] = r
        kind, text = results[key]
        if kind == H.LIGHT_OK:
            if depth == 0:
                trace.append(target.height)
                return trace, None
            verified = cand
            cache = cache[:depth]
            depth = 0
            trace.append(verified.height)
        elif kind == H.LIGHT_ERR_CANT_TRUST:
            if depth == len(cache) - 1:
                pivot = schedule(verified.height, cache[depth].height)
                refused.pop(pivot, None)  # the reference requests this one: ask again
                try:
                    cache.append(block_at(pivot))
                except Exception as e:  # noqa: BLE001 -- light/client.go:706-709
                    return None, VerificationFailed(verified.height, pivot, H.LIGHT_ERR_OTHER, str(e))
            depth += 1
        else:
            return None, VerificationFailed(verified.height, cand.height, kind, text)


@dataclass
class Block:
    """The parts of a types.Block blocksync's checks read."""
    height: int
    block_id: H.BlockID               # BlockID{Hash: block.Hash(), PartSetHeader}
    last_commit: Optional[H.Commit]   # the commit for height-1 carried by this block


def blocksync_replay(ctx, chain_id: str, vals: H.ValidatorSet, blocks: List[Block], last_block_id: H.BlockID,
                     initial_height: int = 1, window: int = 600, depth: Optional[int] = None,
                     verify_commits=None) -> Tuple[int, Optional[Tuple[int, str]]]:
    """poolRoutine's checks for each block pair (first, second) over a static
    validator set (state.Validators == state.LastValidators):
      light: vals.VerifyCommitLight(chainID, first.BlockID, first.Height, second.LastCommit)
      full:  ValidateBlock(first): at state.InitialHeight the LastCommit must
             carry no signatures, else vals.VerifyCommit(chainID,
             state.LastBlockID, first.Height-1, first.LastCommit)
    with state.LastBlockID = `last_block_id` for the first block and the
    previous block's BlockID after it (ApplyBlock).  `window` blocks per
    engine call (the pool buffers up to 600, internal/blocksync/pool.go:32-35);
    a commit read light at height H and full at H+1 is the same object, so its
    signatures are verified once; `depth` windows in flight (in_order;
    default 2 on the engine, 1 with a caller's `verify_commits`, a function
    jobs -> per-job error or None).  Returns (blocks applied, (height,
    error))."""
    if depth is None:
        depth = 1 if verify_commits else 2
    if verify_commits:
        prepare = lambda jobs: jobs

        def run(w):
            return w[:3], verify_commits(w[3])
    else:
        prepare = H.PreparedJobs

        def run(w):  # the C structs were built on the caller's thread (windows())
            H.run_prepared_jobs(ctx, w[3])
            return w[:3], w[3].decode()

    def windows():
        state_last = last_block_id
        for lo in range(0, len(blocks) - 1, window):
            chunk = blocks[lo:lo + window + 1]
            jobs, where, early = [], [], {}
            for i in range(len(chunk) - 1):
                first, second = chunk[i], chunk[i + 1]
                where.append((first.height, len(jobs)))
                jobs.append(H.CommitJob(H.MODE_LIGHT, chain_id, vals, first.block_id, first.height,
                                        second.last_commit))
                if first.height == initial_height:
                    if first.last_commit is not None and first.last_commit.signatures:
                        early[first.height] = "initial block can't have LastCommit signatures"
                    jobs.append(None)
                else:
                    jobs.append(H.CommitJob(H.MODE_FULL, chain_id, vals, state_last, first.height - 1,
                                            first.last_commit))
                state_last = first.block_id
            yield jobs, where, early, prepare([j for j in jobs if j is not None])

    applied = 0
    for (jobs, where, early), res in in_order(windows(), run, depth):
        it = iter(res)
        flat = [next(it) if j is not None else None for j in jobs]
        for height, k in where:
            err = flat[k] or early.get(height) or flat[k + 1]
            if err is not None:
                return applied, (height, err)
            applied += 1
    return applied, None
