"""Consensus per-vote batching (ADR-064,
docs/architecture/adr-064-batch-verification.md:58-64): the reference's
VoteSet (types/vote_set.go) with its signature checks moved into batches.

  * VoteSet.add_vote(vote)   == VoteSet.AddVote (types/vote_set.go:150-245),
                                one vote, one signature check
  * VoteSet.add_votes(votes) == AddVote of each vote in order, with the
                                signature checks of all of them in ONE engine
                                call (tmv_verify_vote_batch)
  * VoteBuffer               the ADR's consensus flow: votes are held until
                                the pending ones carry more than 2/3 of the
                                voting power, verified together, then later
                                votes are verified as they arrive

Bookkeeping (votes by validator, votes by block, the first 2/3 majority,
conflicting votes) follows vote_set.go:247-314 (addVerifiedVote) and
:685-692 (blockVotes).  Error texts are the reference's.  Peer 2/3 claims
(SetPeerMaj23), vote extensions and MakeCommit are out of scope: they touch
no signature.
"""
from __future__ import annotations

from typing import Callable, Dict, List, Optional, Tuple

from . import host as H
from .host import Vote

_TYPE_NAME = {H.PREVOTE_TYPE: "Prevote", H.PRECOMMIT_TYPE: "Precommit"}


def _hexu(b: bytes) -> str:
    return b.hex().upper()


def _fp(b: bytes) -> str:  # %X of libs/bytes.Fingerprint (first 6 bytes, zero padded)
    return _hexu((b + b"\0" * 6)[:6])


def _canonical_time(ts: Tuple[int, int]) -> str:
    import datetime
    secs, nanos = ts
    t = datetime.datetime(1970, 1, 1) + datetime.timedelta(seconds=secs)
    frac = ("%09d" % nanos).rstrip("0")
    return t.strftime("%Y-%m-%dT%H:%M:%S") + ("." + frac if frac else "") + "Z"


def vote_string(v: Vote) -> str:
    """Vote.String() (types/vote.go:191-224) of an extension-free vote."""
    bh = _fp(v.block_id.hash) if v.block_id.hash else "nil"
    return "Vote{%d:%s %d/%d %s %s %s %d @ %s}" % (v.validator_index, _fp(v.validator_address), v.height, v.round,
                                                  _TYPE_NAME.get(v.type, "?"), bh, _fp(v.signature), 0,
                                                  _canonical_time(v.timestamp))


def _block_key(b: H.BlockID):
    return (b.hash, b.psh_total, b.psh_hash)


def _pubkey_string(kind: int, pk: bytes) -> str:
    return ("PubKeyEd25519{%s}" if kind == H.TMV_KIND_ED25519 else "PubKeySr25519{%s}") % _hexu(pk)


VerifyFn = Callable[[str, List[Vote], List[Tuple[int, bytes]]], List[int]]


class VoteSet:
    """types.VoteSet for one (height, round, type), verifying signatures
    through `verify` (list of votes + their validators' keys -> TMV_VOTE_*
    per vote; e.g. lambda c, v, k: host.verify_vote_batch(ctx, c, v, k))."""

    def __init__(self, chain_id: str, height: int, round_: int, msg_type: int, vals: H.ValidatorSet,
                 verify: VerifyFn):
        self.chain_id, self.height, self.round, self.type, self.vals = chain_id, height, round_, msg_type, vals
        self.verify = verify
        n = len(vals.validators)
        self.votes: List[Optional[Vote]] = [None] * n
        self.sum = 0
        self.maj23: Optional[H.BlockID] = None
        self.votes_by_block: Dict[tuple, dict] = {}
        self.signature_batches = 0  # engine calls made (tests / metrics)

    # -------------------------------------------------------------- reference API
    def total_power(self) -> int:
        return self.vals.total_voting_power()

    def has_two_thirds_majority(self) -> bool:
        return self.maj23 is not None

    def two_thirds_majority(self) -> Tuple[Optional[H.BlockID], bool]:
        return (self.maj23, True) if self.maj23 is not None else (H.BlockID(), False)

    def has_two_thirds_any(self) -> bool:
        return self.sum > self.total_power() * 2 // 3

    def get_by_index(self, i: int) -> Optional[Vote]:
        return self.votes[i] if 0 <= i < len(self.votes) else None

    def add_vote(self, vote: Optional[Vote]) -> Tuple[bool, Optional[str]]:
        return self.add_votes([vote])[0]

    def add_votes(self, votes: List[Optional[Vote]]) -> List[Tuple[bool, Optional[str]]]:
        """AddVote of each vote in order; the signatures of every vote that
        passes the pre-signature checks are verified in one batch first."""
        pre = [self._precheck(v) for v in votes]
        cand = [i for i, p in enumerate(pre) if p is None]
        sig_res: Dict[int, int] = {}
        if cand:
            keys = [(self.vals.validators[votes[i].validator_index].key_kind,
                     self.vals.validators[votes[i].validator_index].pub_key) for i in cand]
            res = self.verify(self.chain_id, [votes[i] for i in cand], keys)
            self.signature_batches += 1
            sig_res = dict(zip(cand, res))
        out = []
        for i, v in enumerate(votes):
            if pre[i] is not None:
                out.append(pre[i])
                continue
            out.append(self._add_checked(v, sig_res[i]))
        return out

    # -------------------------------------------------------------- internals
    def _precheck(self, vote: Optional[Vote]) -> Optional[Tuple[bool, Optional[str]]]:
        """types/vote_set.go:163-199: everything addVote checks before the
        signature; None = go on to the signature."""
        if vote is None:
            return False, "nil vote"
        if vote.validator_index < 0:
            return False, "index < 0: invalid validator index"
        if not vote.validator_address:
            return False, "empty address: invalid validator address"
        if (vote.height, vote.round, vote.type) != (self.height, self.round, self.type):
            return False, ("expected %d/%d/%d, but got %d/%d/%d: unexpected step" %
                           (self.height, self.round, self.type, vote.height, vote.round, vote.type))
        if vote.validator_index >= len(self.vals.validators):
            return False, ("cannot find validator %d in valSet of size %d: invalid validator index" %
                           (vote.validator_index, len(self.vals.validators)))
        val = self.vals.validators[vote.validator_index]
        if vote.validator_address != val.address:
            return False, ("vote.ValidatorAddress (%s) does not match address (%s) for vote.ValidatorIndex (%d)\n"
                           "Ensure the genesis file is correct across all validators: invalid validator address" %
                           (_hexu(vote.validator_address), _hexu(val.address), vote.validator_index))
        return None

    def _get_vote(self, idx: int, key: tuple) -> Optional[Vote]:
        ex = self.votes[idx]
        if ex is not None and _block_key(ex.block_id) == key:
            return ex
        bv = self.votes_by_block.get(key)
        return bv["votes"].get(idx) if bv else None

    def _add_checked(self, vote: Vote, sig: int) -> Tuple[bool, Optional[str]]:
        """types/vote_set.go:201-245 from the duplicate check on, with the
        signature result already known."""
        # duplicate / non-deterministic signature checks precede the
        # signature check in the reference: re-run the pre-checks' state-
        # dependent part now, against votes added earlier in this batch
        key = _block_key(vote.block_id)
        ex = self._get_vote(vote.validator_index, key)
        if ex is not None:
            if ex.signature == vote.signature:
                return False, None
            return False, "existing vote: %s; new vote: %s: non-deterministic signature" % (vote_string(ex),
                                                                                          vote_string(vote))
        if sig != H.VOTE_OK:
            val = self.vals.validators[vote.validator_index]
            why = "invalid validator address" if sig == H.VOTE_ERR_INVALID_ADDRESS else "invalid signature"
            return False, "failed to verify vote with ChainID %s and PubKey %s: %s" % (
                self.chain_id, _pubkey_string(val.key_kind, val.pub_key), why)
        added, conflicting = self._add_verified(vote, key, self.vals.validators[vote.validator_index].voting_power)
        if conflicting is not None:
            return added, "conflicting votes from validator %s" % _hexu(conflicting.validator_address)
        return added, None

    def _add_verified(self, vote: Vote, key: tuple, power: int):
        """types/vote_set.go:247-314."""
        idx = vote.validator_index
        conflicting = None
        ex = self.votes[idx]
        if ex is not None:
            conflicting = ex
            if self.maj23 is not None and _block_key(self.maj23) == key:
                self.votes[idx] = vote
        else:
            self.votes[idx] = vote
            self.sum += power
        bv = self.votes_by_block.get(key)
        if bv is not None:
            if conflicting is not None and not bv["peer_maj23"]:
                return False, conflicting
        else:
            if conflicting is not None:
                return False, conflicting
            bv = {"peer_maj23": False, "votes": {}, "sum": 0}
            self.votes_by_block[key] = bv
        orig = bv["sum"]
        quorum = self.total_power() * 2 // 3 + 1
        if idx not in bv["votes"]:  # blockVotes.addVerifiedVote (:685-692)
            bv["votes"][idx] = vote
            bv["sum"] += power
        if orig < quorum <= bv["sum"] and self.maj23 is None:
            self.maj23 = vote.block_id
            for i, v in bv["votes"].items():
                self.votes[i] = v
        return True, conflicting


class VoteBuffer:
    """ADR-064's consensus flow over a VoteSet: votes are held until the
    pending ones carry more than 2/3 of the voting power, then verified and
    added in one batch (add_votes); after that each vote goes straight in.
    Results come back per vote in arrival order as they are decided."""

    def __init__(self, vote_set: VoteSet):
        self.vs = vote_set
        self.pending: List[Vote] = []
        self.pending_power = 0
        self.flushed = False

    def add(self, vote: Vote) -> List[Tuple[Vote, Tuple[bool, Optional[str]]]]:
        if self.flushed:
            return [(vote, self.vs.add_vote(vote))]
        self.pending.append(vote)
        val = self.vs.vals.validators[vote.validator_index] \
            if 0 <= vote.validator_index < len(self.vs.vals.validators) else None
        if val is not None:
            self.pending_power += val.voting_power
        if self.pending_power > self.vs.total_power() * 2 // 3:
            return self.flush()
        return []

    def flush(self) -> List[Tuple[Vote, Tuple[bool, Optional[str]]]]:
        votes, self.pending, self.pending_power = self.pending, [], 0
        self.flushed = True
        return list(zip(votes, self.vs.add_votes(votes)))
