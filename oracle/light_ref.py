"""CPU restatement of the light-client verification the engine's host layer
implements (TEST INFRASTRUCTURE: the checker for tmv_light_verify /
tmv_header_hashes / tmv_verify_commit; never imported by the product path).

Follows, in the reference (file:line under /root/reference):
  types/block.go:385-437        Header.ValidateBasic
  types/block.go:447-478        Header.Hash (merkle of 14 proto-encoded fields)
  types/encoding_helper.go:11-48 cdcEncode (gogotypes String/Int64/BytesValue)
  types/block.go:657-694        CommitSig.ValidateBasic
  types/block.go:874-897        Commit.ValidateBasic
  types/block.go:1386-1396      BlockID.ValidateBasic, types/part_set.go:116-122
  types/light.go:145-172        SignedHeader.ValidateBasic
  types/validation.go:27-359    VerifyCommit / VerifyCommitLight /
                                VerifyCommitLightTrusting, verifyCommitBatch,
                                verifyCommitSingle, verifyBasicValsAndCommit
  crypto/ed25519/ed25519.go:173-233, crypto/sr25519/batch.go:23-47  Add / Verify
  light/verifier.go:33-290      VerifyNonAdjacent, VerifyAdjacent, Verify,
                                ValidateTrustLevel, HeaderExpired,
                                verifyNewHeaderAndVals, checkRequiredHeaderFields
  light/errors.go:15-40         ErrOldHeaderExpired / ErrNewValSetCantBeTrusted /
                                ErrInvalidHeader
  light/client.go:554-727       verifySequential / verifySkipping / schedule
Go formatting (%v of time.Time and time.Duration, %q, %X) is restated so the
error texts are byte-identical.  Signatures go through oracle/ed25519_ref.py
and oracle/sr25519_ref.py (per-entry; under ZIP-215 a batch verdict equals
the per-entry one).

Pinned by the reference's own model-based fixtures light/mbt/json/*.json
(driven by light/mbt/driver_test.go:18-86): every header hash equals its
commit's BlockID hash, every validators_hash equals the supplied set's hash,
and light.Verify's verdict class equals the fixture's verdict
(tests/test_light_mbt.py, tests/golden/mbt_light.json).
"""
from __future__ import annotations

import hashlib
from dataclasses import dataclass, field
from typing import Callable, List, Optional, Tuple

import ed25519_ref
import merkle_ref

KIND_ED25519, KIND_SR25519, KIND_OTHER = 0, 1, 255
FLAG_ABSENT, FLAG_COMMIT, FLAG_NIL = 1, 2, 3
BLOCK_PROTOCOL = 11           # version/version.go:27
MAX_CHAIN_ID_LEN = 50         # types/genesis.go:19
HASH_SIZE, ADDRESS_SIZE = 32, 20
MAX_SIGNATURE_SIZE = 64       # types/signable.go:12
ZERO_TIME_NS = -62135596800 * 10**9
NS = 10**9

# error classes of light.Verify (light/errors.go)
OK, INVALID_HEADER, OLD_HEADER_EXPIRED, CANT_TRUST, OTHER = 0, 1, 2, 3, 4


# ------------------------------------------------------------------ Go formatting
def hexu(b: bytes) -> str:
    return b.hex().upper()


def _civil(days: int):
    z = days + 719468
    era = (z if z >= 0 else z - 146096) // 146097
    doe = z - era * 146097
    yoe = (doe - doe // 1460 + doe // 36524 - doe // 146096) // 365
    y = yoe + era * 400
    doy = doe - (365 * yoe + yoe // 4 - yoe // 100)
    mp = (5 * doy + 2) // 153
    d = doy - (153 * mp + 2) // 5 + 1
    m = mp + 3 if mp < 10 else mp - 9
    return (y + 1 if m <= 2 else y), m, d


def _frac9(nanos: int) -> str:
    if nanos == 0:
        return ""
    return "." + ("%09d" % nanos).rstrip("0")


def go_time(t_ns: int) -> str:
    """time.Time.String() of a UTC instant: 2006-01-02 15:04:05.999999999 -0700 MST."""
    secs, nanos = divmod(t_ns, NS)
    days, rem = divmod(secs, 86400)
    y, m, d = _civil(days)
    return "%04d-%02d-%02d %02d:%02d:%02d%s +0000 UTC" % (y, m, d, rem // 3600, (rem // 60) % 60, rem % 60,
                                                          _frac9(nanos))


def _fmt_frac(v: int, prec: int) -> Tuple[str, int]:
    digits, printed = "", False
    for _ in range(prec):
        dgt = v % 10
        printed = printed or dgt != 0
        if printed:
            digits = str(dgt) + digits
        v //= 10
    return ("." + digits if printed else ""), v


def go_duration(d: int) -> str:
    """time.Duration.String()."""
    if d == 0:
        return "0s"
    neg, u = d < 0, abs(d)
    if u < NS:
        if u < 1000:
            s = "%dns" % u
        elif u < 10**6:
            f, v = _fmt_frac(u, 3)
            s = "%d%sµs" % (v, f)
        else:
            f, v = _fmt_frac(u, 6)
            s = "%d%sms" % (v, f)
    else:
        f, v = _fmt_frac(u, 9)
        s = "%d%ss" % (v % 60, f)
        v //= 60
        if v:
            s = "%dm" % (v % 60) + s
            v //= 60
            if v:
                s = "%dh" % v + s
    return "-" + s if neg else s


def go_quote(s: str) -> str:
    """strconv.Quote for the chain IDs the path handles."""
    out = ['"']
    for ch in s:
        c = ord(ch)
        if ch == '"' or ch == "\\":
            out.append("\\" + ch)
        elif ch in "\a\b\f\n\r\t\v":
            out.append({"\a": "\\a", "\b": "\\b", "\f": "\\f", "\n": "\\n", "\r": "\\r", "\t": "\\t",
                        "\v": "\\v"}[ch])
        elif c < 0x20 or c == 0x7F:
            out.append("\\x%02x" % c)
        else:
            out.append(ch)
    out.append('"')
    return "".join(out)


def canonical_time(t_ns: int) -> str:
    """types.CanonicalTime: RFC3339Nano in UTC (types/canonical.go:61-66)."""
    secs, nanos = divmod(t_ns, NS)
    days, rem = divmod(secs, 86400)
    y, m, d = _civil(days)
    return "%04d-%02d-%02dT%02d:%02d:%02d%sZ" % (y, m, d, rem // 3600, (rem // 60) % 60, rem % 60, _frac9(nanos))


# ------------------------------------------------------------------ types
@dataclass
class BlockID:
    hash: bytes = b""
    psh_total: int = 0
    psh_hash: bytes = b""

    def is_nil(self) -> bool:
        return not self.hash and self.psh_total == 0 and not self.psh_hash

    def __str__(self) -> str:  # BlockID.String / PartSetHeader.String (Fingerprint = 6 bytes)
        return "%s:%d:%s" % (hexu(self.hash), self.psh_total, hexu((self.psh_hash + b"\0" * 6)[:6]))


@dataclass
class CommitSig:
    flag: int = FLAG_ABSENT
    address: bytes = b""
    ts_ns: int = ZERO_TIME_NS
    signature: bytes = b""

    def string(self) -> str:  # types/block.go:631-637
        fp = lambda b: hexu((b + b"\0" * 6)[:6])  # noqa: E731
        return "CommitSig{%s by %s on %d @ %s}" % (fp(self.signature), fp(self.address), self.flag,
                                                   canonical_time(self.ts_ns))


@dataclass
class Commit:
    height: int
    round: int
    block_id: BlockID
    signatures: List[CommitSig] = field(default_factory=list)


@dataclass
class Validator:
    address: bytes
    pub_key: bytes
    voting_power: int
    kind: int = KIND_ED25519
    proposer_priority: int = 0

    def string(self) -> str:  # types/validator.go:129-138
        key = {KIND_ED25519: "PubKeyEd25519", KIND_SR25519: "PubKeySr25519"}.get(self.kind, "PubKey")
        return "Validator{%s %s{%s} VP:%d A:%d}" % (hexu(self.address), key, hexu(self.pub_key), self.voting_power,
                                                   self.proposer_priority)


@dataclass
class ValidatorSet:
    validators: List[Validator]

    def total(self) -> int:
        return sum(v.voting_power for v in self.validators)

    def proposer(self) -> Optional[Validator]:
        """GetProposer with no stored proposer: highest priority, ties to the
        smaller address (types/validator_set.go:322-344, validator.go:52-71)."""
        best = None
        for v in self.validators:
            if best is None or v.proposer_priority > best.proposer_priority or \
                    (v.proposer_priority == best.proposer_priority and v.address < best.address):
                best = v
        return best

    def get_by_address(self, addr: bytes):
        for i, v in enumerate(self.validators):
            if v.address == addr:
                return i, v
        return -1, None

    def hash(self) -> bytes:
        return merkle_ref.validator_set_hash([(v.pub_key, v.kind, v.voting_power) for v in self.validators])


@dataclass
class Header:
    version_block: int = BLOCK_PROTOCOL
    version_app: int = 0
    chain_id: str = ""
    height: int = 0
    time_ns: int = ZERO_TIME_NS
    last_block_id: BlockID = field(default_factory=BlockID)
    last_commit_hash: bytes = b""
    data_hash: bytes = b""
    validators_hash: bytes = b""
    next_validators_hash: bytes = b""
    consensus_hash: bytes = b""
    app_hash: bytes = b""
    last_results_hash: bytes = b""
    evidence_hash: bytes = b""
    proposer_address: bytes = b""


@dataclass
class SignedHeader:
    header: Optional[Header]
    commit: Optional[Commit]


# ------------------------------------------------------------------ protobuf pieces
def _uvarint(u: int) -> bytes:
    u &= (1 << 64) - 1
    out = bytearray()
    while u >= 0x80:
        out.append((u & 0x7F) | 0x80)
        u >>= 7
    out.append(u)
    return bytes(out)


def _bytes_field(tag: int, b: bytes) -> bytes:
    return bytes([tag]) + _uvarint(len(b)) + b


def proto_timestamp(t_ns: int) -> bytes:
    """google.protobuf.Timestamp (gogotypes.StdTimeMarshal): zero fields omitted."""
    secs, nanos = divmod(t_ns, NS)
    out = b""
    if secs:
        out += b"\x08" + _uvarint(secs)
    if nanos:
        out += b"\x10" + _uvarint(nanos)
    return out


def proto_block_id(b: BlockID) -> bytes:
    """tmproto.BlockID: hash (omitted if empty), part_set_header (non-nullable,
    always present) {total (omitted if 0), hash (omitted if empty)}."""
    psh = (b"\x08" + _uvarint(b.psh_total) if b.psh_total else b"") + \
          (_bytes_field(0x12, b.psh_hash) if b.psh_hash else b"")
    return (_bytes_field(0x0A, b.hash) if b.hash else b"") + _bytes_field(0x12, psh)


def cdc_string(s: str) -> bytes:
    return _bytes_field(0x0A, s.encode()) if s else b""


def cdc_int64(v: int) -> bytes:
    return b"\x08" + _uvarint(v) if v else b""


def cdc_bytes(b: bytes) -> bytes:
    return _bytes_field(0x0A, b) if b else b""


def header_leaves(h: Header) -> List[bytes]:
    """The 14 byte slices of Header.Hash, in field order (types/block.go:461-476)."""
    version = (b"\x08" + _uvarint(h.version_block) if h.version_block else b"") + \
              (b"\x10" + _uvarint(h.version_app) if h.version_app else b"")
    return [version, cdc_string(h.chain_id), cdc_int64(h.height), proto_timestamp(h.time_ns),
            proto_block_id(h.last_block_id), cdc_bytes(h.last_commit_hash), cdc_bytes(h.data_hash),
            cdc_bytes(h.validators_hash), cdc_bytes(h.next_validators_hash), cdc_bytes(h.consensus_hash),
            cdc_bytes(h.app_hash), cdc_bytes(h.last_results_hash), cdc_bytes(h.evidence_hash),
            cdc_bytes(h.proposer_address)]


def header_hash(h: Optional[Header]) -> Optional[bytes]:
    """Header.Hash: nil when the header is nil or ValidatorsHash is empty."""
    if h is None or not h.validators_hash:
        return None
    return merkle_ref.hash_from_byte_slices(header_leaves(h))


# ------------------------------------------------------------------ ValidateBasic
def _validate_hash(b: bytes) -> Optional[str]:
    if b and len(b) != HASH_SIZE:
        return "expected size to be %d bytes, got %d bytes" % (HASH_SIZE, len(b))
    return None


def block_id_validate_basic(b: BlockID) -> Optional[str]:
    e = _validate_hash(b.hash)
    if e:
        return "wrong Hash: " + e
    e = _validate_hash(b.psh_hash)
    if e:
        return "wrong PartSetHeader: wrong Hash: " + e
    return None


def header_validate_basic(h: Header) -> Optional[str]:
    if h.version_block != BLOCK_PROTOCOL:
        return "block protocol is incorrect: got: %d, want: %d " % (h.version_block, BLOCK_PROTOCOL)
    if len(h.chain_id.encode()) > MAX_CHAIN_ID_LEN:
        return "chainID is too long; got: %d, max: %d" % (len(h.chain_id.encode()), MAX_CHAIN_ID_LEN)
    if h.height < 0:
        return "negative Height"
    if h.height == 0:
        return "zero Height"
    e = block_id_validate_basic(h.last_block_id)
    if e:
        return "wrong LastBlockID: " + e
    for name, v in (("LastCommitHash", h.last_commit_hash), ("DataHash", h.data_hash),
                    ("EvidenceHash", h.evidence_hash)):
        e = _validate_hash(v)
        if e:
            return "wrong %s: %s" % (name, e)
    if len(h.proposer_address) != ADDRESS_SIZE:
        return "invalid ProposerAddress length; got: %d, expected: %d" % (len(h.proposer_address), ADDRESS_SIZE)
    for name, v in (("ValidatorsHash", h.validators_hash), ("NextValidatorsHash", h.next_validators_hash),
                    ("ConsensusHash", h.consensus_hash), ("LastResultsHash", h.last_results_hash)):
        e = _validate_hash(v)
        if e:
            return "wrong %s: %s" % (name, e)
    return None


def commit_sig_validate_basic(cs: CommitSig) -> Optional[str]:
    if cs.flag not in (FLAG_ABSENT, FLAG_COMMIT, FLAG_NIL):
        return "unknown BlockIDFlag: %d" % cs.flag
    if cs.flag == FLAG_ABSENT:
        if cs.address:
            return "validator address is present"
        if cs.ts_ns != ZERO_TIME_NS:
            return "time is present"
        if cs.signature:
            return "signature is present"
    else:
        if len(cs.address) != ADDRESS_SIZE:
            return "expected ValidatorAddress size to be %d bytes, got %d bytes" % (ADDRESS_SIZE, len(cs.address))
        if not cs.signature:
            return "signature is missing"
        if len(cs.signature) > MAX_SIGNATURE_SIZE:
            return "signature is too big (max: %d)" % MAX_SIGNATURE_SIZE
    return None


def commit_validate_basic(c: Commit) -> Optional[str]:
    if c.height < 0:
        return "negative Height"
    if c.round < 0:
        return "negative Round"
    if c.height >= 1:
        if c.block_id.is_nil():
            return "commit cannot be for nil block"
        if not c.signatures:
            return "no signatures in commit"
        for i, cs in enumerate(c.signatures):
            e = commit_sig_validate_basic(cs)
            if e:
                return "wrong CommitSig #%d: %s" % (i, e)
    return None


def signed_header_validate_basic(sh: SignedHeader, chain_id: str) -> Optional[str]:
    if sh.header is None:
        return "missing header"
    if sh.commit is None:
        return "missing commit"
    e = header_validate_basic(sh.header)
    if e:
        return "invalid header: " + e
    e = commit_validate_basic(sh.commit)
    if e:
        return "invalid commit: " + e
    if sh.header.chain_id != chain_id:
        return "header belongs to another chain %s, not %s" % (go_quote(sh.header.chain_id), go_quote(chain_id))
    if sh.commit.height != sh.header.height:
        return "header and commit height mismatch: %d vs %d" % (sh.header.height, sh.commit.height)
    hh = header_hash(sh.header) or b""
    if hh != sh.commit.block_id.hash:
        return "commit signs block %s, header is block %s" % (hexu(sh.commit.block_id.hash), hexu(hh))
    return None


# ------------------------------------------------------------------ sign-bytes (types/vote.go:149-157)
def vote_sign_bytes(chain_id: str, height: int, round_: int, block_id: Optional[BlockID], ts_ns: int) -> bytes:
    """MarshalDelimited(CanonicalVote) of a precommit (proto/tendermint/types/canonical.pb.go:590-640)."""
    body = b"\x08\x02"
    if height:
        body += b"\x11" + (height & ((1 << 64) - 1)).to_bytes(8, "little")
    if round_:
        body += b"\x19" + (round_ & ((1 << 64) - 1)).to_bytes(8, "little")
    if block_id is not None and not block_id.is_nil():
        psh = (b"\x08" + _uvarint(block_id.psh_total) if block_id.psh_total else b"") + \
              (_bytes_field(0x12, block_id.psh_hash) if block_id.psh_hash else b"")
        cb = (_bytes_field(0x0A, block_id.hash) if block_id.hash else b"") + _bytes_field(0x12, psh)
        body += _bytes_field(0x22, cb)
    body += _bytes_field(0x2A, proto_timestamp(ts_ns))
    if chain_id:
        body += _bytes_field(0x32, chain_id.encode())
    return _uvarint(len(body)) + body


# Optional precomputed signature verdicts: a callable (validator, msg, sig)
# -> bool or None (None: not precomputed, verify here).  The at-size tests
# (tests/test_gpu_at_size.py) install the C restatement's verdicts of a whole
# chain (oracle_c, same ZIP-215 semantics) so the commit / light logic below
# runs over millions of signatures without big-integer verification.
_SIG_ORACLE = None


class signature_oracle:
    """Context manager installing precomputed signature verdicts."""

    def __init__(self, fn):
        self.fn, self.prev = fn, None

    def __enter__(self):
        global _SIG_ORACLE
        self.prev, _SIG_ORACLE = _SIG_ORACLE, self.fn
        return self

    def __exit__(self, *exc):
        global _SIG_ORACLE
        _SIG_ORACLE = self.prev
        return False


def _verify_sig(v: Validator, msg: bytes, sig: bytes) -> bool:
    """PubKey.VerifySignature (crypto/ed25519/ed25519.go:173-180, crypto/sr25519/pubkey.go:49-62)."""
    if _SIG_ORACLE is not None:
        r = _SIG_ORACLE(v, msg, sig)
        if r is not None:
            return r
    if v.kind == KIND_ED25519:
        return len(sig) == 64 and len(v.pub_key) == 32 and ed25519_ref.verify_zip215(v.pub_key, msg, sig)
    if v.kind == KIND_SR25519:
        import sr25519_ref
        return sr25519_ref.verify(v.pub_key, msg, sig)
    raise NotImplementedError("key type without an oracle")


def _batch_add(kind: int, v: Validator, sig: bytes) -> Optional[str]:
    """BatchVerifier.Add errors (crypto/ed25519/ed25519.go:209-224, crypto/sr25519/batch.go:23-37)."""
    if kind == KIND_ED25519:
        if v.kind != KIND_ED25519:
            return "pubkey is not Ed25519"
        if len(v.pub_key) != 32:
            return "pubkey size is incorrect; expected: 32, got %d" % len(v.pub_key)
        if len(sig) != 64:
            return "invalid signature"
        return None
    import sr25519_ref
    if v.kind != KIND_SR25519:
        return "sr25519: pubkey is not sr25519"
    try:
        sr25519_ref.batch_add_check(v.pub_key, sig)
    except sr25519_ref.AddError as e:
        return str(e)
    return None


# ------------------------------------------------------------------ commit verification
def _not_enough(got: int, needed: int) -> str:
    return "invalid commit -- insufficient voting power: got %d, needed more than %d" % (got, needed)


class CommitError(Exception):
    def __init__(self, text: str, not_enough: bool = False):
        super().__init__(text)
        self.text, self.not_enough = text, not_enough


def _verify_commit_loop(chain_id, vals: ValidatorSet, commit: Commit, needed, ignore, count, count_all, by_index):
    prop = vals.proposer()
    batch = len(commit.signatures) >= 2 and prop is not None and prop.kind in (KIND_ED25519, KIND_SR25519)
    tallied, seen = 0, {}
    entries = []  # (idx, ok)
    for idx, cs in enumerate(commit.signatures):
        if ignore(cs):
            continue
        if by_index:
            val = vals.validators[idx]
        else:
            vi, val = vals.get_by_address(cs.address)
            if val is None:
                continue
            if vi in seen:
                raise CommitError("double vote from %s (%d and %d)" % (val.string(), seen[vi], idx))
            seen[vi] = idx
        msg = vote_sign_bytes(chain_id, commit.height, commit.round,
                              commit.block_id if cs.flag == FLAG_COMMIT else None, cs.ts_ns)
        if batch:
            e = _batch_add(prop.kind, val, cs.signature)
            if e:
                raise CommitError(e)
            entries.append((idx, _verify_sig(val, msg, cs.signature)))
        else:
            if not _verify_sig(val, msg, cs.signature):
                raise CommitError("wrong signature (#%d): %s" % (idx, hexu(cs.signature)))
        if count(cs):
            tallied += val.voting_power
        if not count_all and tallied > needed:
            if not batch:
                return
            break
    if tallied <= needed:
        raise CommitError(_not_enough(tallied, needed), not_enough=True)
    if batch:
        for idx, ok in entries:
            if not ok:
                raise CommitError("wrong signature (#%d): %s" % (idx, hexu(commit.signatures[idx].string().encode())))


def _basic(vals, commit, height, block_id):
    if vals is None:
        raise CommitError("nil validator set")
    if commit is None:
        raise CommitError("nil commit")
    if len(vals.validators) != len(commit.signatures):
        raise CommitError("Invalid commit -- wrong set size: %d vs %d" % (len(vals.validators), len(commit.signatures)))
    if height != commit.height:
        raise CommitError("Invalid commit -- wrong height: %d vs %d" % (height, commit.height))
    if (block_id.hash, block_id.psh_total, block_id.psh_hash) != \
            (commit.block_id.hash, commit.block_id.psh_total, commit.block_id.psh_hash):
        raise CommitError("invalid commit -- wrong block ID: want %s, got %s" % (block_id, commit.block_id))


def verify_commit(chain_id, vals, block_id, height, commit) -> Optional[CommitError]:
    try:
        _basic(vals, commit, height, block_id)
        _verify_commit_loop(chain_id, vals, commit, vals.total() * 2 // 3, lambda c: c.flag == FLAG_ABSENT,
                            lambda c: c.flag == FLAG_COMMIT, True, True)
    except CommitError as e:
        return e
    return None


def verify_commit_light(chain_id, vals, block_id, height, commit) -> Optional[CommitError]:
    try:
        _basic(vals, commit, height, block_id)
        _verify_commit_loop(chain_id, vals, commit, vals.total() * 2 // 3, lambda c: c.flag != FLAG_COMMIT,
                            lambda c: True, False, True)
    except CommitError as e:
        return e
    return None


def verify_commit_light_trusting(chain_id, vals, commit, trust=(1, 3)) -> Optional[CommitError]:
    try:
        if vals is None:
            raise CommitError("nil validator set")
        if trust[1] == 0:
            raise CommitError("trustLevel has zero Denominator")
        if commit is None:
            raise CommitError("nil commit")
        prod = vals.total() * trust[0]
        if vals.total() and trust[0] and abs(prod) > (1 << 63) - 1:
            raise CommitError("int64 overflow while calculating voting power needed. please provide smaller "
                              "trustLevel numerator")
        _verify_commit_loop(chain_id, vals, commit, prod // trust[1], lambda c: c.flag != FLAG_COMMIT,
                            lambda c: True, False, False)
    except CommitError as e:
        return e
    return None


# ------------------------------------------------------------------ light/verifier.go
@dataclass
class LightError:
    kind: int
    text: str


def _header_expired(h: Header, trusting_period_ns: int, now_ns: int) -> bool:
    return not (h.time_ns + trusting_period_ns > now_ns)


def _check_required(sh: SignedHeader) -> Optional[str]:
    h = sh.header
    if h.height == 0:
        return "height in trusted header must be set (non zero"
    if h.time_ns == ZERO_TIME_NS:
        return "time in trusted header must be set"
    if not h.chain_id:
        return "chain ID in trusted header must be set"
    return None


def validate_trust_level(num: int, den: int) -> Optional[str]:
    """light/verifier.go:183-191 (uint64 arithmetic; %v of a Fraction is its
    String(), libs/math/fraction.go:20-22)."""
    if (num * 3) % (1 << 64) < den or num >= den or den == 0:
        return "trustLevel must be within [1/3, 1], given %d/%d" % (num, den)
    return None


def _verify_new_header_and_vals(untrusted: SignedHeader, untrusted_vals: ValidatorSet, trusted: SignedHeader,
                                now_ns: int, drift_ns: int) -> Optional[str]:
    e = signed_header_validate_basic(untrusted, trusted.header.chain_id)
    if e:
        return "untrustedHeader.ValidateBasic failed: " + e
    uh, th = untrusted.header, trusted.header
    if uh.height <= th.height:
        return "expected new header height %d to be greater than one of old header %d" % (uh.height, th.height)
    if not uh.time_ns > th.time_ns:
        return "expected new header time %s to be after old header time %s" % (go_time(uh.time_ns),
                                                                               go_time(th.time_ns))
    if not uh.time_ns < now_ns + drift_ns:
        return "new header has a time from the future %s (now: %s; max clock drift: %s)" % (
            go_time(uh.time_ns), go_time(now_ns), go_duration(drift_ns))
    vh = untrusted_vals.hash()
    if uh.validators_hash != vh:
        return "expected new header validators (%s) to match those that were supplied (%s) at height %d" % (
            hexu(uh.validators_hash), hexu(vh), uh.height)
    return None


def _expired(untrusted: SignedHeader, trusting_period_ns: int, now_ns: int) -> LightError:
    return LightError(OLD_HEADER_EXPIRED, "old header has expired at %s (now: %s)" % (
        go_time(untrusted.header.time_ns + trusting_period_ns), go_time(now_ns)))


def verify_non_adjacent(trusted: SignedHeader, trusted_vals: ValidatorSet, untrusted: SignedHeader,
                        untrusted_vals: ValidatorSet, trusting_period_ns: int, now_ns: int, drift_ns: int,
                        trust=(1, 3)) -> Optional[LightError]:
    e = _check_required(trusted)
    if e:
        return LightError(OTHER, e)
    if untrusted.header.height == trusted.header.height + 1:
        return LightError(OTHER, "headers must be non adjacent in height")
    e = validate_trust_level(*trust)
    if e:
        return LightError(OTHER, e)
    if _header_expired(untrusted.header, trusting_period_ns, now_ns):
        return _expired(untrusted, trusting_period_ns, now_ns)
    e = _verify_new_header_and_vals(untrusted, untrusted_vals, trusted, now_ns, drift_ns)
    if e:
        return LightError(INVALID_HEADER, "invalid header: " + e)
    ce = verify_commit_light_trusting(trusted.header.chain_id, trusted_vals, untrusted.commit, trust)
    if ce is not None:
        if ce.not_enough:
            return LightError(CANT_TRUST, "cant trust new val set: " + ce.text)
        return LightError(INVALID_HEADER, "invalid header: " + ce.text)
    ce = verify_commit_light(trusted.header.chain_id, untrusted_vals, untrusted.commit.block_id,
                             untrusted.header.height, untrusted.commit)
    if ce is not None:
        return LightError(INVALID_HEADER, "invalid header: " + ce.text)
    return None


def verify_adjacent(trusted: SignedHeader, untrusted: SignedHeader, untrusted_vals: ValidatorSet,
                    trusting_period_ns: int, now_ns: int, drift_ns: int) -> Optional[LightError]:
    e = _check_required(trusted)
    if e:
        return LightError(OTHER, e)
    if not trusted.header.next_validators_hash:
        return LightError(OTHER, "next validators hash in trusted header is empty")
    if untrusted.header.height != trusted.header.height + 1:
        return LightError(OTHER, "headers must be adjacent in height")
    if _header_expired(untrusted.header, trusting_period_ns, now_ns):
        return _expired(untrusted, trusting_period_ns, now_ns)
    e = _verify_new_header_and_vals(untrusted, untrusted_vals, trusted, now_ns, drift_ns)
    if e:
        return LightError(INVALID_HEADER, "invalid header: " + e)
    if untrusted.header.validators_hash != trusted.header.next_validators_hash:
        return LightError(INVALID_HEADER, "invalid header: expected old header's next validators (%s) to match "
                                          "those from new header (%s)" % (hexu(trusted.header.next_validators_hash),
                                                                          hexu(untrusted.header.validators_hash)))
    ce = verify_commit_light(trusted.header.chain_id, untrusted_vals, untrusted.commit.block_id,
                             untrusted.header.height, untrusted.commit)
    if ce is not None:
        return LightError(INVALID_HEADER, "invalid header: " + ce.text)
    return None


def verify(trusted: SignedHeader, trusted_vals: ValidatorSet, untrusted: SignedHeader,
           untrusted_vals: ValidatorSet, trusting_period_ns: int, now_ns: int, drift_ns: int,
           trust=(1, 3)) -> Optional[LightError]:
    """light.Verify (light/verifier.go:158-177)."""
    if untrusted.header.height != trusted.header.height + 1:
        return verify_non_adjacent(trusted, trusted_vals, untrusted, untrusted_vals, trusting_period_ns, now_ns,
                                   drift_ns, trust)
    return verify_adjacent(trusted, untrusted, untrusted_vals, trusting_period_ns, now_ns, drift_ns)


# ------------------------------------------------------------------ light/client.go drivers
@dataclass
class LightBlock:
    signed_header: SignedHeader
    vals: ValidatorSet


def verify_sequential(trusted: LightBlock, blocks: List[LightBlock], trusting_period_ns: int, now_ns: int,
                      drift_ns: int) -> Tuple[int, Optional[Tuple[int, int, LightError]]]:
    """Client.verifySequential's loop (light/client.go:567-626) with a single
    primary: VerifyAdjacent per height; returns (headers verified,
    (from, to, error) of ErrVerificationFailed or None)."""
    done = 0
    for lb in blocks:
        e = verify_adjacent(trusted.signed_header, lb.signed_header, lb.vals, trusting_period_ns, now_ns, drift_ns)
        if e is not None:
            return done, (trusted.signed_header.header.height, lb.signed_header.header.height, e)
        trusted = lb
        done += 1
    return done, None


def schedule(last_verified: int, last_failed: int) -> int:
    """Client.schedule: verifySkippingNumerator/Denominator = 9/16 (light/client.go:45-46,721-725)."""
    return last_verified + (last_failed - last_verified) * 9 // 16


def verify_skipping(trusted: LightBlock, target: LightBlock, provider: Callable[[int], LightBlock],
                    trusting_period_ns: int, now_ns: int, drift_ns: int, trust=(1, 3)):
    """Client.verifySkipping (light/client.go:647-727): returns (trace heights,
    None) or (None, (from, to, error))."""
    cache = [target]
    depth = 0
    verified = trusted
    trace = [trusted.signed_header.header.height]
    while True:
        cand = cache[depth]
        e = verify(verified.signed_header, verified.vals, cand.signed_header, cand.vals, trusting_period_ns,
                   now_ns, drift_ns, trust)
        if e is None:
            if depth == 0:
                trace.append(target.signed_header.header.height)
                return trace, None
            verified = cand
            cache = cache[:depth]
            depth = 0
            trace.append(verified.signed_header.header.height)
        elif e.kind == CANT_TRUST:
            if depth == len(cache) - 1:
                pivot = schedule(verified.signed_header.header.height, cache[depth].signed_header.header.height)
                try:
                    cache.append(provider(pivot))
                except Exception as pe:  # light/client.go:706-709: the provider's error, wrapped
                    return None, (verified.signed_header.header.height, pivot, LightError(OTHER, str(pe)))
            depth += 1
        else:
            return None, (verified.signed_header.header.height, cand.signed_header.header.height, e)


def sha256(b: bytes) -> bytes:
    return hashlib.sha256(b).digest()
