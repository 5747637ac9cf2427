"""Python view of the C++ host layer (include/tmhost.h): the types the
reference's commit verification works on, and thin ctypes calls into
libtmgpu.so's tmv_verify_commit / tmv_vote_sign_bytes / tmv_batch_*.

Mirrors (names and argument meaning):
  crypto.BatchVerifier / batch.CreateBatchVerifier  -> BatchVerifier / create_batch_verifier
  types.VerifyCommit / VerifyCommitLight / VerifyCommitLightTrusting
                                                   -> verify_commit / verify_commit_light /
                                                      verify_commit_light_trusting
Errors are returned as strings (None = ok), byte-identical to the Go error
text; infrastructure failures raise NativeError.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field
from typing import List, Optional, Tuple

from . import _native
from ._native import NativeError, TMV_KIND_ED25519, TMV_KIND_SR25519

KIND_OTHER = 255
BLOCK_ID_FLAG_ABSENT, BLOCK_ID_FLAG_COMMIT, BLOCK_ID_FLAG_NIL = 1, 2, 3
MODE_FULL, MODE_LIGHT, MODE_LIGHT_TRUSTING = 0, 1, 2
ZERO_TIME = (-62135596800, 0)

_u8p = ctypes.POINTER(ctypes.c_uint8)


class CBlockID(ctypes.Structure):
    _fields_ = [("hash", _u8p), ("hash_len", ctypes.c_uint32), ("psh_total", ctypes.c_uint32),
                ("psh_hash", _u8p), ("psh_hash_len", ctypes.c_uint32)]


class CValidator(ctypes.Structure):
    _fields_ = [("address", _u8p), ("address_len", ctypes.c_uint32), ("pub_key", _u8p),
                ("pub_key_len", ctypes.c_uint32), ("key_kind", ctypes.c_uint8), ("voting_power", ctypes.c_int64),
                ("proposer_priority", ctypes.c_int64)]


class CCommitSig(ctypes.Structure):
    _fields_ = [("block_id_flag", ctypes.c_uint8), ("validator_address", _u8p),
                ("validator_address_len", ctypes.c_uint32), ("ts_seconds", ctypes.c_int64),
                ("ts_nanos", ctypes.c_int32), ("signature", _u8p), ("signature_len", ctypes.c_uint32)]


class CCommit(ctypes.Structure):
    _fields_ = [("height", ctypes.c_int64), ("round", ctypes.c_int32), ("block_id", CBlockID),
                ("sigs", ctypes.POINTER(CCommitSig)), ("n_sigs", ctypes.c_uint32)]


@dataclass
class BlockID:
    hash: bytes = b""
    psh_total: int = 0
    psh_hash: bytes = b""

    def equals(self, o: "BlockID") -> bool:
        return (self.hash, self.psh_total, self.psh_hash) == (o.hash, o.psh_total, o.psh_hash)


@dataclass
class Validator:
    address: bytes
    pub_key: bytes
    voting_power: int
    key_kind: int = TMV_KIND_ED25519
    proposer_priority: int = 0


@dataclass
class ValidatorSet:
    validators: List[Validator]
    proposer_index: int = -1

    def total_voting_power(self) -> int:
        return sum(v.voting_power for v in self.validators)


@dataclass
class CommitSig:
    block_id_flag: int = BLOCK_ID_FLAG_ABSENT
    validator_address: bytes = b""
    timestamp: Tuple[int, int] = ZERO_TIME
    signature: bytes = b""


@dataclass
class Commit:
    height: int
    round: int
    block_id: BlockID
    signatures: List[CommitSig] = field(default_factory=list)


class _Keep:
    """Holds the ctypes buffers alive for the duration of a call."""

    def __init__(self):
        self.refs = []

    def buf(self, b: bytes):
        if not b:
            return None, 0
        a = (ctypes.c_uint8 * len(b)).from_buffer_copy(b)
        self.refs.append(a)
        return ctypes.cast(a, _u8p), len(b)


def _c_block_id(k: _Keep, b: BlockID) -> CBlockID:
    h, hl = k.buf(b.hash)
    p, pl = k.buf(b.psh_hash)
    return CBlockID(h, hl, b.psh_total, p, pl)


def _np_dtype(struct) -> "np.dtype":
    """numpy view of a ctypes Structure (pointers as uint64), same offsets."""
    import numpy as np
    conv = {ctypes.c_uint8: np.uint8, ctypes.c_uint32: np.uint32, ctypes.c_int32: np.int32,
            ctypes.c_int64: np.int64, ctypes.c_int: np.int32}
    names, formats, offsets = [], [], []
    for name, ty in struct._fields_:
        names.append(name)
        formats.append(conv.get(ty, np.uint64))
        offsets.append(getattr(struct, name).offset)
    return np.dtype({"names": names, "formats": formats, "offsets": offsets, "itemsize": ctypes.sizeof(struct)})


_DT = {}


def _dt(key, struct):
    d = _DT.get(key)
    if d is None:
        d = _DT[key] = _np_dtype(struct)
    return d


def _blob_ptrs(k: _Keep, items: List[bytes]):
    """Concatenate byte strings into one kept buffer; per-item (pointer, len),
    pointer NULL for an empty item (as _Keep.buf)."""
    import numpy as np
    blob = b"".join(items)
    lens = np.fromiter((len(x) for x in items), dtype=np.uint32, count=len(items))
    if not blob:
        return np.zeros(len(items), np.uint64), lens
    buf = np.frombuffer(blob, dtype=np.uint8)
    k.refs.append(blob)
    offs = np.zeros(len(items), np.uint64)
    np.cumsum(lens[:-1], out=offs[1:])
    ptrs = np.where(lens > 0, offs + np.uint64(buf.ctypes.data), np.uint64(0))
    return ptrs, lens


def _c_validators(k: _Keep, vals: ValidatorSet):
    """tmv_validator[] for a validator set, built column-wise."""
    import numpy as np
    dt = _dt("v", CValidator)
    vs = vals.validators
    a = np.zeros(max(1, len(vs)), dtype=dt)
    if vs:
        a["address"][:len(vs)], a["address_len"][:len(vs)] = _blob_ptrs(k, [v.address for v in vs])
        a["pub_key"][:len(vs)], a["pub_key_len"][:len(vs)] = _blob_ptrs(k, [v.pub_key for v in vs])
        a["key_kind"][:len(vs)] = [v.key_kind for v in vs]
        a["voting_power"][:len(vs)] = [v.voting_power for v in vs]
        a["proposer_priority"][:len(vs)] = [v.proposer_priority for v in vs]
    k.refs.append(a)
    return ctypes.cast(a.ctypes.data, ctypes.POINTER(CValidator))


def _c_commit(k: _Keep, commit: Commit) -> CCommit:
    """tmv_commit for a Commit; its tmv_commit_sig[] built column-wise."""
    import numpy as np
    dt = _dt("s", CCommitSig)
    ss = commit.signatures
    n = len(ss)
    a = np.zeros(max(1, n), dtype=dt)
    if n:
        a["block_id_flag"][:n] = [s.block_id_flag for s in ss]
        a["validator_address"][:n], a["validator_address_len"][:n] = _blob_ptrs(k, [s.validator_address for s in ss])
        a["ts_seconds"][:n] = [s.timestamp[0] for s in ss]
        a["ts_nanos"][:n] = [s.timestamp[1] for s in ss]
        a["signature"][:n], a["signature_len"][:n] = _blob_ptrs(k, [s.signature for s in ss])
    k.refs.append(a)
    c = CCommit(commit.height, commit.round, _c_block_id(k, commit.block_id),
                ctypes.cast(a.ctypes.data, ctypes.POINTER(CCommitSig)), n)
    k.refs.append(c)
    return c


def _setup(L):
    if getattr(L, "_tmhost_ready", False):
        return L
    L.tmv_vote_sign_bytes.restype = ctypes.c_size_t
    L.tmv_vote_sign_bytes.argtypes = [ctypes.c_char_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_int32,
                                      ctypes.POINTER(CBlockID), ctypes.c_int64, ctypes.c_int32, _u8p, ctypes.c_size_t]
    L.tmv_vote_template_encode.restype = ctypes.c_size_t
    L.tmv_vote_template_encode.argtypes = [ctypes.c_char_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_int32,
                                           ctypes.POINTER(CBlockID), _u8p, ctypes.c_size_t,
                                           ctypes.POINTER(ctypes.c_uint32)]
    L.tmv_verify_commit.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_char_p, ctypes.POINTER(CValidator),
                                    ctypes.c_uint32, ctypes.c_int32, ctypes.POINTER(CBlockID), ctypes.c_int64,
                                    ctypes.POINTER(CCommit), ctypes.c_int64, ctypes.c_int64, ctypes.c_char_p,
                                    ctypes.c_size_t]
    L.tmv_batch_new.restype = ctypes.c_void_p
    L.tmv_batch_new.argtypes = [ctypes.c_void_p, ctypes.c_uint8]
    L.tmv_batch_add.argtypes = [ctypes.c_void_p, ctypes.c_uint8, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p,
                                ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t]
    L.tmv_batch_len.restype = ctypes.c_size_t
    L.tmv_batch_len.argtypes = [ctypes.c_void_p]
    L.tmv_batch_verify.argtypes = [ctypes.c_void_p, _u8p, ctypes.POINTER(ctypes.c_int64), ctypes.c_char_p,
                                   ctypes.c_size_t]
    L.tmv_batch_free.argtypes = [ctypes.c_void_p]
    L._tmhost_ready = True
    return L


def vote_sign_bytes(chain_id: str, vote_type: int, height: int, round_: int, block_id: Optional[BlockID],
                    timestamp: Tuple[int, int], lib=None) -> bytes:
    """types.VoteSignBytes through the C++ encoder (tmv_vote_sign_bytes)."""
    L = _setup(lib or _native.lib())
    k = _Keep()
    bid = ctypes.byref(_c_block_id(k, block_id)) if block_id is not None else None
    out = (ctypes.c_uint8 * 512)()
    n = L.tmv_vote_sign_bytes(chain_id.encode(), vote_type, height, round_, bid, timestamp[0], timestamp[1],
                              ctypes.cast(out, _u8p), 512)
    return bytes(out[:n])


def vote_template(chain_id: str, vote_type: int, height: int, round_: int, block_id: Optional[BlockID],
                  lib=None) -> Tuple[bytes, bytes, bytes]:
    """The (head, block, chain) segments of tmv_verify_votes' template through
    the C++ encoder (tmv_vote_template_encode)."""
    L = _setup(lib or _native.lib())
    k = _Keep()
    bid = ctypes.byref(_c_block_id(k, block_id)) if block_id is not None else None
    out = (ctypes.c_uint8 * 1024)()
    lens = (ctypes.c_uint32 * 3)()
    n = L.tmv_vote_template_encode(chain_id.encode(), vote_type, height, round_, bid, ctypes.cast(out, _u8p), 1024,
                                   lens)
    b = bytes(out[:n])
    h, k2 = lens[0], lens[0] + lens[1]
    return b[:h], b[h:k2], b[k2:]


def _commit_call(fn, ctx_handle, mode, chain_id, vals: Optional[ValidatorSet], block_id: Optional[BlockID],
                 height: int, commit: Optional[Commit], trust: Tuple[int, int]) -> Optional[str]:
    k = _Keep()
    cvals, nv, prop = None, 0, -1
    if vals is not None:
        cvals, nv, prop = _c_validators(k, vals), len(vals.validators), vals.proposer_index
    ccommit = ctypes.byref(_c_commit(k, commit)) if commit is not None else None
    bid = ctypes.byref(_c_block_id(k, block_id)) if block_id is not None else None
    err = ctypes.create_string_buffer(4096)
    rc = fn(ctx_handle, mode, chain_id.encode(), cvals, nv, prop, bid, height, ccommit, trust[0], trust[1], err,
            len(err))
    if rc < 0:
        raise NativeError(f"commit verification failed ({rc}): {err.value.decode(errors='replace')}")
    return err.value.decode() if rc == 1 else None


def verify_commit(ctx, chain_id: str, vals, block_id, height, commit) -> Optional[str]:
    L = _setup(_native.lib())
    return _commit_call(L.tmv_verify_commit, ctx.handle, MODE_FULL, chain_id, vals, block_id, height, commit, (0, 1))


def verify_commit_light(ctx, chain_id: str, vals, block_id, height, commit) -> Optional[str]:
    L = _setup(_native.lib())
    return _commit_call(L.tmv_verify_commit, ctx.handle, MODE_LIGHT, chain_id, vals, block_id, height, commit, (0, 1))


def verify_commit_light_trusting(ctx, chain_id: str, vals, commit, trust_level=(1, 3)) -> Optional[str]:
    L = _setup(_native.lib())
    return _commit_call(L.tmv_verify_commit, ctx.handle, MODE_LIGHT_TRUSTING, chain_id, vals, None, 0, commit,
                        trust_level)


class BatchVerifier:
    """crypto.BatchVerifier over tmv_batch_* (crypto/crypto.go:66-76).
    `lib` / a raw context handle select another library exporting the same
    C-ABI (the CPU test harness)."""

    def __init__(self, ctx, key_kind: int, lib=None):
        self._L = _setup(lib or _native.lib())
        self._h = self._L.tmv_batch_new(getattr(ctx, "handle", ctx), key_kind)
        if not self._h:
            raise NativeError("no batch verifier for this key type")
        self.deferred_add_error: Optional[Tuple[int, str]] = None

    def add(self, key_kind: int, pub_key: bytes, msg: bytes, sig: bytes) -> Optional[str]:
        err = ctypes.create_string_buffer(512)
        rc = self._L.tmv_batch_add(self._h, key_kind, pub_key, len(pub_key), msg, len(msg), sig, len(sig), err, 512)
        if rc < 0:
            raise NativeError("tmv_batch_add failed")
        return err.value.decode() if rc == 1 else None

    def __len__(self):
        return self._L.tmv_batch_len(self._h)

    def verify(self) -> Tuple[bool, List[bool]]:
        n = len(self)
        out = (ctypes.c_uint8 * max(1, n))()
        idx = ctypes.c_int64(-1)
        err = ctypes.create_string_buffer(512)
        rc = self._L.tmv_batch_verify(self._h, ctypes.cast(out, _u8p), ctypes.byref(idx), err, 512)
        if rc < 0:
            raise NativeError(f"tmv_batch_verify failed ({rc}): {err.value.decode(errors='replace')}")
        self.deferred_add_error = (idx.value, err.value.decode()) if rc == 2 else None
        return rc == 1, [bool(out[i]) for i in range(n)]

    def __del__(self):
        try:
            if self._h:
                self._L.tmv_batch_free(self._h)
        except Exception:
            pass


def create_batch_verifier(ctx, key_kind: int, lib=None) -> Optional[BatchVerifier]:
    """batch.CreateBatchVerifier (crypto/batch/batch.go:11-21): None for key
    types without batch support (the C-ABI returns NULL for them)."""
    try:
        return BatchVerifier(ctx, key_kind, lib)
    except NativeError:
        return None


def supports_batch_verifier(key_kind: int) -> bool:
    return key_kind in (TMV_KIND_ED25519, TMV_KIND_SR25519)


class PreparedCommitCall:
    """A tmv_verify_commit call with its C structs built once (for timing the
    L3 path without Python marshalling in the loop)."""

    def __init__(self, ctx, mode, chain_id, vals, block_id, height, commit, trust=(0, 1)):
        L = _setup(_native.lib())
        self._L, self._ctx = L, ctx
        k = _Keep()
        arr = _c_validators(k, vals)
        cc = _c_commit(k, commit)
        bid = _c_block_id(k, block_id) if block_id is not None else None
        self._keep = (k, arr, cc, bid)
        self._args = (mode, chain_id.encode(), arr, len(vals.validators), vals.proposer_index,
                      ctypes.byref(bid) if bid is not None else None, height, ctypes.byref(cc), trust[0], trust[1])
        self._err = ctypes.create_string_buffer(4096)

    def __call__(self) -> Optional[str]:
        rc = self._L.tmv_verify_commit(self._ctx.handle, *self._args, self._err, len(self._err))
        if rc < 0:
            raise NativeError(f"tmv_verify_commit failed ({rc}): {self._err.value.decode(errors='replace')}")
        return self._err.value.decode() if rc == 1 else None


class CCommitJob(ctypes.Structure):
    _fields_ = [("mode", ctypes.c_int), ("chain_id", ctypes.c_char_p), ("vals", ctypes.POINTER(CValidator)),
                ("n_vals", ctypes.c_uint32), ("proposer_index", ctypes.c_int32),
                ("block_id", ctypes.POINTER(CBlockID)), ("height", ctypes.c_int64),
                ("commit", ctypes.POINTER(CCommit)), ("trust_num", ctypes.c_int64), ("trust_den", ctypes.c_int64)]


@dataclass
class CommitJob:
    """One commit check: mode MODE_FULL / MODE_LIGHT / MODE_LIGHT_TRUSTING."""
    mode: int
    chain_id: str
    vals: Optional[ValidatorSet]
    block_id: Optional[BlockID]
    height: int
    commit: Optional[Commit]
    trust: Tuple[int, int] = (1, 3)


class PreparedJobs:
    """C structs for a list of CommitJob, built once.  Jobs that share a
    Commit object (by identity) share one tmv_commit, so the engine verifies
    their common signatures once (blocksync checks each commit twice)."""

    def __init__(self, jobs: List[CommitJob]):
        k = _Keep()
        vcache, ccache = {}, {}
        arr = (CCommitJob * max(1, len(jobs)))()
        for j, jb in enumerate(jobs):
            cv, nv, prop = None, 0, -1
            if jb.vals is not None:
                key = id(jb.vals)
                if key not in vcache:
                    vcache[key] = _c_validators(k, jb.vals)
                cv, nv, prop = vcache[key], len(jb.vals.validators), jb.vals.proposer_index
            cc = None
            if jb.commit is not None:
                key = id(jb.commit)
                if key not in ccache:
                    ccache[key] = _c_commit(k, jb.commit)
                cc = ctypes.pointer(ccache[key])
            bid = None
            if jb.block_id is not None:
                b = _c_block_id(k, jb.block_id)
                k.refs.append(b)
                bid = ctypes.pointer(b)
            cid = jb.chain_id.encode()
            k.refs.append(cid)
            arr[j] = CCommitJob(jb.mode, cid, cv, nv, prop, bid, jb.height, cc, jb.trust[0], jb.trust[1])
        self.keep = (k, vcache, ccache)
        self.arr = arr
        self.n = len(jobs)
        self.stride = 512
        self.errs = ctypes.create_string_buffer(self.stride * max(1, self.n))
        self.results = (ctypes.c_int32 * max(1, self.n))()

    def decode(self) -> List[Optional[str]]:
        out = []
        buf = None  # one copy of the error buffer (ctypes' .raw copies all of it on every access)
        for j in range(self.n):
            if self.results[j]:
                if buf is None:
                    buf = self.errs.raw
                out.append(buf[j * self.stride:(j + 1) * self.stride].split(b"\0", 1)[0].decode())
            else:
                out.append(None)
        return out


def _setup_many(L):
    if not getattr(L, "_tmhost_many", False):
        L.tmv_verify_commits.argtypes = [ctypes.c_void_p, ctypes.POINTER(CCommitJob), ctypes.c_uint32,
                                         ctypes.POINTER(ctypes.c_int32), ctypes.c_char_p, ctypes.c_size_t]
        L._tmhost_many = True
    return L


def run_prepared_jobs(ctx, pj: PreparedJobs) -> int:
    L = _setup_many(_setup(_native.lib()))
    rc = L.tmv_verify_commits(ctx.handle, pj.arr, pj.n, pj.results, pj.errs, pj.stride)
    if rc < 0:
        raise NativeError(f"tmv_verify_commits failed ({rc}): {_native.last_error()}")
    return rc


def verify_commits(ctx, jobs: List[CommitJob]) -> List[Optional[str]]:
    """Cross-commit batching: every job's result equals verify_commit* of that
    job alone; all signatures go to the GPU in one batch."""
    pj = PreparedJobs(jobs)
    run_prepared_jobs(ctx, pj)
    return pj.decode()


# ---------------------------------------------------------------- light client
# light.Verify / VerifyAdjacent / VerifyNonAdjacent (light/verifier.go:33-177)
# and Header.Hash (types/block.go:447-478) through tmv_light_verify_many /
# tmv_header_hashes (include/tmhost.h).

LIGHT_VERIFY, LIGHT_ADJACENT, LIGHT_NON_ADJACENT = 0, 1, 2
LIGHT_OK, LIGHT_ERR_INVALID_HEADER, LIGHT_ERR_OLD_HEADER_EXPIRED, LIGHT_ERR_CANT_TRUST, LIGHT_ERR_OTHER = 0, 1, 2, 3, 4
BLOCK_PROTOCOL = 11  # version/version.go:27


class CBytes(ctypes.Structure):
    _fields_ = [("p", _u8p), ("len", ctypes.c_uint32)]


_HASH_FIELDS = ("last_commit_hash", "data_hash", "validators_hash", "next_validators_hash", "consensus_hash",
                "app_hash", "last_results_hash", "evidence_hash", "proposer_address")


class CHeader(ctypes.Structure):
    _fields_ = ([("version_block", ctypes.c_uint64), ("version_app", ctypes.c_uint64), ("chain_id", ctypes.c_char_p),
                 ("height", ctypes.c_int64), ("time_seconds", ctypes.c_int64), ("time_nanos", ctypes.c_int32),
                 ("last_block_id", CBlockID)] + [(f, CBytes) for f in _HASH_FIELDS])


class CSignedHeader(ctypes.Structure):
    _fields_ = [("header", ctypes.POINTER(CHeader)), ("commit", ctypes.POINTER(CCommit))]


class CValidatorSet(ctypes.Structure):
    _fields_ = [("vals", ctypes.POINTER(CValidator)), ("n_vals", ctypes.c_uint32), ("proposer_index", ctypes.c_int32)]


class CLightJob(ctypes.Structure):
    _fields_ = [("mode", ctypes.c_int), ("trusted", ctypes.POINTER(CSignedHeader)),
                ("trusted_vals", ctypes.POINTER(CValidatorSet)), ("untrusted", ctypes.POINTER(CSignedHeader)),
                ("untrusted_vals", ctypes.POINTER(CValidatorSet)), ("trusting_period_ns", ctypes.c_int64),
                ("now_seconds", ctypes.c_int64), ("now_nanos", ctypes.c_int32),
                ("max_clock_drift_ns", ctypes.c_int64), ("trust_num", ctypes.c_uint64),
                ("trust_den", ctypes.c_uint64)]


@dataclass
class Header:
    """types.Header (types/block.go:338-366)."""
    chain_id: str
    height: int
    time: Tuple[int, int]
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
    version_block: int = BLOCK_PROTOCOL
    version_app: int = 0


@dataclass
class SignedHeader:
    """types.SignedHeader (types/light.go:131-136)."""
    header: Optional[Header]
    commit: Optional[Commit]

    @property
    def height(self) -> int:
        return self.header.height


@dataclass
class LightBlock:
    """types.LightBlock: a signed header and the validator set at its height."""
    signed_header: SignedHeader
    vals: ValidatorSet
    next_vals: Optional[ValidatorSet] = None

    @property
    def height(self) -> int:
        return self.signed_header.header.height


@dataclass
class LightJob:
    """One light-client verification (the arguments of light.Verify)."""
    trusted: SignedHeader
    trusted_next_vals: Optional[ValidatorSet]
    untrusted: SignedHeader
    untrusted_vals: Optional[ValidatorSet]
    trusting_period_ns: int
    now: Tuple[int, int]
    max_clock_drift_ns: int = 10 * 10**9  # light/client.go:52 defaultMaxClockDrift
    trust: Tuple[int, int] = (1, 3)       # light.DefaultTrustLevel
    mode: int = LIGHT_VERIFY


def _c_bytes(k: _Keep, b: bytes) -> CBytes:
    p, n = k.buf(b)
    return CBytes(p, n)


def _c_header(k: _Keep, h: Header) -> CHeader:
    cid = h.chain_id.encode()
    k.refs.append(cid)
    c = CHeader(h.version_block, h.version_app, cid, h.height, h.time[0], h.time[1], _c_block_id(k, h.last_block_id),
                *[_c_bytes(k, getattr(h, f)) for f in _HASH_FIELDS])
    k.refs.append(c)
    return c


class PreparedLightJobs:
    """C structs for a list of LightJob, built once; headers, commits and
    validator sets shared by object identity are passed once (the engine
    converts and hashes each distinct one once)."""

    def __init__(self, jobs: List[LightJob]):
        k = _Keep()
        hcache, ccache, vcache, shcache = {}, {}, {}, {}

        def header(h):
            if h is None:
                return None
            if id(h) not in hcache:
                hcache[id(h)] = (h, ctypes.pointer(_c_header(k, h)))
            return hcache[id(h)][1]

        def commit(c):
            if c is None:
                return None
            if id(c) not in ccache:
                cc = _c_commit(k, c)
                ccache[id(c)] = (c, ctypes.pointer(cc))
            return ccache[id(c)][1]

        def signed(sh):
            if sh is None:
                return None
            if id(sh) not in shcache:
                s = CSignedHeader(header(sh.header), commit(sh.commit))
                k.refs.append(s)
                shcache[id(sh)] = (sh, ctypes.pointer(s))
            return shcache[id(sh)][1]

        def vset(vs):
            if vs is None:
                return None
            if id(vs) not in vcache:
                s = CValidatorSet(_c_validators(k, vs), len(vs.validators), vs.proposer_index)
                k.refs.append(s)
                vcache[id(vs)] = (vs, ctypes.pointer(s))
            return vcache[id(vs)][1]

        arr = (CLightJob * max(1, len(jobs)))()
        for j, jb in enumerate(jobs):
            arr[j] = CLightJob(jb.mode, signed(jb.trusted), vset(jb.trusted_next_vals), signed(jb.untrusted),
                               vset(jb.untrusted_vals), jb.trusting_period_ns, jb.now[0], jb.now[1],
                               jb.max_clock_drift_ns, jb.trust[0], jb.trust[1])
        self.keep = (k, hcache, ccache, vcache, shcache)
        self.arr, self.n = arr, len(jobs)
        self.stride = 1024
        self.errs = ctypes.create_string_buffer(self.stride * max(1, self.n))
        self.results = (ctypes.c_int32 * max(1, self.n))()

    def decode(self) -> List[Tuple[int, Optional[str]]]:
        out = []
        buf = None  # one copy of the error buffer (ctypes' .raw copies all of it on every access)
        for j in range(self.n):
            kind = self.results[j]
            if kind == LIGHT_OK:
                out.append((kind, None))
                continue
            if buf is None:
                buf = self.errs.raw
            out.append((kind, buf[j * self.stride:(j + 1) * self.stride].split(b"\0", 1)[0].decode()))
        return out


def _setup_light(L):
    if not getattr(L, "_tmhost_light", False):
        L.tmv_light_verify_many.argtypes = [ctypes.c_void_p, ctypes.POINTER(CLightJob), ctypes.c_uint32,
                                            ctypes.POINTER(ctypes.c_int32), ctypes.c_char_p, ctypes.c_size_t]
        L.tmv_header_hashes.argtypes = [ctypes.c_void_p, ctypes.POINTER(CHeader), ctypes.c_uint32, _u8p, _u8p]
        L._tmhost_light = True
    return L


def run_light_jobs(fn, ctx_handle, pj: PreparedLightJobs) -> List[Tuple[int, Optional[str]]]:
    """fn = tmv_light_verify_many (or the CPU harness's twin)."""
    rc = fn(ctx_handle, pj.arr, pj.n, pj.results, pj.errs, pj.stride)
    if rc < 0:
        raise NativeError(f"tmv_light_verify_many failed ({rc}): {_native.last_error()}")
    return pj.decode()


def light_verify_many(ctx, jobs: List[LightJob]) -> List[Tuple[int, Optional[str]]]:
    """Each job's (TMV_LIGHT_* class, error text or None), all jobs in one pass."""
    L = _setup_light(_setup(_native.lib()))
    return run_light_jobs(L.tmv_light_verify_many, ctx.handle, PreparedLightJobs(jobs))


def light_verify(ctx, job: LightJob) -> Tuple[int, Optional[str]]:
    return light_verify_many(ctx, [job])[0]


def header_hashes_call(fn, ctx_handle, headers: List[Header]) -> List[Optional[bytes]]:
    k = _Keep()
    arr = (CHeader * max(1, len(headers)))()
    for i, h in enumerate(headers):
        arr[i] = _c_header(k, h)
    out = (ctypes.c_uint8 * (32 * max(1, len(headers))))()
    has = (ctypes.c_uint8 * max(1, len(headers)))()
    rc = fn(ctx_handle, arr, len(headers), ctypes.cast(out, _u8p), ctypes.cast(has, _u8p))
    if rc < 0:
        raise NativeError(f"tmv_header_hashes failed ({rc})")
    return [bytes(out[32 * i:32 * i + 32]) if has[i] else None for i in range(len(headers))]


def header_hashes(ctx, headers: List[Header]) -> List[Optional[bytes]]:
    """Header.Hash of each header (None where the reference returns nil)."""
    L = _setup_light(_setup(_native.lib()))
    return header_hashes_call(L.tmv_header_hashes, ctx.handle, headers)


# ---------------------------------------------------------------- consensus votes (ADR-064)
VOTE_OK, VOTE_ERR_INVALID_ADDRESS, VOTE_ERR_INVALID_SIGNATURE = 0, 1, 2
PREVOTE_TYPE, PRECOMMIT_TYPE = 1, 2


class CVoteIn(ctypes.Structure):
    _fields_ = [("type", ctypes.c_int32), ("height", ctypes.c_int64), ("round", ctypes.c_int32),
                ("block_id", ctypes.POINTER(CBlockID)), ("ts_seconds", ctypes.c_int64), ("ts_nanos", ctypes.c_int32),
                ("validator_address", _u8p), ("validator_address_len", ctypes.c_uint32),
                ("signature", _u8p), ("signature_len", ctypes.c_uint32), ("key_kind", ctypes.c_uint8),
                ("pub_key", _u8p), ("pub_key_len", ctypes.c_uint32)]


@dataclass
class Vote:
    """types.Vote (types/vote.go:50-62), the fields consensus votes carry."""
    type: int
    height: int
    round: int
    block_id: BlockID
    timestamp: Tuple[int, int]
    validator_address: bytes
    validator_index: int
    signature: bytes = b""


def verify_vote_batch_call(fn, ctx_handle, chain_id: str, votes: List[Vote], keys: List[Tuple[int, bytes]]
                           ) -> List[int]:
    """votes[i] checked against keys[i] = (key kind, public key); fn =
    tmv_verify_vote_batch (or the CPU harness's twin).  Returns TMV_VOTE_* per vote."""
    k = _Keep()
    arr = (CVoteIn * max(1, len(votes)))()
    for i, (v, (kind, pk)) in enumerate(zip(votes, keys)):
        bid = None
        if v.block_id is not None and (v.block_id.hash or v.block_id.psh_total or v.block_id.psh_hash):
            b = _c_block_id(k, v.block_id)
            k.refs.append(b)
            bid = ctypes.pointer(b)
        a, al = k.buf(v.validator_address)
        s, sl = k.buf(v.signature)
        p, pl = k.buf(pk)
        arr[i] = CVoteIn(v.type, v.height, v.round, bid, v.timestamp[0], v.timestamp[1], a, al, s, sl, kind, p, pl)
    res = (ctypes.c_int32 * max(1, len(votes)))()
    rc = fn(ctx_handle, chain_id.encode(), arr, len(votes), res)
    if rc < 0:
        raise NativeError(f"tmv_verify_vote_batch failed ({rc}): {_native.last_error()}")
    return [res[i] for i in range(len(votes))]


def verify_vote_batch(ctx, chain_id: str, votes: List[Vote], keys: List[Tuple[int, bytes]]) -> List[int]:
    L = _setup(_native.lib())
    if not getattr(L, "_tmhost_votes", False):
        L.tmv_verify_vote_batch.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.POINTER(CVoteIn),
                                            ctypes.c_uint32, ctypes.POINTER(ctypes.c_int32)]
        L._tmhost_votes = True
    return verify_vote_batch_call(L.tmv_verify_vote_batch, ctx.handle, chain_id, votes, keys)
