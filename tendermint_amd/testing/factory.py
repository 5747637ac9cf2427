"""Deterministic synthetic workloads for the configs of BASELINE.json.

Keys follow the reference's test convention GenPrivKeyFromSecret
(crypto/ed25519/ed25519.go:162-165: seed = SHA-256(secret)) with secrets
"key: %x" (types/validator_set_test.go:1621-1631).  Messages are real
commit-vote sign-bytes (types/block.go:859-862), 109-125 bytes.

C2: 10,000 ed25519 signatures, seed 0xED25519, 9,900 honest
plus 100 edge cases: 20 bit flips (R/S/M), 15 S+l, 15 undecodable R or A
(all invalid), 20 small-order (A, R) with S = 0, 15 non-canonical (y >= p)
torsion encodings, 15 "-0" sign-bit encodings (all VALID under ZIP-215).
"""
from __future__ import annotations

import hashlib
import random
from dataclasses import dataclass, field
from typing import List, Tuple

import numpy as np

from ..types.canonical import BlockID, PartSetHeader, Timestamp, vote_sign_bytes, PRECOMMIT_TYPE
from ._openssl import Ed25519Signer

P = 2**255 - 19
L = 2**252 + 27742317777372353535851937790883648493
_D = (-121665 * pow(121666, P - 2, P)) % P

# The 14 ZIP-215 small-order encodings, derived by
# oracle/ed25519_ref.small_order_encodings() and pinned in
# tests/golden/zip215_small_order.json.
SMALL_ORDER_CANONICAL = [
    bytes(32),                                   # (0, 0) order 4 family: y = 0
    bytes.fromhex("01" + "00" * 31),             # identity
    bytes.fromhex("26e8958fc2b227b045c3f489f2ef98f0d5dfac05d3c63339b13802886d53fc05"),
    bytes.fromhex("26e8958fc2b227b045c3f489f2ef98f0d5dfac05d3c63339b13802886d53fc85"),
    bytes.fromhex("c7176a703d4dd84fba3c0b760d10670f2a2053fa2c39ccc64ec7fd7792ac037a"),
    bytes.fromhex("c7176a703d4dd84fba3c0b760d10670f2a2053fa2c39ccc64ec7fd7792ac03fa"),
    bytes.fromhex("ec" + "ff" * 30 + "7f"),      # order 2 (y = -1)
    bytes.fromhex("00" * 31 + "80"),             # y = 0, sign 1
]
SMALL_ORDER_NONCANONICAL_Y = [                   # y >= p
    bytes.fromhex("ed" + "ff" * 30 + "7f"),
    bytes.fromhex("ed" + "ff" * 31),
    bytes.fromhex("ee" + "ff" * 30 + "7f"),
    bytes.fromhex("ee" + "ff" * 31),
]
SMALL_ORDER_NEG_ZERO = [                          # x = 0 with the sign bit set
    bytes.fromhex("01" + "00" * 30 + "80"),
    bytes.fromhex("ec" + "ff" * 31),
]


def key_seed(i: int, tag: str = "key") -> bytes:
    """GenPrivKeyFromSecret([]byte(fmt.Sprintf("key: %x", i))) seed."""
    return hashlib.sha256(f"{tag}: {i:x}".encode()).digest()


def _is_square(x: int) -> bool:
    return x == 0 or pow(x, (P - 1) // 2, P) == 1


def undecodable_encodings(count: int, rng: random.Random) -> List[bytes]:
    """Encodings whose y gives a non-square (y^2-1)/(d y^2+1): rejected by ZIP-215 decoding."""
    out = []
    while len(out) < count:
        y = rng.randrange(P)
        u = (y * y - 1) % P
        v = (_D * y * y + 1) % P
        if not _is_square(u * pow(v, P - 2, P) % P):
            out.append(int.to_bytes(y | (rng.randrange(2) << 255), 32, "little"))
    return out


@dataclass
class Batch:
    pk: np.ndarray        # n*32 uint8
    sig: np.ndarray       # n*64 uint8
    msg: np.ndarray       # concatenated uint8
    off: np.ndarray       # n+1 uint32
    kinds: List[str] = field(default_factory=list)  # per-entry label (for tests)

    @property
    def n(self) -> int:
        return len(self.off) - 1

    @staticmethod
    def from_entries(entries: List[Tuple[bytes, bytes, bytes]], kinds=None) -> "Batch":
        n = len(entries)
        pk = np.frombuffer(b"".join(e[0] for e in entries), np.uint8).copy() if n else np.zeros(0, np.uint8)
        sig = np.frombuffer(b"".join(e[2] for e in entries), np.uint8).copy() if n else np.zeros(0, np.uint8)
        off = np.zeros(n + 1, np.uint32)
        if n:
            off[1:] = np.cumsum([len(e[1]) for e in entries])
        m = b"".join(e[1] for e in entries)
        msg = np.frombuffer(m, np.uint8).copy() if m else np.zeros(0, np.uint8)
        return Batch(pk, sig, msg, off, list(kinds) if kinds else ["honest"] * n)

    def entry(self, i: int) -> Tuple[bytes, bytes, bytes]:
        return (self.pk[32 * i:32 * i + 32].tobytes(), self.msg[self.off[i]:self.off[i + 1]].tobytes(),
                self.sig[64 * i:64 * i + 64].tobytes())

    @staticmethod
    def concat(batches) -> "Batch":
        """Entries of several batches in order, as one batch."""
        pk = np.concatenate([b.pk for b in batches])
        sig = np.concatenate([b.sig for b in batches])
        msg = np.concatenate([b.msg for b in batches])
        lens = np.concatenate([b.off[1:] - b.off[:-1] for b in batches])
        off = np.zeros(len(lens) + 1, np.uint32)
        off[1:] = np.cumsum(lens)
        return Batch(pk, sig, msg, off, [k for b in batches for k in b.kinds])

    def take(self, idx) -> "Batch":
        """Entries idx[0], idx[1], ... (any order, repeats allowed), vectorised."""
        idx = np.asarray(idx, np.int64)
        lens = (self.off[1:] - self.off[:-1]).astype(np.int64)[idx]
        off = np.zeros(len(idx) + 1, np.uint32)
        off[1:] = np.cumsum(lens)
        starts = self.off[:-1].astype(np.int64)[idx]
        pos = np.arange(int(off[-1]), dtype=np.int64) - np.repeat(off[:-1].astype(np.int64), lens) + \
            np.repeat(starts, lens)
        return Batch(self.pk.reshape(-1, 32)[idx].reshape(-1), self.sig.reshape(-1, 64)[idx].reshape(-1),
                     self.msg[pos] if len(pos) else np.zeros(0, np.uint8), off,
                     [self.kinds[i] for i in idx] if self.kinds else [])

    def tile(self, n: int) -> "Batch":
        """Repeat entries cyclically up to n (throughput runs on >10k)."""
        idx = np.arange(n) % self.n
        pk = self.pk.reshape(-1, 32)[idx].reshape(-1)
        sig = self.sig.reshape(-1, 64)[idx].reshape(-1)
        lens = (self.off[1:] - self.off[:-1])[idx]
        off = np.zeros(n + 1, np.uint32)
        off[1:] = np.cumsum(lens)
        msg = np.concatenate([self.msg[self.off[i]:self.off[i + 1]] for i in idx]) if n else np.zeros(0, np.uint8)
        return Batch(pk, sig, msg, off, [self.kinds[i] for i in idx])


def commit_vote_message(chain_id: str, height: int, round_: int, block_id: BlockID, secs: int, nanos: int) -> bytes:
    return vote_sign_bytes(chain_id, PRECOMMIT_TYPE, height, round_, block_id, Timestamp(secs, nanos))


def random_block_id(rng: random.Random) -> BlockID:
    return BlockID(bytes(rng.randrange(256) for _ in range(32)),
                   PartSetHeader(rng.randrange(1, 1 << 16), bytes(rng.randrange(256) for _ in range(32))))


C2_VALID_KINDS = ("honest", "small_order", "noncanonical_y", "neg_zero")  # valid under ZIP-215


def _c2_plan(n: int, seed: int, edge_scale: float):
    rng = random.Random(seed)
    counts = {"bitflip": 20, "s_plus_l": 15, "undecodable": 15, "small_order": 20,
              "noncanonical_y": 15, "neg_zero": 15}
    counts = {k: max(1, int(round(v * edge_scale * n / 10_000))) if n >= 100 else 0 for k, v in counts.items()}
    kinds = []
    for k, c in counts.items():
        kinds += [k] * c
    kinds += ["honest"] * (n - len(kinds))
    rng.shuffle(kinds)
    return rng, counts, kinds


def c2_kinds(n: int = 10_000, seed: int = 0xED25519, edge_scale: float = 1.0) -> List[str]:
    """The per-entry kinds make_c2_batch(n, seed) assigns, without signing
    anything: its exact validity vector is [k in C2_VALID_KINDS for k in
    c2_kinds(...)] (bench.py's strong-scaling leg checks a gathered 1M
    vector on every rank against it)."""
    return _c2_plan(n, seed, edge_scale)[2]


def make_c2_batch(n: int = 10_000, seed: int = 0xED25519, chain_id: str = "test_chain_id",
                  edge_scale: float = 1.0) -> Batch:
    """Config 2: n ed25519 signatures over commit-vote sign-bytes, 1% edge cases."""
    rng, counts, kinds = _c2_plan(n, seed, edge_scale)
    block_id = random_block_id(rng)
    base_secs = 1577836800  # 2020-01-01T00:00:00Z
    undec = undecodable_encodings(counts.get("undecodable", 0) or 1, rng)
    undec_i = 0
    entries = []
    for i, kind in enumerate(kinds):
        height = 1 + rng.randrange(1 << 20)
        msg = commit_vote_message(chain_id, height, rng.randrange(3), block_id,
                                  base_secs + rng.randrange(1 << 24), rng.randrange(10**9))
        if kind in ("small_order", "noncanonical_y", "neg_zero"):
            pool = {"small_order": SMALL_ORDER_CANONICAL, "noncanonical_y": SMALL_ORDER_NONCANONICAL_Y,
                    "neg_zero": SMALL_ORDER_NEG_ZERO}[kind]
            a = rng.choice(pool if rng.randrange(2) else SMALL_ORDER_CANONICAL)
            r = rng.choice(pool)
            if rng.randrange(2):
                a, r = r, a
            entries.append((a, msg, r + bytes(32)))
            continue
        signer = Ed25519Signer(key_seed(i))
        sig = signer.sign(msg)
        pk = signer.public_key
        if kind == "bitflip":
            where = rng.randrange(3)
            if where == 0:
                b = bytearray(sig); b[rng.randrange(32)] ^= 1 << rng.randrange(8); sig = bytes(b)
            elif where == 1:
                b = bytearray(sig); b[32 + rng.randrange(31)] ^= 1 << rng.randrange(8); sig = bytes(b)
            else:
                b = bytearray(msg); b[rng.randrange(len(b))] ^= 1 << rng.randrange(8); msg = bytes(b)
        elif kind == "s_plus_l":
            s = int.from_bytes(sig[32:], "little") + L
            sig = sig[:32] + s.to_bytes(32, "little")
        elif kind == "undecodable":
            bad = undec[undec_i % len(undec)]
            undec_i += 1
            if rng.randrange(2):
                sig = bad + sig[32:]
            else:
                pk = bad
        entries.append((pk, msg, sig))
    return Batch.from_entries(entries, kinds)


def make_commit_batch(n_vals: int, chain_id: str = "test_chain_id", height: int = 3, round_: int = 0,
                      seed: int = 1) -> Batch:
    """Config 1 shape: one commit of n_vals validators, all flags Commit,
    timestamps 2020-01-01T00:00:00Z + i ms."""
    rng = random.Random(seed)
    block_id = random_block_id(rng)
    entries = []
    base = 1577836800
    for i in range(n_vals):
        signer = Ed25519Signer(key_seed(i))
        ms = i
        msg = commit_vote_message(chain_id, height, round_, block_id, base + ms // 1000, (ms % 1000) * 1_000_000)
        entries.append((signer.public_key, msg, signer.sign(msg)))
    return Batch.from_entries(entries)


def make_sr25519_batch(n: int, seed: int = 0x5125519, chain_id: str = "test_chain_id",
                       bad_frac: float = 0.01) -> Batch:
    """sr25519 signatures over commit-vote sign-bytes; ~bad_frac corrupted
    (bit flips / missing marker / bad key encodings)."""
    from .sr25519_factory import Sr25519Signer, mini_from_secret
    rng = random.Random(seed)
    block_id = random_block_id(rng)
    entries, kinds = [], []
    base_secs = 1577836800
    for i in range(n):
        signer = Sr25519Signer(mini_from_secret(f"key: {i:x}".encode()))
        msg = commit_vote_message(chain_id, 1 + rng.randrange(1 << 20), rng.randrange(3), block_id,
                                  base_secs + rng.randrange(1 << 24), rng.randrange(10**9))
        sig = signer.sign(msg, b"%d" % i)
        pk = signer.public_key
        kind = "honest"
        if rng.random() < bad_frac:
            kind = rng.choice(["flip_r", "flip_s", "flip_m", "no_marker", "bad_pk"])
            if kind == "flip_r":
                b = bytearray(sig); b[rng.randrange(32)] ^= 1 << rng.randrange(8); sig = bytes(b)
            elif kind == "flip_s":
                b = bytearray(sig); b[32 + rng.randrange(31)] ^= 1 << rng.randrange(8); sig = bytes(b)
            elif kind == "flip_m":
                b = bytearray(msg); b[rng.randrange(len(b))] ^= 1 << rng.randrange(8); msg = bytes(b)
            elif kind == "no_marker":
                b = bytearray(sig); b[63] &= 0x7F; sig = bytes(b)
            else:
                pk = (int.from_bytes(pk, "little") | 1).to_bytes(32, "little")
        entries.append((pk, msg, sig))
        kinds.append(kind)
    return Batch.from_entries(entries, kinds)


def make_mixed_batch(n: int, seed: int = 0xC5, sr_frac: float = 0.5):
    """Config 5 shape: interleaved ed25519 + sr25519 entries.  Returns
    (kind uint8 array, Batch)."""
    rng = random.Random(seed)
    n_sr = int(n * sr_frac)
    ed = make_c2_batch(n - n_sr, seed=seed) if n - n_sr else Batch.from_entries([])
    sr = make_sr25519_batch(n_sr, seed=seed + 1) if n_sr else Batch.from_entries([])
    order = [0] * (n - n_sr) + [1] * n_sr
    rng.shuffle(order)
    entries, kinds, labels = [], [], []
    ie = isr = 0
    for k in order:
        if k == 0:
            entries.append(ed.entry(ie)); labels.append(ed.kinds[ie]); ie += 1
        else:
            entries.append(sr.entry(isr)); labels.append("sr:" + sr.kinds[isr]); isr += 1
        kinds.append(k)
    return np.array(kinds, np.uint8), Batch.from_entries(entries, labels)


def make_c1_commit(n_vals: int = 150, chain_id: str = "test_chain_id", height: int = 3, seed: int = 1):
    """Config 1: n validators (GenPrivKeyFromSecret("key: %x")),
    power 5n each (types/validator_set_test.go:1544 convention), height 3,
    round 0, random BlockID, all flags Commit, timestamps
    2020-01-01T00:00:00Z + i ms.  Returns (ValidatorSet, BlockID, Commit) of
    tendermint_amd.host."""
    from .. import host as H
    rng = random.Random(seed)
    bid = random_block_id(rng)
    signers = sorted((Ed25519Signer(key_seed(i)) for i in range(n_vals)),
                     key=lambda s: hashlib.sha256(s.public_key).digest()[:20])
    vals = H.ValidatorSet([H.Validator(hashlib.sha256(s.public_key).digest()[:20], s.public_key, 5 * n_vals)
                           for s in signers], proposer_index=0)
    hbid = H.BlockID(bid.hash, bid.part_set_header.total, bid.part_set_header.hash)
    sigs = []
    for i, s in enumerate(signers):
        ts = (1577836800, i * 1_000_000)
        msg = commit_vote_message(chain_id, height, 0, bid, ts[0], ts[1])
        sigs.append(H.CommitSig(H.BLOCK_ID_FLAG_COMMIT, vals.validators[i].address, ts, s.sign(msg)))
    return vals, hbid, H.Commit(height, 0, hbid, sigs)


def _simple_validator_bytes(v) -> bytes:
    """Validator.Bytes() (types/validator.go:154-170): SimpleValidator protobuf."""
    pub = bytes([(3 if v.key_kind == 1 else 1) << 3 | 2, 32]) + v.pub_key  # kind 1 = sr25519: oneof field 3
    out = bytes([0x0A, len(pub)]) + pub
    if v.voting_power:
        u, var = v.voting_power & ((1 << 64) - 1), bytearray()
        while True:
            var.append((u & 0x7F) | (0x80 if u >> 7 else 0))
            u >>= 7
            if not u:
                break
        out += b"\x10" + bytes(var)
    return out


def _merkle(items) -> bytes:
    """merkle.HashFromByteSlices (crypto/merkle/tree.go:11-27)."""
    if not items:
        return hashlib.sha256(b"").digest()
    if len(items) == 1:
        return hashlib.sha256(b"\x00" + items[0]).digest()
    k = 1 << (len(items).bit_length() - 1)
    k = k >> 1 if k == len(items) else k
    return hashlib.sha256(b"\x01" + _merkle(items[:k]) + _merkle(items[k:])).digest()


def _valset_hash(vals) -> bytes:
    """ValidatorSet.Hash (types/validator_set.go:344-350) of the generated set,
    so headers carry the hash the light client checks (light/verifier.go:266)."""
    return _merkle([_simple_validator_bytes(v) for v in vals.validators])


def _uvarint(u: int) -> bytes:
    u &= (1 << 64) - 1
    out = bytearray()
    while u >= 0x80:
        out.append((u & 0x7F) | 0x80)
        u >>= 7
    out.append(u)
    return bytes(out)


def _field(tag: int, b: bytes) -> bytes:
    return bytes([tag]) + _uvarint(len(b)) + b


def header_hash(h) -> bytes:
    """Header.Hash (types/block.go:447-478) of a host.Header, for generating
    chains whose commits sign their headers (the engine recomputes and checks
    it, light/verifier.go:243 -> types/light.go:168)."""
    ts = (b"\x08" + _uvarint(h.time[0]) if h.time[0] else b"") + (b"\x10" + _uvarint(h.time[1]) if h.time[1] else b"")
    lb = h.last_block_id
    psh = (b"\x08" + _uvarint(lb.psh_total) if lb.psh_total else b"") + (_field(0x12, lb.psh_hash) if lb.psh_hash else b"")
    bz = lambda b: _field(0x0A, b) if b else b""  # noqa: E731
    leaves = [(b"\x08" + _uvarint(h.version_block) if h.version_block else b"") +
              (b"\x10" + _uvarint(h.version_app) if h.version_app else b""),
              bz(h.chain_id.encode()), b"\x08" + _uvarint(h.height) if h.height else b"", ts,
              (_field(0x0A, lb.hash) if lb.hash else b"") + _field(0x12, psh),
              bz(h.last_commit_hash), bz(h.data_hash), bz(h.validators_hash), bz(h.next_validators_hash),
              bz(h.consensus_hash), bz(h.app_hash), bz(h.last_results_hash), bz(h.evidence_hash),
              bz(h.proposer_address)]
    return _merkle(leaves)


def _header_and_block_id(H, chain_id, height, t, vals, nvals, last_block_id, rng):
    """A header over (vals, nvals) and the BlockID of its hash."""
    hdr = H.Header(chain_id=chain_id, height=height, time=t, last_block_id=last_block_id,
                   last_commit_hash=_rand32(rng), data_hash=_rand32(rng), validators_hash=_valset_hash(vals),
                   next_validators_hash=_valset_hash(nvals), consensus_hash=_rand32(rng), app_hash=_rand32(rng)[:20],
                   proposer_address=vals.validators[0].address)
    return hdr, H.BlockID(header_hash(hdr), 1, _rand32(rng))


def _signed_header(H, chain_id, height, round_, t, vals, nvals, signers_sorted, last_block_id, rng, sign=True):
    """A header over (vals, nvals) and the commit of all signers for it."""
    hdr, hbid = _header_and_block_id(H, chain_id, height, t, vals, nvals, last_block_id, rng)
    bid = BlockID(hbid.hash, PartSetHeader(hbid.psh_total, hbid.psh_hash))
    sigs = []
    for i, s in enumerate(signers_sorted):
        ts = (t[0], t[1] + i)
        msg = commit_vote_message(chain_id, height, round_, bid, ts[0], ts[1])
        sigs.append(H.CommitSig(H.BLOCK_ID_FLAG_COMMIT, vals.validators[i].address, ts, s.sign(msg) if sign else b""))
    return H.SignedHeader(hdr, H.Commit(height, round_, hbid, sigs))


@dataclass
class PackedVotes:
    """Every commit vote of a generated chain as one packed batch (the
    input of a test's checker): commit c's votes are entries [commit_off[c],
    commit_off[c + 1]) in signature order; key_idx / seeds name the signer."""
    batch: "Batch"
    commit_off: np.ndarray


class _VoteSink:
    """Collects commit votes (messages built and signed in bulk, bulk.py)."""

    def __init__(self, seeds: List[bytes]):
        self.seeds = seeds
        self.msgs, self.offs, self.keys, self.counts = [], [], [], []

    def add_commit(self, chain_id, height, round_, hbid, key_ids, secs, nanos):
        from . import bulk
        bid = BlockID(hbid.hash, PartSetHeader(hbid.psh_total, hbid.psh_hash))
        m, o = bulk.vote_messages(bulk.commit_vote_head(height, round_, bid), chain_id, secs, nanos)
        self.msgs.append(m)
        self.offs.append(o)
        self.keys.append(np.asarray(key_ids, np.uint32))
        self.counts.append(len(key_ids))

    def sign(self, pks: List[bytes]) -> PackedVotes:
        from . import bulk
        msg = np.concatenate(self.msgs) if self.msgs else np.zeros(0, np.uint8)
        lens = np.concatenate([o[1:] - o[:-1] for o in self.offs]) if self.offs else np.zeros(0, np.uint32)
        off = np.zeros(len(lens) + 1, np.uint32)
        off[1:] = np.cumsum(lens)
        keys = np.concatenate(self.keys) if self.keys else np.zeros(0, np.uint32)
        sig = bulk.sign_many(self.seeds, keys, msg, off)
        pk_tab = np.frombuffer(b"".join(pks), np.uint8).reshape(-1, 32)
        pk = pk_tab[keys].reshape(-1) if len(keys) else np.zeros(0, np.uint8)
        co = np.zeros(len(self.counts) + 1, np.int64)
        co[1:] = np.cumsum(self.counts)
        return PackedVotes(Batch(pk, sig, msg, off), co)


def _commit_sigs(H, packed: PackedVotes, c: int, addrs, secs, nanos):
    lo = int(packed.commit_off[c])
    raw = packed.batch.sig[64 * lo:64 * int(packed.commit_off[c + 1])].tobytes()
    return [H.CommitSig(H.BLOCK_ID_FLAG_COMMIT, a, (int(s), int(ns)), raw[64 * i:64 * i + 64])
            for i, (a, s, ns) in enumerate(zip(addrs, secs, nanos))]


def _rand32(rng) -> bytes:
    return bytes(rng.randrange(256) for _ in range(32))


def make_light_chain(n_headers: int, n_vals: int = 100, chain_id: str = "test", rotate: int = 1, seed: int = 7,
                     packed: bool = False):
    """Config 3 shape (light/helpers_test.go:165-216 genLightBlocksWithKeys):
    n_vals validators of power 2, `rotate` keys replaced per height, round 1,
    every validator signs, one header per second.  Returns (trusted
    LightBlock at height 1, [LightBlock] for heights 2..n_headers+1); every
    LightBlock carries its validator set and the next one, every header's
    Hash() is the BlockID its commit signs.  packed=True also returns every
    commit's votes as one PackedVotes (trusted block first).  The set at
    step s (height s + 1) is keys [s rotate, s rotate + n_vals) (ChangeKeys:
    the oldest `rotate` keys leave, new ones join); messages and signatures
    are made in bulk (bulk.py)."""
    from .. import host as H
    from . import bulk
    rng = random.Random(seed)
    n_keys = (n_headers + 1) * rotate + n_vals
    seeds = [key_seed(k, "lkey") for k in range(n_keys)]
    pks = bulk.public_keys(seeds)
    addr = [hashlib.sha256(pk).digest()[:20] for pk in pks]
    sets = {}

    def valset(step):
        if step not in sets:
            ks = sorted(range(step * rotate, step * rotate + n_vals), key=lambda k: addr[k])
            sets[step] = (ks, H.ValidatorSet([H.Validator(addr[k], pks[k], 2) for k in ks], proposer_index=0))
            sets.pop(step - 2, None)
        return sets[step]

    t0 = 1577836800
    sink = _VoteSink(seeds)
    heads = []
    last_bid = H.BlockID()
    for h in range(1, n_headers + 2):
        ks, vals = valset(h - 1)
        _, nvals = valset(h)
        hdr, hbid = _header_and_block_id(H, chain_id, h, (t0 + h, 0), vals, nvals, last_bid, rng)
        sink.add_commit(chain_id, h, 1, hbid, ks, [t0 + h] * n_vals, list(range(n_vals)))
        heads.append((hdr, hbid, vals, nvals))
        last_bid = hbid
    pv = sink.sign(pks)
    out = []
    for c, (hdr, hbid, vals, nvals) in enumerate(heads):
        sigs = _commit_sigs(H, pv, c, [v.address for v in vals.validators], [hdr.time[0]] * n_vals, range(n_vals))
        out.append(H.LightBlock(H.SignedHeader(hdr, H.Commit(hdr.height, 1, hbid, sigs)), vals, nvals))
    if packed:
        return out[0], out[1:], pv
    return out[0], out[1:]


def make_block_chain(n_blocks: int, n_vals: int = 175, chain_id: str = "test_chain_id", seed: int = 11,
                     packed: bool = False):
    """Config 4 shape: a chain of n_blocks (heights 1..n_blocks, initial height
    1) with a static n_vals-validator set; block h carries LastCommit = the
    commit for h-1 (none at height 1).  Returns (ValidatorSet, [Block]);
    packed=True also returns the votes of the commits for heights
    1..n_blocks as one PackedVotes (commit c = height c + 1)."""
    from .. import host as H
    from ..chains import Block
    from . import bulk
    rng = random.Random(seed)
    seeds = [key_seed(i, "bkey") for i in range(n_vals)]
    pks = bulk.public_keys(seeds)
    addr = [hashlib.sha256(pk).digest()[:20] for pk in pks]
    ks = sorted(range(n_vals), key=lambda k: addr[k])
    vals = H.ValidatorSet([H.Validator(addr[k], pks[k], 10) for k in ks], proposer_index=0)
    sink = _VoteSink(seeds)
    bids = []
    nanos = [i * 1000 for i in range(n_vals)]
    for h in range(1, n_blocks + 1):
        bid = random_block_id(rng)
        hbid = H.BlockID(bid.hash, bid.part_set_header.total, bid.part_set_header.hash)
        bids.append(hbid)
        sink.add_commit(chain_id, h, 0, hbid, ks, [1577836800 + h] * n_vals, nanos)
    pv = sink.sign(pks)
    addrs = [v.address for v in vals.validators]
    blocks = []
    prev_commit = None
    for h, hbid in enumerate(bids, start=1):
        blocks.append(Block(h, hbid, prev_commit))
        prev_commit = H.Commit(h, 0, hbid, _commit_sigs(H, pv, h - 1, addrs, [1577836800 + h] * n_vals, nanos))
    if packed:
        return vals, blocks, pv
    return vals, blocks
