// Host-side mirror of the reference's commit-verification layer, in C++
// (the reference is compiled Go; no Go toolchain exists here).  Header-only
// so the CPU test harness (tests/native/commit_check.cpp) can instantiate the
// same control flow with a test-double verifier, while libtmgpu.so
// instantiates it with the GPU batch verifier.
//
//   types/validation.go        VerifyCommit / VerifyCommitLight /
//                              VerifyCommitLightTrusting / verifyCommitBatch /
//                              verifyCommitSingle / verifyBasicValsAndCommit
//   types/block.go:584-694     CommitSig (+ String), BlockIDFlag
//   types/block.go:815-862     Commit, GetVote, VoteSignBytes
//   types/block.go:1398-1418   BlockID IsNil / String
//   types/part_set.go:103-113  PartSetHeader String / IsZero / Equals
//   types/validator.go:129-138 Validator.String
//   types/validator_set.go     GetByAddress, TotalVotingPower, GetProposer,
//                              ErrNotEnoughVotingPowerSigned, safeMul
//   types/errors.go            ErrInvalidCommitHeight / Signatures
//   types/vote.go:149-157, types/canonical.go, canonical.pb.go  sign-bytes
//   crypto/batch/batch.go      CreateBatchVerifier / SupportsBatchVerifier
// Error strings are byte-identical to the Go originals (tests assert the
// substrings the reference's types/validation_test.go asserts).
#pragma once
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <functional>
#include <memory>
#include <optional>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

namespace tmh {

using Bytes = std::vector<uint8_t>;
using Error = std::optional<std::string>;

// A read-only view of bytes owned elsewhere (the caller's C structs during a
// tmv_verify_commits call, or a Bytes): commit signatures are not copied.
struct ByteView {
  const uint8_t *p = nullptr;
  size_t n = 0;
  ByteView() = default;
  ByteView(const uint8_t *ptr, size_t len) : p(len ? ptr : nullptr), n(len) {}
  ByteView(const Bytes &b) : p(b.data()), n(b.size()) {}  // NOLINT: implicit on purpose
  const uint8_t *data() const { return p; }
  size_t size() const { return n; }
  bool empty() const { return n == 0; }
  const uint8_t *begin() const { return p; }
  const uint8_t *end() const { return p + n; }
  bool operator==(const ByteView &o) const { return n == o.n && (n == 0 || std::memcmp(p, o.p, n) == 0); }
  bool operator!=(const ByteView &o) const { return !(*this == o); }
  bool operator<(const ByteView &o) const {  // lexicographic, as bytes.Compare / a Bytes comparison
    const int c = std::memcmp(p, o.p, std::min(n, o.n));
    return c < 0 || (c == 0 && n < o.n);
  }
};

// ---------------------------------------------------------------- Go-style formatting
inline std::string HexUpper(const uint8_t *p, size_t n) {
  static const char *d = "0123456789ABCDEF";
  std::string s;
  s.reserve(2 * n);
  for (size_t i = 0; i < n; i++) {
    s.push_back(d[p[i] >> 4]);
    s.push_back(d[p[i] & 15]);
  }
  return s;
}
inline std::string HexUpper(ByteView b) { return HexUpper(b.data(), b.size()); }
inline std::string HexUpper(const std::string &s) {
  return HexUpper(reinterpret_cast<const uint8_t *>(s.data()), s.size());
}
// libs/bytes.Fingerprint: first 6 bytes, zero padded
inline Bytes Fingerprint(ByteView b) {
  Bytes f(6, 0);
  std::memcpy(f.data(), b.data(), std::min<size_t>(6, b.size()));
  return f;
}

struct Timestamp {
  int64_t seconds = -62135596800LL;  // Go's zero time.Time
  int32_t nanos = 0;
};

// time.RFC3339Nano of a UTC instant (CanonicalTime, types/canonical.go:61-66)
inline std::string CanonicalTime(const Timestamp &t) {
  int64_t secs = t.seconds;
  int64_t days = secs / 86400, rem = secs % 86400;
  if (rem < 0) { rem += 86400; days -= 1; }
  // civil_from_days (proleptic Gregorian)
  int64_t z = days + 719468;
  const int64_t era = (z >= 0 ? z : z - 146096) / 146097;
  const int64_t doe = z - era * 146097;
  const int64_t yoe = (doe - doe / 1460 + doe / 36524 - doe / 146096) / 365;
  int64_t y = yoe + era * 400;
  const int64_t doy = doe - (365 * yoe + yoe / 4 - yoe / 100);
  const int64_t mp = (5 * doy + 2) / 153;
  const int64_t dd = doy - (153 * mp + 2) / 5 + 1;
  const int64_t mm = mp + (mp < 10 ? 3 : -9);
  if (mm <= 2) y += 1;
  char buf[64];
  std::snprintf(buf, sizeof buf, "%04lld-%02lld-%02lldT%02lld:%02lld:%02lld", (long long)y, (long long)mm,
                (long long)dd, (long long)(rem / 3600), (long long)((rem / 60) % 60), (long long)(rem % 60));
  std::string s(buf);
  if (t.nanos != 0) {
    char f[16];
    std::snprintf(f, sizeof f, "%09d", t.nanos);
    std::string frac(f);
    while (!frac.empty() && frac.back() == '0') frac.pop_back();
    s += "." + frac;
  }
  return s + "Z";
}

// ---------------------------------------------------------------- keys
enum class KeyType : uint8_t { Ed25519 = 0, Sr25519 = 1, Other = 255 };

// A public key: its type and a view of its bytes (the caller's tmv_validator
// / tmv_batch_add arguments, which outlive the call that reads them).
struct PubKey {
  KeyType type = KeyType::Ed25519;
  ByteView bytes;
  std::string Type() const {
    return type == KeyType::Ed25519 ? "ed25519" : type == KeyType::Sr25519 ? "sr25519" : "other";
  }
  std::string String() const {  // crypto/ed25519/ed25519.go:182, crypto/sr25519/pubkey.go:68
    if (type == KeyType::Ed25519) return "PubKeyEd25519{" + HexUpper(bytes) + "}";
    if (type == KeyType::Sr25519) return "PubKeySr25519{" + HexUpper(bytes) + "}";
    return "PubKey{" + HexUpper(bytes) + "}";
  }
};

// ---------------------------------------------------------------- crypto.BatchVerifier
// crypto/crypto.go:66-76.  Add appends; Verify returns (all ok, vector in
// Add order).  Add-time failures that need curve decoding (sr25519 public
// key / signature encoding, crypto/sr25519/batch.go:30-37) are detected on
// the device and surfaced by DeferredAddError() after Verify; the commit
// verifier below orders them exactly where the reference's Add would have
// returned them.
class BatchVerifier {
 public:
  virtual ~BatchVerifier() = default;
  virtual Error Add(const PubKey &key, const Bytes &msg, const Bytes &sig) = 0;
  virtual std::pair<bool, std::vector<bool>> Verify() = 0;
  // (batch index, message) of the first entry whose Add would have failed
  virtual std::optional<std::pair<size_t, std::string>> DeferredAddError() const { return std::nullopt; }
  // true when DeferredAddError() can be non-empty (sr25519)
  virtual bool MayDeferAddErrors() const { return false; }
};

using BatchVerifierFactory = std::function<std::unique_ptr<BatchVerifier>(KeyType)>;
using SingleVerifier = std::function<bool(const PubKey &, const Bytes &msg, const Bytes &sig)>;

// crypto/batch/batch.go:26-33
inline bool SupportsBatchVerifier(const PubKey &pk) {
  return pk.type == KeyType::Ed25519 || pk.type == KeyType::Sr25519;
}

// ---------------------------------------------------------------- types
enum BlockIDFlag : uint8_t { BlockIDFlagAbsent = 1, BlockIDFlagCommit = 2, BlockIDFlagNil = 3 };

struct PartSetHeader {
  uint32_t total = 0;
  Bytes hash;
  bool IsZero() const { return total == 0 && hash.empty(); }
  bool Equals(const PartSetHeader &o) const { return total == o.total && hash == o.hash; }
  std::string String() const { return std::to_string(total) + ":" + HexUpper(Fingerprint(hash)); }
};

struct BlockID {
  Bytes hash;
  PartSetHeader part_set_header;
  bool IsNil() const { return hash.empty() && part_set_header.IsZero(); }
  bool Equals(const BlockID &o) const { return hash == o.hash && part_set_header.Equals(o.part_set_header); }
  std::string String() const { return HexUpper(hash) + ":" + part_set_header.String(); }
};

struct CommitSig {
  BlockIDFlag block_id_flag = BlockIDFlagAbsent;
  ByteView validator_address;  // views into the caller's tmv_commit_sig
  Timestamp timestamp;
  ByteView signature;
  // types/block.go:633-639
  std::string String() const {
    return "CommitSig{" + HexUpper(Fingerprint(signature)) + " by " + HexUpper(Fingerprint(validator_address)) +
           " on " + std::to_string((int)block_id_flag) + " @ " + CanonicalTime(timestamp) + "}";
  }
  // types/block.go:643-657
  BlockID BlockIDFor(const BlockID &commit_block_id) const {
    return block_id_flag == BlockIDFlagCommit ? commit_block_id : BlockID{};
  }
};

constexpr int32_t kPrevoteType = 1;
constexpr int32_t kPrecommitType = 2;

inline size_t UvarintLen(uint64_t x) {
  size_t n = 1;
  while (x >= 0x80) { x >>= 7; n++; }
  return n;
}
inline uint8_t *PutUvarintP(uint8_t *p, uint64_t x) {
  while (x >= 0x80) { *p++ = (uint8_t)(x | 0x80); x >>= 7; }
  *p++ = (uint8_t)x;
  return p;
}
inline uint8_t *PutFixed64P(uint8_t *p, int64_t v) {
  for (int i = 0; i < 8; i++) *p++ = (uint8_t)((uint64_t)v >> (8 * i));
  return p;
}
inline uint8_t *PutBytesField(uint8_t *p, uint8_t tag, const Bytes &b) {
  *p++ = tag;
  p = PutUvarintP(p, b.size());
  if (!b.empty()) std::memcpy(p, b.data(), b.size());
  return p + b.size();
}

// types.VoteSignBytes: MarshalDelimited(CanonicalizeVote(chainID, vote)),
// field by field as gogoproto emits CanonicalVote (proto3: zero fields
// omitted; the timestamp is always present).  block_id == nullptr or a nil
// BlockID omits field 4 (types/canonical.go:18-32).  The message is split
// into the parts shared by a commit's votes -- fields 1-3 (head), field 4
// (block) and field 6 (chain) -- and the per-vote timestamp field 5, so that
// the host encoder and the device one (tmv_verify_votes) assemble the same
// pieces: uvarint(len(body)) || head || [block] || ts field || chain.
inline size_t VoteHeadLen(int32_t type, int64_t height, int32_t round) {
  return (type != 0 ? 1 + UvarintLen((uint64_t)(uint32_t)type) : 0) + (height != 0 ? 9 : 0) + (round != 0 ? 9 : 0);
}
inline uint8_t *PutVoteHead(uint8_t *p, int32_t type, int64_t height, int32_t round) {
  if (type != 0) { *p++ = 0x08; p = PutUvarintP(p, (uint64_t)(uint32_t)type); }
  if (height != 0) { *p++ = 0x11; p = PutFixed64P(p, height); }
  if (round != 0) { *p++ = 0x19; p = PutFixed64P(p, (int64_t)round); }
  return p;
}
// field 4 (CanonicalBlockID), empty for a nil BlockID
inline size_t VoteBlockLen(const BlockID *block_id, size_t *psh_len_out = nullptr, size_t *cb_len_out = nullptr) {
  if (!block_id || block_id->IsNil()) return 0;
  const PartSetHeader &ph = block_id->part_set_header;
  size_t psh_len = 0, cb_len = 0;
  if (ph.total != 0) psh_len += 1 + UvarintLen(ph.total);
  if (!ph.hash.empty()) psh_len += 1 + UvarintLen(ph.hash.size()) + ph.hash.size();
  if (!block_id->hash.empty()) cb_len += 1 + UvarintLen(block_id->hash.size()) + block_id->hash.size();
  cb_len += 1 + UvarintLen(psh_len) + psh_len;
  if (psh_len_out) *psh_len_out = psh_len;
  if (cb_len_out) *cb_len_out = cb_len;
  return 1 + UvarintLen(cb_len) + cb_len;
}
inline uint8_t *PutVoteBlock(uint8_t *p, const BlockID *block_id) {
  size_t psh_len = 0, cb_len = 0;
  if (VoteBlockLen(block_id, &psh_len, &cb_len) == 0) return p;
  const PartSetHeader &ph = block_id->part_set_header;
  *p++ = 0x22;
  p = PutUvarintP(p, cb_len);
  if (!block_id->hash.empty()) p = PutBytesField(p, 0x0a, block_id->hash);
  *p++ = 0x12;
  p = PutUvarintP(p, psh_len);
  if (ph.total != 0) { *p++ = 0x08; p = PutUvarintP(p, ph.total); }
  if (!ph.hash.empty()) p = PutBytesField(p, 0x12, ph.hash);
  return p;
}
inline size_t VoteChainLen(const std::string &chain_id) {
  return chain_id.empty() ? 0 : 1 + UvarintLen(chain_id.size()) + chain_id.size();
}
inline uint8_t *PutVoteChain(uint8_t *p, const std::string &chain_id) {
  if (chain_id.empty()) return p;
  *p++ = 0x32;
  p = PutUvarintP(p, chain_id.size());
  std::memcpy(p, chain_id.data(), chain_id.size());
  return p + chain_id.size();
}
// field 5 (google.protobuf.Timestamp, always present)
inline size_t VoteTimestampInner(const Timestamp &ts) {
  return (ts.seconds != 0 ? 1 + UvarintLen((uint64_t)ts.seconds) : 0) +
         (ts.nanos != 0 ? 1 + UvarintLen((uint64_t)(int64_t)ts.nanos) : 0);
}
inline size_t VoteTimestampLen(const Timestamp &ts) {
  const size_t t = VoteTimestampInner(ts);
  return 1 + UvarintLen(t) + t;
}
inline uint8_t *PutVoteTimestamp(uint8_t *p, const Timestamp &ts) {
  *p++ = 0x2a;
  p = PutUvarintP(p, VoteTimestampInner(ts));
  if (ts.seconds != 0) { *p++ = 0x08; p = PutUvarintP(p, (uint64_t)ts.seconds); }
  if (ts.nanos != 0) { *p++ = 0x10; p = PutUvarintP(p, (uint64_t)(int64_t)ts.nanos); }
  return p;
}

// Appends the encoding to `out` (no allocation when `out` has capacity).
inline void AppendVoteSignBytes(Bytes &out, const std::string &chain_id, int32_t type, int64_t height,
                                int32_t round, const BlockID *block_id, const Timestamp &ts) {
  const size_t body = VoteHeadLen(type, height, round) + VoteBlockLen(block_id) + VoteTimestampLen(ts) +
                      VoteChainLen(chain_id);
  const size_t at = out.size();
  out.resize(at + UvarintLen(body) + body);
  uint8_t *p = PutUvarintP(out.data() + at, body);
  p = PutVoteHead(p, type, height, round);
  p = PutVoteBlock(p, block_id);
  p = PutVoteTimestamp(p, ts);
  PutVoteChain(p, chain_id);
}

// The three shared segments of tmv_verify_votes' template, back to back.
struct VoteTemplate {
  Bytes bytes;
  uint32_t head_len = 0, block_len = 0, chain_len = 0;
};
inline VoteTemplate EncodeVoteTemplate(const std::string &chain_id, int32_t type, int64_t height, int32_t round,
                                       const BlockID *block_id) {
  VoteTemplate t;
  t.head_len = (uint32_t)VoteHeadLen(type, height, round);
  t.block_len = (uint32_t)VoteBlockLen(block_id);
  t.chain_len = (uint32_t)VoteChainLen(chain_id);
  t.bytes.resize((size_t)t.head_len + t.block_len + t.chain_len);
  uint8_t *p = PutVoteHead(t.bytes.data(), type, height, round);
  p = PutVoteBlock(p, block_id);
  PutVoteChain(p, chain_id);
  return t;
}

// One vote's sign-bytes from its commit's template (the host twin of
// k_vote_signbytes).
inline void AppendVoteFromTemplate(Bytes &out, const VoteTemplate &t, bool with_block, const Timestamp &ts) {
  const size_t body = (size_t)t.head_len + (with_block ? t.block_len : 0) + VoteTimestampLen(ts) + t.chain_len;
  const size_t at = out.size();
  out.resize(at + UvarintLen(body) + body);
  uint8_t *p = PutUvarintP(out.data() + at, body);
  const uint8_t *b = t.bytes.data();
  std::memcpy(p, b, t.head_len);
  p += t.head_len;
  if (with_block && t.block_len) {
    std::memcpy(p, b + t.head_len, t.block_len);
    p += t.block_len;
  }
  p = PutVoteTimestamp(p, ts);
  if (t.chain_len) std::memcpy(p, b + t.head_len + t.block_len, t.chain_len);
}

inline Bytes VoteSignBytes(const std::string &chain_id, int32_t type, int64_t height, int32_t round,
                           const BlockID *block_id, const Timestamp &ts) {
  Bytes out;
  AppendVoteSignBytes(out, chain_id, type, height, round, block_id, ts);
  return out;
}

struct Commit {
  int64_t height = 0;
  int32_t round = 0;
  BlockID block_id;
  std::vector<CommitSig> signatures;
  // types/block.go:836-862: only the timestamp and the flag differ per index
  Bytes VoteSignBytes(const std::string &chain_id, int32_t idx) const {
    Bytes out;
    AppendVoteSignBytes(out, chain_id, idx);
    return out;
  }
  void AppendVoteSignBytes(Bytes &out, const std::string &chain_id, int32_t idx) const {
    const CommitSig &cs = signatures[(size_t)idx];
    // BlockIDFor: the commit's BlockID for a Commit flag, else the nil BlockID
    tmh::AppendVoteSignBytes(out, chain_id, kPrecommitType, height, round,
                             cs.block_id_flag == BlockIDFlagCommit ? &block_id : nullptr, cs.timestamp);
  }
};

// Views into the caller's tmv_validator array: converting a validator set
// allocates nothing per validator.
struct Validator {
  ByteView address;
  PubKey pub_key;
  int64_t voting_power = 0;
  int64_t proposer_priority = 0;
  std::string String() const {  // types/validator.go:129-138
    return "Validator{" + HexUpper(address) + " " + pub_key.String() + " VP:" + std::to_string(voting_power) +
           " A:" + std::to_string(proposer_priority) + "}";
  }
};

struct ValidatorSet {
  std::vector<Validator> validators;
  int proposer = -1;  // index of the current proposer, -1 = derive from priorities
  int64_t total_voting_power = 0;  // 0 = not precomputed (see UpdateTotalVotingPower)

  size_t Size() const { return validators.size(); }
  // Read-only: plans of one batch run on several threads over a shared set,
  // so the getter never writes; converters call UpdateTotalVotingPower once.
  int64_t TotalVotingPower() const {
    if (total_voting_power != 0) return total_voting_power;
    int64_t t = 0;
    for (const auto &v : validators) t += v.voting_power;
    return t;
  }
  void UpdateTotalVotingPower() {
    total_voting_power = 0;
    total_voting_power = TotalVotingPower();
  }
  // types/validator_set.go:267-274 (linear scan, like the reference)
  std::pair<int32_t, const Validator *> GetByAddress(ByteView addr) const {
    for (size_t i = 0; i < validators.size(); i++)
      if (validators[i].address == addr) return {(int32_t)i, &validators[i]};
    return {-1, nullptr};
  }
  // types/validator_set.go:322-344: highest priority, ties to the smaller address
  const Validator *GetProposer() const {
    if (validators.empty()) return nullptr;
    if (proposer >= 0 && (size_t)proposer < validators.size()) return &validators[(size_t)proposer];
    const Validator *best = nullptr;
    for (const auto &v : validators) {
      if (!best || v.proposer_priority > best->proposer_priority ||
          (v.proposer_priority == best->proposer_priority && v.address < best->address))
        best = &v;
    }
    return best;
  }
};

// ---------------------------------------------------------------- errors
inline std::string ErrNotEnoughVotingPowerSigned(int64_t got, int64_t needed) {
  return "invalid commit -- insufficient voting power: got " + std::to_string(got) + ", needed more than " +
         std::to_string(needed);
}
inline std::string ErrInvalidCommitSignatures(size_t expected, size_t actual) {
  return "Invalid commit -- wrong set size: " + std::to_string(expected) + " vs " + std::to_string(actual);
}
inline std::string ErrInvalidCommitHeight(int64_t expected, int64_t actual) {
  return "Invalid commit -- wrong height: " + std::to_string(expected) + " vs " + std::to_string(actual);
}

// types/validator_set.go:910-931
inline std::pair<int64_t, bool> SafeMul(int64_t a, int64_t b) {
  if (a == 0 || b == 0) return {0, false};
  const int64_t ab = b < 0 ? -b : b, aa = a < 0 ? -a : a;
  if (aa > INT64_MAX / ab) return {0, true};
  return {a * b, false};
}

// ---------------------------------------------------------------- Add-time checks
// crypto/ed25519/ed25519.go:209-224 and crypto/sr25519/batch.go:23-37.
// `sync` is an error the reference's Add returns that needs no curve work;
// sr25519 decoding failures are found on the device: `deferred_sig` is the
// text to report if the device flags the signature encoding (status -2).
struct AddCheck {
  Error sync;
  std::string deferred_sig;
  const uint8_t *sig64 = nullptr;  // the 64 bytes handed to the device (zeros when the length is wrong)
};

inline const uint8_t *ZeroSignature() {
  static const uint8_t z[64] = {0};
  return z;
}

inline bool ScalarCanonical(const uint8_t s[32]) {
  static const uint8_t L[32] = {0xed, 0xd3, 0xf5, 0x5c, 0x1a, 0x63, 0x12, 0x58, 0xd6, 0x9c, 0xf7,
                                0xa2, 0xde, 0xf9, 0xde, 0x14, 0,    0,    0,    0,    0,    0,
                                0,    0,    0,    0,    0,    0,    0,    0,    0,    0x10};
  for (int i = 31; i >= 0; i--) {
    if (s[i] < L[i]) return true;
    if (s[i] > L[i]) return false;
  }
  return false;
}

inline AddCheck CheckAdd(KeyType batch_kind, const PubKey &key, ByteView sig) {
  AddCheck r;
  if (batch_kind == KeyType::Ed25519) {
    if (key.type != KeyType::Ed25519) { r.sync = std::string("pubkey is not Ed25519"); return r; }
    if (key.bytes.size() != 32) {
      r.sync = "pubkey size is incorrect; expected: 32, got " + std::to_string(key.bytes.size());
      return r;
    }
    if (sig.size() != 64) { r.sync = std::string("invalid signature"); return r; }
    r.sig64 = sig.data();
    return r;
  }
  if (key.type != KeyType::Sr25519) { r.sync = std::string("sr25519: pubkey is not sr25519"); return r; }
  if (key.bytes.size() != 32) {
    r.sync = "sr25519: invalid public key: sr25519: bad PublicKey size: " + std::to_string(key.bytes.size());
    return r;
  }
  r.sig64 = ZeroSignature();  // a zero signature has no schnorrkel marker: the device reports -2
  if (sig.size() != 64) {
    r.deferred_sig = "sr25519: unable to decode signature: sr25519: bad Signature size: " + std::to_string(sig.size());
    return r;
  }
  r.sig64 = sig.data();
  uint8_t sc[32];
  std::memcpy(sc, sig.data() + 32, 32);
  if (!(sc[31] & 0x80)) {
    r.deferred_sig = "sr25519: unable to decode signature: sr25519: signature is not marked as a schnorrkel signature";
  } else {
    sc[31] &= 0x7f;
    if (!ScalarCanonical(sc)) r.deferred_sig = "sr25519: unable to decode signature: sr25519: non-canonical scalar";
  }
  return r;
}

inline std::string DeferredPubKeyError() {
  return "sr25519: invalid public key: sr25519: failed to decompress public key";
}

// ---------------------------------------------------------------- commit verification
constexpr int kBatchVerifyThreshold = 2;  // types/validation.go:12

// One signature to verify: status 1 valid, 0 invalid, -1 / -2 device-found
// sr25519 Add errors (public key / signature encoding).
// A view into the validator set and the commit (both outlive the check).
// The message is not materialised on the host: it is the commit's vote
// sign-bytes for the plan's chain_id at pl.sig_idx[i], built on the device
// from the commit's template (tmv_verify_votes).
struct SigEntry {
  KeyType kind;
  ByteView pk;  // the validator's key (entries of one key share its data pointer)
  uint32_t sig_len;
  const uint8_t *sig;
};

// A commit check up to the point where signature results are needed.
// Plan (loop of verifyCommitBatch / verifyCommitSingle) -> the backend
// verifies the entries of many plans in one device batch -> Finish.
struct CommitPlan {
  Error early;                       // decided before any signature result
  bool batch = false;                // verifyCommitBatch (true) or verifyCommitSingle
  bool defer_add = false;            // sr25519 batch: device statuses -1/-2 are Add errors
  int64_t tallied = 0, needed = 0;
  std::vector<SigEntry> entries;     // in Add order
  std::vector<int> sig_idx;          // commit.Signatures index of each entry
  std::vector<std::string> deferred_sig;  // per entry when defer_add (sr25519 batch), else empty
  std::vector<uint8_t> crosses;      // single: this entry crosses the threshold (early ok)
  const Commit *commit = nullptr;
  std::string chain_id;              // the messages are this commit's votes on chain_id
};

struct CommitVerifier {
  static bool ShouldBatchVerify(const ValidatorSet &vals, const Commit &commit) {
    const Validator *p = vals.GetProposer();
    return commit.signatures.size() >= (size_t)kBatchVerifyThreshold && p && SupportsBatchVerifier(p->pub_key);
  }

  using SigPred = bool (*)(const CommitSig &);

  // The loop of types/validation.go:179-227 (batch) / :284-327 (single).
  static void PlanLoop(CommitPlan &pl, const std::string &chain_id, const ValidatorSet &vals, const Commit &commit,
                       SigPred ignore, SigPred count, bool count_all, bool by_index) {
    KeyType bkind = KeyType::Other;
    if (pl.batch) {
      const Validator *proposer = vals.GetProposer();
      if (!proposer || !SupportsBatchVerifier(proposer->pub_key) ||
          commit.signatures.size() < (size_t)kBatchVerifyThreshold) {
        pl.early = std::string("unsupported signature algorithm or insufficient signatures for batch verification");
        return;
      }
      bkind = proposer->pub_key.type;
      pl.defer_add = bkind == KeyType::Sr25519;
    }
    std::unordered_map<int32_t, int> seen;
    pl.entries.reserve(commit.signatures.size());
    pl.sig_idx.reserve(commit.signatures.size());
    pl.crosses.reserve(commit.signatures.size());
    if (pl.defer_add) pl.deferred_sig.reserve(commit.signatures.size());
    for (size_t idx = 0; idx < commit.signatures.size(); idx++) {
      const CommitSig &cs = commit.signatures[idx];
      if (ignore(cs)) continue;
      const Validator *val;
      if (by_index) {
        val = &vals.validators[idx];
      } else {
        auto [vi, v] = vals.GetByAddress(cs.validator_address);
        if (!v) continue;
        auto it = seen.find(vi);
        if (it != seen.end()) {
          pl.early = "double vote from " + v->String() + " (" + std::to_string(it->second) + " and " +
                     std::to_string(idx) + ")";
          return;
        }
        seen[vi] = (int)idx;
        val = v;
      }
      SigEntry e{val->pub_key.type, val->pub_key.bytes, 0, nullptr};
      if (pl.batch) {
        AddCheck ac = CheckAdd(bkind, val->pub_key, cs.signature);
        if (ac.sync) {  // bv.Add error, returned verbatim (:211-213)
          pl.early = ac.sync;
          return;
        }
        e.sig = ac.sig64;
        e.sig_len = 64;
        if (pl.defer_add) pl.deferred_sig.push_back(std::move(ac.deferred_sig));  // sr25519 only
      } else {
        e.sig = cs.signature.data();
        e.sig_len = (uint32_t)cs.signature.size();
      }
      pl.entries.push_back(e);
      pl.sig_idx.push_back((int)idx);
      if (count(cs)) pl.tallied += val->voting_power;
      const bool cross = !count_all && pl.tallied > pl.needed;
      pl.crosses.push_back(cross ? 1 : 0);
      if (cross) break;
    }
  }

  // Signature results -> the reference's return value.  *not_enough is set
  // when the error is types.ErrNotEnoughVotingPowerSigned (the light client
  // maps that type to ErrNewValSetCantBeTrusted, light/verifier.go:72-75).
  static Error Finish(const CommitPlan &pl, const int8_t *st, bool *not_enough = nullptr) {
    if (not_enough) *not_enough = false;
    if (pl.early) return pl.early;
    const Commit &commit = *pl.commit;
    if (pl.batch) {
      // a device-found Add error wins, as the reference's Add returns it in the loop
      if (pl.defer_add) {
        for (size_t i = 0; i < pl.entries.size(); i++) {
          if (st[i] == -1) return DeferredPubKeyError();
          if (st[i] == -2)
            return pl.deferred_sig[i].empty() ? std::string("sr25519: unable to decode signature") : pl.deferred_sig[i];
        }
      }
      if (pl.tallied <= pl.needed) {
        if (not_enough) *not_enough = true;
        return ErrNotEnoughVotingPowerSigned(pl.tallied, pl.needed);
      }
      for (size_t i = 0; i < pl.entries.size(); i++) {
        if (st[i] != 1) {
          const int idx = pl.sig_idx[i];
          return "wrong signature (#" + std::to_string(idx) + "): " + HexUpper(commit.signatures[(size_t)idx].String());
        }
      }
      if (pl.entries.empty()) return std::string("BUG: batch verification failed with no invalid signatures");
      return std::nullopt;
    }
    for (size_t i = 0; i < pl.entries.size(); i++) {
      if (st[i] != 1) {
        const int idx = pl.sig_idx[i];
        return "wrong signature (#" + std::to_string(idx) + "): " + HexUpper(commit.signatures[(size_t)idx].signature);
      }
      if (pl.crosses[i]) return std::nullopt;
    }
    if (pl.tallied <= pl.needed) {
      if (not_enough) *not_enough = true;
      return ErrNotEnoughVotingPowerSigned(pl.tallied, pl.needed);
    }
    return std::nullopt;
  }

  static Error VerifyBasic(const ValidatorSet *vals, const Commit *commit, int64_t height, const BlockID &block_id) {
    if (!vals) return std::string("nil validator set");
    if (!commit) return std::string("nil commit");
    if (vals->Size() != commit->signatures.size()) return ErrInvalidCommitSignatures(vals->Size(), commit->signatures.size());
    if (height != commit->height) return ErrInvalidCommitHeight(height, commit->height);
    if (!block_id.Equals(commit->block_id))
      return "invalid commit -- wrong block ID: want " + block_id.String() + ", got " + commit->block_id.String();
    return std::nullopt;
  }

  static bool IgnoreAbsent(const CommitSig &c) { return c.block_id_flag == BlockIDFlagAbsent; }
  static bool CountCommit(const CommitSig &c) { return c.block_id_flag == BlockIDFlagCommit; }
  static bool IgnoreNotCommit(const CommitSig &c) { return c.block_id_flag != BlockIDFlagCommit; }
  static bool CountAll(const CommitSig &) { return true; }

  enum Mode { kFull = 0, kLight = 1, kLightTrusting = 2 };

  // types/validation.go:27-53 (kFull), :61-86 (kLight), :96-132 (kLightTrusting)
  static CommitPlan Plan(Mode mode, const std::string &chain_id, const ValidatorSet *vals, const BlockID &block_id,
                         int64_t height, const Commit *commit, int64_t num, int64_t den) {
    CommitPlan pl;
    pl.commit = commit;
    pl.chain_id = chain_id;
    if (mode == kLightTrusting) {
      if (!vals) { pl.early = std::string("nil validator set"); return pl; }
      if (den == 0) { pl.early = std::string("trustLevel has zero Denominator"); return pl; }
      if (!commit) { pl.early = std::string("nil commit"); return pl; }
      auto [prod, overflow] = SafeMul(vals->TotalVotingPower(), num);
      if (overflow) {
        pl.early = std::string(
            "int64 overflow while calculating voting power needed. please provide smaller trustLevel numerator");
        return pl;
      }
      pl.needed = prod / den;
      pl.batch = ShouldBatchVerify(*vals, *commit);
      PlanLoop(pl, chain_id, *vals, *commit, IgnoreNotCommit, CountAll, false, false);
      return pl;
    }
    if ((pl.early = VerifyBasic(vals, commit, height, block_id))) return pl;
    pl.needed = vals->TotalVotingPower() * 2 / 3;
    pl.batch = ShouldBatchVerify(*vals, *commit);
    if (mode == kFull) PlanLoop(pl, chain_id, *vals, *commit, IgnoreAbsent, CountCommit, true, true);
    else PlanLoop(pl, chain_id, *vals, *commit, IgnoreNotCommit, CountAll, false, true);
    return pl;
  }
};

}  // namespace tmh
