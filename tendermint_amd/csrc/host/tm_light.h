// Host-side mirror of the light client's header verification, in C++ (the
// reference is compiled Go; no Go toolchain exists here).  Header-only, like
// tm_types.h, so the CPU harness (tests/native/commit_check.cpp) runs the
// same control flow.
//
//   types/block.go:385-437        Header.ValidateBasic
//   types/block.go:447-478        Header.Hash (leaves; the merkle root is
//                                 computed by the engine, tmv_merkle_roots,
//                                 or on the host for a few headers)
//   types/encoding_helper.go:11-48 cdcEncode
//   types/block.go:657-694,874-897 CommitSig / Commit ValidateBasic
//   types/block.go:1386-1396, types/part_set.go:116-122  BlockID / PSH ValidateBasic
//   types/light.go:145-172        SignedHeader.ValidateBasic
//   light/verifier.go:33-290      VerifyNonAdjacent / VerifyAdjacent / Verify /
//                                 ValidateTrustLevel / HeaderExpired /
//                                 verifyNewHeaderAndVals / checkRequiredHeaderFields
//   light/errors.go:15-40         ErrOldHeaderExpired / ErrNewValSetCantBeTrusted /
//                                 ErrInvalidHeader
// Error strings are byte-identical to the Go originals, including Go's %v of
// time.Time / time.Duration and %q.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "../sha256_dev.h"
#include "tm_types.h"

namespace tmh {

// ---------------------------------------------------------------- Go formatting
constexpr int64_t kNanosPerSecond = 1000000000LL;

inline __int128 TimeNs(const Timestamp &t) { return (__int128)t.seconds * kNanosPerSecond + t.nanos; }
inline Timestamp FromNs(__int128 ns) {
  __int128 s = ns / kNanosPerSecond, r = ns % kNanosPerSecond;
  if (r < 0) { r += kNanosPerSecond; s -= 1; }
  return Timestamp{(int64_t)s, (int32_t)r};
}
inline bool IsZeroTime(const Timestamp &t) { return t.seconds == -62135596800LL && t.nanos == 0; }

// time.Time.String() of a UTC instant: "2006-01-02 15:04:05.999999999 -0700 MST"
inline std::string GoTime(const Timestamp &t) {
  std::string s = CanonicalTime(t);  // RFC 3339 with the same trimmed fraction
  s[10] = ' ';
  s.pop_back();  // 'Z'
  return s + " +0000 UTC";
}

// time.Duration.String()
inline std::string GoDuration(int64_t d) {
  if (d == 0) return "0s";
  const bool neg = d < 0;
  uint64_t u = neg ? (uint64_t)0 - (uint64_t)d : (uint64_t)d;
  auto frac = [](uint64_t &v, int prec) {
    std::string digits;
    bool printed = false;
    for (int i = 0; i < prec; i++) {
      const uint64_t dg = v % 10;
      printed = printed || dg != 0;
      if (printed) digits.insert(digits.begin(), (char)('0' + dg));
      v /= 10;
    }
    return printed ? "." + digits : std::string();
  };
  std::string s;
  if (u < (uint64_t)kNanosPerSecond) {
    if (u < 1000) {
      s = std::to_string(u) + "ns";
    } else if (u < 1000000) {
      const std::string f = frac(u, 3);
      s = std::to_string(u) + f + "\xc2\xb5s";  // µs
    } else {
      const std::string f = frac(u, 6);
      s = std::to_string(u) + f + "ms";
    }
  } else {
    const std::string f = frac(u, 9);
    s = std::to_string(u % 60) + f + "s";
    u /= 60;
    if (u > 0) {
      s = std::to_string(u % 60) + "m" + s;
      u /= 60;
      if (u > 0) s = std::to_string(u) + "h" + s;
    }
  }
  return neg ? "-" + s : s;
}

// strconv.Quote for ASCII and well-formed UTF-8 (printable runes kept)
inline std::string GoQuote(const std::string &in) {
  std::string o = "\"";
  for (size_t i = 0; i < in.size(); i++) {
    const unsigned char c = (unsigned char)in[i];
    switch (c) {
      case '"': o += "\\\""; continue;
      case '\\': o += "\\\\"; continue;
      case '\a': o += "\\a"; continue;
      case '\b': o += "\\b"; continue;
      case '\f': o += "\\f"; continue;
      case '\n': o += "\\n"; continue;
      case '\r': o += "\\r"; continue;
      case '\t': o += "\\t"; continue;
      case '\v': o += "\\v"; continue;
      default: break;
    }
    if (c < 0x20 || c == 0x7f) {
      char b[8];
      std::snprintf(b, sizeof b, "\\x%02x", c);
      o += b;
    } else if (c < 0x80) {
      o.push_back((char)c);
    } else {  // keep a well-formed multi-byte sequence, escape a stray byte
      const int n = c >= 0xf0 ? 4 : c >= 0xe0 ? 3 : c >= 0xc0 ? 2 : 0;
      bool ok = n > 0 && i + n <= in.size();
      for (int k = 1; ok && k < n; k++) ok = ((unsigned char)in[i + k] & 0xc0) == 0x80;
      if (ok) {
        o.append(in, i, (size_t)n);
        i += (size_t)n - 1;
      } else {
        char b[8];
        std::snprintf(b, sizeof b, "\\x%02x", c);
        o += b;
      }
    }
  }
  return o + "\"";
}

// ---------------------------------------------------------------- header
constexpr uint64_t kBlockProtocol = 11;   // version/version.go:27
constexpr size_t kMaxChainIDLen = 50;     // types/genesis.go:19
constexpr size_t kHashSize = 32;          // crypto.HashSize
constexpr size_t kAddressSize = 20;       // crypto.AddressSize
constexpr size_t kMaxSignatureSize = 64;  // types/signable.go:12

struct Header {
  uint64_t version_block = 0, version_app = 0;
  std::string chain_id;
  int64_t height = 0;
  Timestamp time;
  BlockID last_block_id;
  // views into the caller's tmv_header (no copies: a light window converts
  // ~10^3 headers per call)
  ByteView last_commit_hash, data_hash, validators_hash, next_validators_hash, consensus_hash, app_hash,
      last_results_hash, evidence_hash, proposer_address;
};

struct SignedHeader {
  const Header *header = nullptr;
  const Commit *commit = nullptr;
};

// The 14 byte slices of Header.Hash (types/block.go:461-476), appended to
// `blob` with their end offsets in `off` (off must start with the blob's
// current size).
inline void AppendHeaderLeaves(const Header &h, Bytes &blob, std::vector<uint32_t> &off) {
  uint8_t tmp[16];
  auto end = [&]() { off.push_back((uint32_t)blob.size()); };
  auto put = [&](const uint8_t *p, size_t n) { blob.insert(blob.end(), p, p + n); };
  auto varint_field = [&](uint8_t tag, uint64_t v) {
    if (!v) return;
    tmp[0] = tag;
    put(tmp, (size_t)(PutUvarintP(tmp + 1, v) - tmp));
  };
  auto bytes_field = [&](uint8_t tag, const uint8_t *p, size_t n) {
    tmp[0] = tag;
    put(tmp, (size_t)(PutUvarintP(tmp + 1, n) - tmp));
    put(p, n);
  };
  auto cdc_bytes = [&](ByteView b) {  // gogotypes.BytesValue, nil when empty
    if (!b.empty()) bytes_field(0x0a, b.data(), b.size());
    end();
  };
  // version: tmversion.Consensus{block, app}
  varint_field(0x08, h.version_block);
  varint_field(0x10, h.version_app);
  end();
  // chain_id: StringValue
  if (!h.chain_id.empty()) bytes_field(0x0a, reinterpret_cast<const uint8_t *>(h.chain_id.data()), h.chain_id.size());
  end();
  // height: Int64Value (proto3 omits 0)
  varint_field(0x08, (uint64_t)h.height);
  end();
  // time: google.protobuf.Timestamp
  varint_field(0x08, (uint64_t)h.time.seconds);
  varint_field(0x10, (uint64_t)(int64_t)h.time.nanos);
  end();
  // last_block_id: tmproto.BlockID, part_set_header always present
  {
    const PartSetHeader &ph = h.last_block_id.part_set_header;
    size_t psh = 0;
    if (ph.total) psh += 1 + UvarintLen(ph.total);
    if (!ph.hash.empty()) psh += 1 + UvarintLen(ph.hash.size()) + ph.hash.size();
    if (!h.last_block_id.hash.empty()) bytes_field(0x0a, h.last_block_id.hash.data(), h.last_block_id.hash.size());
    tmp[0] = 0x12;
    put(tmp, (size_t)(PutUvarintP(tmp + 1, psh) - tmp));
    varint_field(0x08, ph.total);
    if (!ph.hash.empty()) bytes_field(0x12, ph.hash.data(), ph.hash.size());
  }
  end();
  cdc_bytes(h.last_commit_hash);
  cdc_bytes(h.data_hash);
  cdc_bytes(h.validators_hash);
  cdc_bytes(h.next_validators_hash);
  cdc_bytes(h.consensus_hash);
  cdc_bytes(h.app_hash);
  cdc_bytes(h.last_results_hash);
  cdc_bytes(h.evidence_hash);
  cdc_bytes(h.proposer_address);
}
constexpr uint32_t kHeaderLeaves = 14;

// ---------------------------------------------------------------- host merkle (few trees)
// crypto/merkle: leaf = SHA-256(0x00 || leaf), inner = SHA-256(0x01 || l || r),
// split at the largest power of two below n (tree.go:11-27,100-112); the
// engine's tmv_merkle_roots computes the same roots on the device.
inline void Sha256Bytes(uint32_t st[8], const uint8_t *pre, size_t pre_n, const uint8_t *p, size_t n) {
  tmv::sha256_init(st);
  const uint64_t total = pre_n + n;
  uint8_t blk[64];
  size_t fill = 0;
  auto feed = [&](const uint8_t *q, size_t m) {
    while (m) {
      const size_t c = std::min(m, 64 - fill);
      std::memcpy(blk + fill, q, c);
      fill += c;
      q += c;
      m -= c;
      if (fill == 64) {
        uint32_t w[16];
        for (int i = 0; i < 16; i++)
          w[i] = (uint32_t)blk[4 * i] << 24 | (uint32_t)blk[4 * i + 1] << 16 | (uint32_t)blk[4 * i + 2] << 8 |
                 blk[4 * i + 3];
        tmv::sha256_compress(st, w);
        fill = 0;
      }
    }
  };
  feed(pre, pre_n);
  feed(p, n);
  uint8_t pad[72] = {0x80};
  const size_t padn = (fill < 56 ? 56 - fill : 120 - fill);
  feed(pad, padn);
  uint8_t len[8];
  for (int i = 0; i < 8; i++) len[i] = (uint8_t)((total * 8) >> (56 - 8 * i));
  feed(len, 8);
}

struct Digest {
  uint32_t w[8];
};

inline Digest MerkleRootHostRange(const Digest *leaves, size_t n) {
  if (n == 1) return leaves[0];
  size_t k = 1;
  while (k * 2 < n) k *= 2;
  const Digest l = MerkleRootHostRange(leaves, k), r = MerkleRootHostRange(leaves + k, n - k);
  Digest o;
  tmv::sha256_inner(o.w, l.w, r.w);
  return o;
}

// HashFromByteSlices of the leaves [off[i], off[i+1]) of `blob`, i < n
inline void MerkleRootHost(const uint8_t *blob, const uint32_t *off, size_t n, uint8_t out[32]) {
  Digest root;
  if (n == 0) {
    Sha256Bytes(root.w, nullptr, 0, nullptr, 0);
  } else {
    std::vector<Digest> lv(n);
    static const uint8_t zero = 0;
    for (size_t i = 0; i < n; i++) Sha256Bytes(lv[i].w, &zero, 1, blob + off[i], off[i + 1] - off[i]);
    root = MerkleRootHostRange(lv.data(), n);
  }
  for (int i = 0; i < 8; i++)
    for (int b = 0; b < 4; b++) out[4 * i + b] = (uint8_t)(root.w[i] >> (24 - 8 * b));
}

inline Bytes HeaderHashHost(const Header &h) {
  if (h.validators_hash.empty()) return {};  // types/block.go:448-450
  Bytes blob;
  std::vector<uint32_t> off{0};
  AppendHeaderLeaves(h, blob, off);
  Bytes out(32);
  MerkleRootHost(blob.data(), off.data(), kHeaderLeaves, out.data());
  return out;
}

// ValidatorSet.Hash on the host (types/validator_set.go:344-350 over
// SimpleValidator bytes, types/validator.go:154-170).  PublicKey oneof
// (proto/tendermint/crypto/keys.proto): ed25519 = 1, secp256k1 = 2 (the only
// other key type of the reference, KeyType::Other here), sr25519 = 3.
inline Bytes ValidatorSetHashHost(const ValidatorSet &vs) {
  Bytes blob;
  std::vector<uint32_t> off{0};
  for (const Validator &v : vs.validators) {
    const uint8_t field = v.pub_key.type == KeyType::Sr25519 ? 0x1a : v.pub_key.type == KeyType::Other ? 0x12 : 0x0a;
    const size_t kl = v.pub_key.bytes.size();
    uint8_t tmp[16];
    blob.push_back(0x0a);
    uint8_t *p = PutUvarintP(tmp, 1 + UvarintLen(kl) + kl);
    blob.insert(blob.end(), tmp, p);
    blob.push_back(field);
    p = PutUvarintP(tmp, kl);
    blob.insert(blob.end(), tmp, p);
    blob.insert(blob.end(), v.pub_key.bytes.begin(), v.pub_key.bytes.end());
    if (v.voting_power) {
      blob.push_back(0x10);
      p = PutUvarintP(tmp, (uint64_t)v.voting_power);
      blob.insert(blob.end(), tmp, p);
    }
    off.push_back((uint32_t)blob.size());
  }
  Bytes out(32);
  MerkleRootHost(blob.data(), off.data(), vs.validators.size(), out.data());
  return out;
}

// ---------------------------------------------------------------- ValidateBasic
inline Error ValidateHash(ByteView h) {
  if (!h.empty() && h.size() != kHashSize)
    return "expected size to be " + std::to_string(kHashSize) + " bytes, got " + std::to_string(h.size()) + " bytes";
  return std::nullopt;
}

inline Error BlockIDValidateBasic(const BlockID &b) {
  if (Error e = ValidateHash(b.hash)) return "wrong Hash: " + *e;
  if (Error e = ValidateHash(b.part_set_header.hash)) return "wrong PartSetHeader: wrong Hash: " + *e;
  return std::nullopt;
}

inline Error HeaderValidateBasic(const Header &h) {
  if (h.version_block != kBlockProtocol)
    return "block protocol is incorrect: got: " + std::to_string(h.version_block) +
           ", want: " + std::to_string(kBlockProtocol) + " ";
  if (h.chain_id.size() > kMaxChainIDLen)
    return "chainID is too long; got: " + std::to_string(h.chain_id.size()) + ", max: " + std::to_string(kMaxChainIDLen);
  if (h.height < 0) return std::string("negative Height");
  if (h.height == 0) return std::string("zero Height");
  if (Error e = BlockIDValidateBasic(h.last_block_id)) return "wrong LastBlockID: " + *e;
  if (Error e = ValidateHash(h.last_commit_hash)) return "wrong LastCommitHash: " + *e;
  if (Error e = ValidateHash(h.data_hash)) return "wrong DataHash: " + *e;
  if (Error e = ValidateHash(h.evidence_hash)) return "wrong EvidenceHash: " + *e;
  if (h.proposer_address.size() != kAddressSize)
    return "invalid ProposerAddress length; got: " + std::to_string(h.proposer_address.size()) +
           ", expected: " + std::to_string(kAddressSize);
  if (Error e = ValidateHash(h.validators_hash)) return "wrong ValidatorsHash: " + *e;
  if (Error e = ValidateHash(h.next_validators_hash)) return "wrong NextValidatorsHash: " + *e;
  if (Error e = ValidateHash(h.consensus_hash)) return "wrong ConsensusHash: " + *e;
  if (Error e = ValidateHash(h.last_results_hash)) return "wrong LastResultsHash: " + *e;
  return std::nullopt;
}

inline Error CommitSigValidateBasic(const CommitSig &cs) {
  const int f = (int)cs.block_id_flag;
  if (f != BlockIDFlagAbsent && f != BlockIDFlagCommit && f != BlockIDFlagNil)
    return "unknown BlockIDFlag: " + std::to_string(f);
  if (f == BlockIDFlagAbsent) {
    if (!cs.validator_address.empty()) return std::string("validator address is present");
    if (!IsZeroTime(cs.timestamp)) return std::string("time is present");
    if (!cs.signature.empty()) return std::string("signature is present");
    return std::nullopt;
  }
  if (cs.validator_address.size() != kAddressSize)
    return "expected ValidatorAddress size to be " + std::to_string(kAddressSize) + " bytes, got " +
           std::to_string(cs.validator_address.size()) + " bytes";
  if (cs.signature.empty()) return std::string("signature is missing");
  if (cs.signature.size() > kMaxSignatureSize)
    return "signature is too big (max: " + std::to_string(kMaxSignatureSize) + ")";
  return std::nullopt;
}

inline Error CommitValidateBasic(const Commit &c) {
  if (c.height < 0) return std::string("negative Height");
  if (c.round < 0) return std::string("negative Round");
  if (c.height >= 1) {
    if (c.block_id.IsNil()) return std::string("commit cannot be for nil block");
    if (c.signatures.empty()) return std::string("no signatures in commit");
    for (size_t i = 0; i < c.signatures.size(); i++)
      if (Error e = CommitSigValidateBasic(c.signatures[i])) return "wrong CommitSig #" + std::to_string(i) + ": " + *e;
  }
  return std::nullopt;
}

// types/light.go:145-172; header_hash = Header.Hash() (empty = nil)
inline Error SignedHeaderValidateBasic(const SignedHeader &sh, const std::string &chain_id, const Bytes &header_hash) {
  if (!sh.header) return std::string("missing header");
  if (!sh.commit) return std::string("missing commit");
  if (Error e = HeaderValidateBasic(*sh.header)) return "invalid header: " + *e;
  if (Error e = CommitValidateBasic(*sh.commit)) return "invalid commit: " + *e;
  if (sh.header->chain_id != chain_id)
    return "header belongs to another chain " + GoQuote(sh.header->chain_id) + ", not " + GoQuote(chain_id);
  if (sh.commit->height != sh.header->height)
    return "header and commit height mismatch: " + std::to_string(sh.header->height) + " vs " +
           std::to_string(sh.commit->height);
  if (!(ByteView(header_hash) == ByteView(sh.commit->block_id.hash)))
    return "commit signs block " + HexUpper(sh.commit->block_id.hash) + ", header is block " + HexUpper(header_hash);
  return std::nullopt;
}

// ---------------------------------------------------------------- light/verifier.go
enum LightKind : int {
  kLightOk = 0,
  kLightInvalidHeader = 1,     // ErrInvalidHeader
  kLightOldHeaderExpired = 2,  // ErrOldHeaderExpired
  kLightCantTrust = 3,         // ErrNewValSetCantBeTrusted
  kLightOther = 4,             // errors.New / fmt.Errorf
};

struct LightResult {
  int kind = kLightOk;
  std::string text;
};

enum LightMode : int { kLightVerify = 0, kLightAdjacent = 1, kLightNonAdjacent = 2 };

struct LightJob {
  LightMode mode = kLightVerify;
  SignedHeader trusted;
  const ValidatorSet *trusted_vals = nullptr;  // trusted next validators (Verify / NonAdjacent)
  SignedHeader untrusted;
  const ValidatorSet *untrusted_vals = nullptr;
  int64_t trusting_period_ns = 0;
  Timestamp now;
  int64_t max_clock_drift_ns = 0;
  uint64_t trust_num = 1, trust_den = 3;
};

// One commit check a light job needs, and how its error maps (light/verifier.go:70-88,149-152).
struct LightCommitCheck {
  CommitVerifier::Mode mode;
  const ValidatorSet *vals;
  const Commit *commit;
  BlockID block_id;
  int64_t height;
  std::string chain_id;
  int64_t trust_num, trust_den;
};

// Everything before the signature checks; then 0-2 commit checks whose errors
// Finish maps in order.
struct LightPlan {
  std::optional<LightResult> early;
  std::vector<LightCommitCheck> checks;  // [trusting,] light
  bool first_is_trusting = false;
};

inline bool HeaderExpired(const Header &h, int64_t trusting_period_ns, const Timestamp &now) {
  return !(TimeNs(h.time) + trusting_period_ns > TimeNs(now));  // !expirationTime.After(now)
}

inline Error CheckRequiredHeaderFields(const SignedHeader &sh) {
  if (sh.header->height == 0) return std::string("height in trusted header must be set (non zero");
  if (IsZeroTime(sh.header->time)) return std::string("time in trusted header must be set");
  if (sh.header->chain_id.empty()) return std::string("chain ID in trusted header must be set");
  return std::nullopt;
}

inline Error ValidateTrustLevel(uint64_t num, uint64_t den) {
  if (num * 3 < den || num >= den || den == 0)
    return "trustLevel must be within [1/3, 1], given " + std::to_string(num) + "/" + std::to_string(den);
  return std::nullopt;
}

// hashes: Header.Hash of the untrusted header, ValidatorSet.Hash of untrusted_vals
inline Error VerifyNewHeaderAndVals(const LightJob &j, const Bytes &untrusted_header_hash,
                                    const Bytes &untrusted_vals_hash) {
  const Header &th = *j.trusted.header;
  if (Error e = SignedHeaderValidateBasic(j.untrusted, th.chain_id, untrusted_header_hash))
    return "untrustedHeader.ValidateBasic failed: " + *e;
  const Header &uh = *j.untrusted.header;
  if (uh.height <= th.height)
    return "expected new header height " + std::to_string(uh.height) + " to be greater than one of old header " +
           std::to_string(th.height);
  if (!(TimeNs(uh.time) > TimeNs(th.time)))
    return "expected new header time " + GoTime(uh.time) + " to be after old header time " + GoTime(th.time);
  if (!(TimeNs(uh.time) < TimeNs(j.now) + j.max_clock_drift_ns))
    return "new header has a time from the future " + GoTime(uh.time) + " (now: " + GoTime(j.now) +
           "; max clock drift: " + GoDuration(j.max_clock_drift_ns) + ")";
  if (!(ByteView(uh.validators_hash) == ByteView(untrusted_vals_hash)))
    return "expected new header validators (" + HexUpper(uh.validators_hash) + ") to match those that were supplied (" +
           HexUpper(untrusted_vals_hash) + ") at height " + std::to_string(uh.height);
  return std::nullopt;
}

inline LightResult Expired(const LightJob &j) {
  const Timestamp at = FromNs(TimeNs(j.untrusted.header->time) + j.trusting_period_ns);
  return LightResult{kLightOldHeaderExpired, "old header has expired at " + GoTime(at) + " (now: " + GoTime(j.now) + ")"};
}

inline LightPlan PlanLight(const LightJob &j, const Bytes &untrusted_header_hash, const Bytes &untrusted_vals_hash) {
  LightPlan p;
  auto other = [&](const std::string &s) { p.early = LightResult{kLightOther, s}; };
  if (!j.trusted.header || !j.untrusted.header) { other("missing header"); return p; }
  const Header &th = *j.trusted.header, &uh = *j.untrusted.header;
  LightMode mode = j.mode;
  if (mode == kLightVerify) mode = uh.height != th.height + 1 ? kLightNonAdjacent : kLightAdjacent;
  if (Error e = CheckRequiredHeaderFields(j.trusted)) { other(*e); return p; }
  if (mode == kLightNonAdjacent) {
    if (uh.height == th.height + 1) { other("headers must be non adjacent in height"); return p; }
    if (Error e = ValidateTrustLevel(j.trust_num, j.trust_den)) { other(*e); return p; }
  } else {
    if (th.next_validators_hash.empty()) { other("next validators hash in trusted header is empty"); return p; }
    if (uh.height != th.height + 1) { other("headers must be adjacent in height"); return p; }
  }
  if (HeaderExpired(uh, j.trusting_period_ns, j.now)) { p.early = Expired(j); return p; }
  if (!j.untrusted_vals) { p.early = LightResult{kLightInvalidHeader, "invalid header: nil validator set"}; return p; }
  if (Error e = VerifyNewHeaderAndVals(j, untrusted_header_hash, untrusted_vals_hash)) {
    p.early = LightResult{kLightInvalidHeader, "invalid header: " + *e};
    return p;
  }
  if (mode == kLightAdjacent && !(ByteView(uh.validators_hash) == ByteView(th.next_validators_hash))) {
    p.early = LightResult{kLightInvalidHeader, "invalid header: expected old header's next validators (" +
                                                   HexUpper(th.next_validators_hash) +
                                                   ") to match those from new header (" + HexUpper(uh.validators_hash) +
                                                   ")"};
    return p;
  }
  const Commit *c = j.untrusted.commit;
  if (mode == kLightNonAdjacent) {
    p.first_is_trusting = true;
    p.checks.push_back(LightCommitCheck{CommitVerifier::kLightTrusting, j.trusted_vals, c, BlockID{}, 0, th.chain_id,
                                        (int64_t)j.trust_num, (int64_t)j.trust_den});
  }
  p.checks.push_back(
      LightCommitCheck{CommitVerifier::kLight, j.untrusted_vals, c, c->block_id, uh.height, th.chain_id, 0, 1});
  return p;
}

// errs[i] / not_enough[i]: result of checks[i] (not_enough = the error is
// types.ErrNotEnoughVotingPowerSigned)
inline LightResult FinishLight(const LightPlan &p, const Error *errs, const bool *not_enough) {
  if (p.early) return *p.early;
  for (size_t i = 0; i < p.checks.size(); i++) {
    if (!errs[i]) continue;
    if (i == 0 && p.first_is_trusting && not_enough[i])
      return LightResult{kLightCantTrust, "cant trust new val set: " + *errs[i]};
    return LightResult{kLightInvalidHeader, "invalid header: " + *errs[i]};
  }
  return LightResult{};
}

}  // namespace tmh
