// Vote sign-bytes from a per-commit template (tmv_verify_votes, SURVEY
// §8(f) rank 1).  Commit.VoteSignBytes (types/block.go:836-862) over
// CanonicalizeVote (types/canonical.go:52-63) differs between the votes of
// one commit only in field 5 (the timestamp) and in whether field 4 (the
// BlockID) is present, so a vote's message is
//   uvarint(len(body)) || head || [block] || 0x2a uvarint(len(ts)) ts || chain
// with ts = [0x08 uvarint(seconds)] [0x10 uvarint(nanos)] (proto3 omits zero
// fields; negative values are 10-byte varints of the sign-extended value).
// The same length functions size the messages on the host (offsets) and on
// the device (k_vote_signbytes), so the two cannot disagree.
#pragma once
#include <cstdint>
#include "curve25519.h"
#include "../../include/tmverify.h"

namespace tmv {

// Device copy of a template: byte ranges into the template blob.
struct VoteTab {
  uint32_t head_at, head_len, block_at, block_len, chain_at, chain_len;
};

TMV_HD uint32_t uvarint_len(uint64_t x) {
  uint32_t n = 1;
  while (x >= 0x80) { x >>= 7; n++; }
  return n;
}

TMV_HD uint32_t vote_ts_inner(int64_t secs, int32_t nanos) {
  return (secs != 0 ? 1 + uvarint_len((uint64_t)secs) : 0) +
         (nanos != 0 ? 1 + uvarint_len((uint64_t)(int64_t)nanos) : 0);
}

TMV_HD uint32_t vote_body_len(const VoteTab &t, const tmv_vote &v) {
  const uint32_t ts = vote_ts_inner(v.ts_seconds, v.ts_nanos);
  return t.head_len + ((v.tmpl & TMV_VOTE_WITH_BLOCK) ? t.block_len : 0) + 1 + uvarint_len(ts) + ts + t.chain_len;
}

TMV_HD uint32_t vote_msg_len(const VoteTab &t, const tmv_vote &v) {
  const uint32_t body = vote_body_len(t, v);
  return uvarint_len(body) + body;
}

}  // namespace tmv
