"""Synthetic workload generator (C1/C2 shapes)."""
import collections

from tendermint_amd.testing.factory import make_c2_batch, make_commit_batch


def test_c2_composition():
    b = make_c2_batch()
    c = collections.Counter(b.kinds)
    assert b.n == 10_000 and c["honest"] == 9900
    assert (c["bitflip"], c["s_plus_l"], c["undecodable"], c["small_order"], c["noncanonical_y"],
            c["neg_zero"]) == (20, 15, 15, 20, 15, 15)
    lens = b.off[1:] - b.off[:-1]
    assert lens.min() >= 100 and lens.max() <= 130


def test_commit_batch_shape():
    b = make_commit_batch(150)
    assert b.n == 150
    lens = b.off[1:] - b.off[:-1]
    assert 109 <= lens.min() and lens.max() <= 125


def test_bulk_messages_and_signatures_match_per_vote_path():
    """bulk.vote_messages == commit_vote_message for every vote (zero /
    negative seconds, zero / large nanos, empty chain id), and the factory's
    own RFC 8032 signer == OpenSSL's == the per-signature signer."""
    import random

    import numpy as np

    from tendermint_amd.testing import bulk
    from tendermint_amd.testing._openssl import Ed25519Signer
    from tendermint_amd.testing.factory import commit_vote_message, key_seed, random_block_id

    rng = random.Random(5)
    bid = random_block_id(rng)
    secs = [0, -62135596800, 1577836800, 1 << 40, 7] + [1577836800 + rng.randrange(1 << 24) for _ in range(59)]
    nanos = [0, 0, 999_999_999, 1, 0] + [rng.randrange(10**9) for _ in range(59)]
    for chain, height, rnd in (("test_chain_id", 3, 0), ("", 1, 2), ("x" * 50, (1 << 62) + 5, 1 << 30)):
        m, o = bulk.vote_messages(bulk.commit_vote_head(height, rnd, bid), chain, secs, nanos)
        for i in range(len(secs)):
            assert m[o[i]:o[i + 1]].tobytes() == commit_vote_message(chain, height, rnd, bid, secs[i], nanos[i])
    seeds = [key_seed(i, "bulk") for i in range(7)]
    ki = np.array([rng.randrange(7) for _ in range(len(secs))], np.uint32)
    fast = bulk.sign_many(seeds, ki, m, o)
    ossl = bulk.sign_many(seeds, ki, m, o, openssl=True)
    assert np.array_equal(fast, ossl)
    signers = [Ed25519Signer(s) for s in seeds]
    assert bulk.public_keys(seeds) == [s.public_key for s in signers]
    for i in range(len(secs)):
        assert fast[64 * i:64 * i + 64].tobytes() == signers[ki[i]].sign(m[o[i]:o[i + 1]].tobytes())


def test_chain_generators_pack_every_vote():
    """make_light_chain / make_block_chain(packed=True): commit c's votes are
    the packed entries [commit_off[c], commit_off[c+1]) -- same signatures,
    keys and sign-bytes as the commit objects."""
    from tendermint_amd.testing.factory import commit_vote_message, make_block_chain, make_light_chain
    from tendermint_amd.types.canonical import BlockID, PartSetHeader

    trusted, blocks, pv = make_light_chain(6, 5, rotate=2, packed=True)
    vals_by_commit = [trusted.vals] + [b.vals for b in blocks]
    commits = [trusted.signed_header.commit] + [b.signed_header.commit for b in blocks]
    _, bblocks, bpv = make_block_chain(5, 4, packed=True)
    bvals = _
    for pvx, cms, vsets in ((pv, commits, vals_by_commit),
                            (bpv, [b.last_commit for b in bblocks[1:]], [bvals] * 4)):
        for c, (cm, vs) in enumerate(zip(cms, vsets)):
            lo = int(pvx.commit_off[c])
            bid = BlockID(cm.block_id.hash, PartSetHeader(cm.block_id.psh_total, cm.block_id.psh_hash))
            for i, s in enumerate(cm.signatures):
                pk, msg, sig = pvx.batch.entry(lo + i)
                assert sig == s.signature and pk == vs.validators[i].pub_key
                chain = "test" if pvx is pv else "test_chain_id"
                assert msg == commit_vote_message(chain, cm.height, cm.round, bid, *s.timestamp)
