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
