"""BASELINE C3 at its configured size on the MI355X: light.Client sequential
verification of 10,000 headers x 100 validators (light/helpers_test.go:165-216
shape, light/client.go:567-626), 1.0 M commit signatures, every one checked
against the C oracle (tests/at_size.py states the three checks)."""
import random

import pytest

import at_size as A
import chain_fixtures as CF
import light_ref as L
from tendermint_amd import chains, host as H
from tendermint_amd.testing.factory import make_light_chain

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def c3(ctx):
    """The chain verified clean, then with its seeded corruptions: the
    oracle's vector of every vote and the oracle's VerifyAdjacent result of
    every header."""
    trusted, blocks, pv = make_light_chain(A.C3_HEADERS, A.C3_VALS, packed=True)
    now = (blocks[-1].signed_header.header.time[0] + 5, 0)
    clean = chains.verify_sequential(ctx, trusted, blocks, A.PERIOD, now, A.DRIFT, window=1000)
    rng = random.Random(0xC3)
    # commit c of the packed votes is light block c (c = 0: the trusted block)
    picks = sorted(rng.sample(range(1, A.C3_HEADERS + 1), 60))
    blocks_c = list(blocks)
    for n_pick, c in enumerate(picks):
        i = rng.randrange(A.C3_VALS)
        A.corrupt_sig(blocks_c[c - 1].signed_header.commit, i, pv, int(pv.commit_off[c]) + i, rng,
                      s_plus_l=(n_pick % 10 == 0))
    tampered = min(picks[len(picks) // 2] + 3, A.C3_HEADERS)  # its hash no longer matches its commit
    blocks_c[tampered - 1].signed_header.header.app_hash = b"tampered"
    A.progress("C3: chain generated and verified clean")
    vec = A.oracle_vector(pv)
    A.progress("C3: oracle vector")
    conv = CF.OracleBlocks()
    now_ns = now[0] * L.NS + now[1]
    want = []
    with L.signature_oracle(A.Verdicts(pv, vec)):
        prev = conv(trusted)
        for lb in blocks_c:
            cur = conv(lb)
            e = L.verify_adjacent(prev.signed_header, cur.signed_header, cur.vals, A.PERIOD, now_ns, A.DRIFT)
            want.append((L.OK, None) if e is None else (e.kind, e.text))
            prev = cur
    A.progress("C3: oracle results of every job")
    return dict(trusted=trusted, blocks=blocks_c, pv=pv, now=now, picks=picks, tampered=tampered, vec=vec,
                want=want, clean=clean)


def test_c3_clean_chain_verifies(c3):
    """The uncorrupted 10,000-header chain verifies end to end (windows of
    1,000 headers through the sequential driver)."""
    assert c3["clean"] == (A.C3_HEADERS, None)


def test_c3_signature_vector_vs_oracle(ctx, c3):
    """Every vote of every window through the key-cached batch path equals
    the oracle's vector (60 invalid of 1,000,100)."""
    assert int((~c3["vec"].astype(bool)).sum()) == len(c3["picks"])
    A.engine_vector_check(ctx, c3["pv"], c3["vec"], 1000)


def test_c3_every_header_vs_oracle(ctx, c3):
    """tmv_light_verify_many over windows of 1,000 headers: every
    VerifyAdjacent result (class and text) equals the oracle's."""
    got, prev = [], c3["trusted"]
    for lo in range(0, A.C3_HEADERS, 1000):
        jobs = []
        for lb in c3["blocks"][lo:lo + 1000]:
            jobs.append(H.LightJob(prev.signed_header, None, lb.signed_header, lb.vals, A.PERIOD, c3["now"], A.DRIFT,
                                   mode=H.LIGHT_ADJACENT))
            prev = lb
        got += H.light_verify_many(ctx, jobs)
    want = c3["want"]
    diff = [h for h, (g, w) in enumerate(zip(got, want)) if g != w]
    assert not diff, f"headers {diff[:5]}: engine {[got[h] for h in diff[:2]]} vs oracle {[want[h] for h in diff[:2]]}"
    failing = [h for h, w in enumerate(want) if w[0] != L.OK]
    # the tampered header fails; flips outside the 2/3 prefix pass, as in the reference
    assert c3["tampered"] - 1 in failing and 10 <= len(failing) < len(c3["picks"]) + 1


def test_c3_sequential_driver_first_error(ctx, c3):
    """chains.verify_sequential over all 10,000 headers stops at the header
    and with the error of the one-at-a-time loop (light/client.go:567-626)."""
    want, blocks, trusted = c3["want"], c3["blocks"], c3["trusted"]
    first = next(h for h, w in enumerate(want) if w[0] != L.OK)
    n, err = chains.verify_sequential(ctx, trusted, blocks, A.PERIOD, c3["now"], A.DRIFT, window=1000)
    assert n == first
    assert (err.from_height, err.to_height, err.kind, err.reason) == \
        (blocks[first - 1].height if first else trusted.height, blocks[first].height) + want[first]
