"""Light-client verification through libtmgpu.so on the MI355X
(tmv_light_verify_many, tmv_header_hashes, tmv_merkle_roots): the
reference's own model-based fixtures (light/mbt/json, driver_test.go:18-86)
and mutations of them, against the oracle (oracle/light_ref.py)."""
import json
import random

import pytest

import light_ref as L
import mbt_fixtures as M
from tendermint_amd import host as H

pytestmark = pytest.mark.gpu

CASES = M.load_cases()
HOST_CASES = M.load_host_cases()


@pytest.mark.parametrize("i", range(len(CASES)), ids=[c["file"].rsplit("/", 1)[1] for c in CASES])
def test_mbt_verdicts(ctx, i):
    """driver_test.go's loop through tmv_light_verify: each input's class is
    the fixture's verdict and class + text equal the oracle's."""
    want = [(L.OK, None) if r is None else (r.kind, r.text) for _, r in M.run_driver(CASES[i], L.verify)]
    got = []
    for inp, r in M.run_host_driver(HOST_CASES[i], lambda jobs: H.light_verify_many(ctx, jobs)):
        got.append(r)
        assert r[0] in M.VERDICT_KIND[inp["verdict"]], (inp["verdict"], r)
    assert got == want


def test_mbt_header_hashes_device(ctx):
    """Header.Hash of the 39 fixture headers on the device (one
    tmv_merkle_roots launch) = the BlockID each commit signs."""
    hs = [c["trusted"] for c in HOST_CASES] + [i["signed_header"] for c in HOST_CASES for i in c["inputs"]]
    assert len(hs) >= 32  # above TMV_DEVICE_HASH_MIN
    assert H.header_hashes(ctx, [s.header for s in hs]) == [s.commit.block_id.hash for s in hs]


def test_header_hashes_random_vs_oracle(ctx):
    """2,000 random headers (chain IDs up to 50 bytes, long app hashes: leaves
    of 1-3 SHA-256 blocks, nil and empty fields) vs the oracle's Header.Hash."""
    rng = random.Random(3)
    hosts, oracles = [], []
    for i in range(2000):
        rb = lambda n: bytes(rng.randrange(256) for _ in range(n))  # noqa: E731
        d = dict(chain_id="c" * rng.randrange(0, 51), height=rng.choice([0, 1, rng.randrange(1, 1 << 62)]),
                 time_ns=rng.randrange(-10**18, 10**18), last_commit_hash=rb(rng.choice([0, 32])),
                 data_hash=rb(rng.choice([0, 32])), validators_hash=rb(rng.choice([32, 32, 0])),
                 next_validators_hash=rb(32), consensus_hash=rb(32), app_hash=rb(rng.choice([0, 8, 32, 100, 200])),
                 last_results_hash=rb(rng.choice([0, 32])), evidence_hash=rb(rng.choice([0, 32])),
                 proposer_address=rb(20))
        lb = L.BlockID(rb(rng.choice([0, 32])), rng.choice([0, 1, 300]), rb(rng.choice([0, 32])))
        vb, va = rng.choice([(11, 0), (11, 1), (0, 0), (300, 1 << 40)])
        o = L.Header(version_block=vb, version_app=va, last_block_id=lb, **d)
        t = divmod(d["time_ns"], L.NS)
        hd = {k: v for k, v in d.items() if k != "time_ns"}
        hosts.append(H.Header(time=t, last_block_id=H.BlockID(lb.hash, lb.psh_total, lb.psh_hash), version_block=vb,
                              version_app=va, **hd))
        oracles.append(o)
    assert H.header_hashes(ctx, hosts) == [L.header_hash(o) for o in oracles]


def test_mutations_vs_oracle(ctx):
    """The CPU suite's 300 fixture mutations (tests/test_light_mbt.py), sent
    as ONE tmv_light_verify_many window, class and text equal to the oracle."""
    from test_light_mbt import _mutations
    rng = random.Random(1234)
    with open(M.GOLDEN) as f:
        raw = json.load(f)["cases"]
    jobs, want = [], []
    for _ in range(300):
        cj = raw[rng.randrange(len(raw))]
        ij = cj["input"][rng.randrange(len(cj["input"]))]
        t, tv, u, uv, now, period, drift, trust, mode = _mutations(rng, cj, ij)
        now_ns = now[0] * L.NS + now[1]
        if mode == 0:
            r = L.verify(M.signed_header(t), M.valset(tv), M.signed_header(u), M.valset(uv), period, now_ns, drift,
                         trust)
        elif mode == 1:
            r = L.verify_adjacent(M.signed_header(t), M.signed_header(u), M.valset(uv), period, now_ns, drift)
        else:
            r = L.verify_non_adjacent(M.signed_header(t), M.valset(tv), M.signed_header(u), M.valset(uv), period,
                                      now_ns, drift, trust)
        want.append((L.OK, None) if r is None else (r.kind, r.text))
        jobs.append(H.LightJob(M.host_signed_header(t), M.host_valset(tv), M.host_signed_header(u),
                               M.host_valset(uv), period, tuple(now), drift, trust, mode))
    assert H.light_verify_many(ctx, jobs) == want
