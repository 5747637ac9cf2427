"""The reference's own model-based light-client fixtures
(light/mbt/json/*.json, light/mbt/driver_test.go:18-86) pin the oracle:
real ed25519 commit signatures, header hashes, validator-set hashes and the
expected light.Verify verdicts.  The GPU path is checked against the same
data in tests/test_gpu_light.py."""
import pytest

import light_ref as L
import mbt_fixtures as M

CASES = M.load_cases()


def _signed_headers():
    for c in CASES:
        yield c["file"], c["trusted"]
        for i, inp in enumerate(c["inputs"]):
            yield f"{c['file']}#{i}", inp["signed_header"]


def test_fixture_shape():
    assert len(CASES) == 9
    assert sum(len(c["inputs"]) for c in CASES) == 30
    assert {inp["verdict"] for c in CASES for inp in c["inputs"]} == {"SUCCESS", "NOT_ENOUGH_TRUST", "INVALID"}


def test_header_hash_equals_commit_block_id():
    """Header.Hash (types/block.go:447-478) of every fixture header is the
    BlockID its commit signs (SignedHeader.ValidateBasic, types/light.go:168)."""
    n = 0
    for name, sh in _signed_headers():
        assert L.header_hash(sh.header) == sh.commit.block_id.hash, name
        n += 1
    assert n == 39


def test_validator_set_hashes():
    """ValidatorSet.Hash of every supplied set equals the header's
    validators_hash / next_validators_hash (light/verifier.go:266)."""
    n = 0
    for c in CASES:
        assert c["trusted_next_vals"].hash() == c["trusted"].header.next_validators_hash
        n += 1
        for inp in c["inputs"]:
            h = inp["signed_header"].header
            assert inp["vals"].hash() == h.validators_hash
            assert inp["next_vals"].hash() == h.next_validators_hash
            n += 2
    assert n == 69


def test_signatures_verify():
    """Every Commit-flag signature by a member of the header's own validator
    set verifies under the oracle (ZIP-215) over the canonical vote sign-bytes."""
    n = 0
    for c in CASES:
        for inp in c["inputs"]:
            sh, vals = inp["signed_header"], inp["vals"]
            for cs in sh.commit.signatures:
                if cs.flag != L.FLAG_COMMIT:
                    continue
                _, v = vals.get_by_address(cs.address)
                if v is None:
                    continue
                msg = L.vote_sign_bytes(sh.header.chain_id, sh.commit.height, sh.commit.round, sh.commit.block_id,
                                        cs.ts_ns)
                assert L._verify_sig(v, msg, cs.signature)
                n += 1
    assert n >= 40


@pytest.mark.parametrize("case", CASES, ids=[c["file"].rsplit("/", 1)[1] for c in CASES])
def test_oracle_reproduces_verdicts(case):
    """light.Verify restated (oracle/light_ref.py) returns the fixture's
    verdict class for every input (driver_test.go:62-78)."""
    for inp, r in M.run_driver(case, L.verify):
        kind = L.OK if r is None else r.kind
        assert kind in M.VERDICT_KIND[inp["verdict"]], (inp["verdict"], r)


def test_go_formatting():
    assert L.go_time(0) == "1970-01-01 00:00:00 +0000 UTC"
    assert L.go_time(1405 * L.NS) == "1970-01-01 00:23:25 +0000 UTC"
    assert L.go_time(1603270053 * L.NS + 160327005) == "2020-10-21 08:47:33.160327005 +0000 UTC"
    assert L.go_time(1500) == "1970-01-01 00:00:00.0000015 +0000 UTC"
    for d, s in [(0, "0s"), (1, "1ns"), (1100, "1.1µs"), (2_200_000, "2.2ms"), (10**9, "1s"),
                 (3_500_000_000, "3.5s"), (60 * 10**9, "1m0s"), (3600 * 10**9, "1h0m0s"),
                 (1400 * 10**9, "23m20s"), (-1500 * 10**6, "-1.5s"), (90061 * 10**9 + 5, "25h1m1.000000005s")]:
        assert L.go_duration(d) == s, (d, s)
    assert L.go_quote('a"b\\c') == '"a\\"b\\\\c"'


# ---------------------------------------------------------------- product host layer (C++) on the CPU
# tests/native/commit_check.cpp runs tm_light_abi.cpp / tm_types.h with the
# device entry points replaced by host doubles whose signature checks are the
# C oracle's (real ed25519), so the reference's own signed fixtures exercise
# the product's light-client code here; tests/test_gpu_light.py runs the same
# data through libtmgpu.so on the MI355X.
HOST_CASES = M.load_host_cases()


@pytest.fixture(scope="module")
def fake_real():
    import commit_fixtures as F
    fb = F.FakeBackend()
    fb.real_signatures(True)
    yield fb
    fb.real_signatures(False)


def _oracle_results(case):
    return [(L.OK, None) if r is None else (r.kind, r.text) for _, r in M.run_driver(case, L.verify)]


@pytest.mark.parametrize("i", range(len(CASES)), ids=[c["file"].rsplit("/", 1)[1] for c in CASES])
def test_host_layer_matches_oracle(fake_real, i):
    """tmv_light_verify_many (C++) == the oracle, class and text, on every input;
    the class is the fixture's verdict."""
    got = [r for _, r in M.run_host_driver(HOST_CASES[i], fake_real.light_verify_many)]
    assert got == _oracle_results(CASES[i])
    for inp, (kind, _) in zip(HOST_CASES[i]["inputs"], got):
        assert kind in M.VERDICT_KIND[inp["verdict"]]


def test_host_header_hashes(fake_real):
    """tmv_header_hashes on the 39 fixture headers (host path below the device
    threshold, device double above it) equals the commits' BlockID hashes."""
    hs = [c["trusted"].header for c in HOST_CASES] + [i["signed_header"].header for c in HOST_CASES
                                                      for i in c["inputs"]]
    want = [c["trusted"].commit.block_id.hash for c in HOST_CASES] + \
           [i["signed_header"].commit.block_id.hash for c in HOST_CASES for i in c["inputs"]]
    assert fake_real.header_hashes(hs) == want          # 39 >= 32: tmv_merkle_roots
    assert fake_real.header_hashes(hs[:5]) == want[:5]  # host merkle
    from tendermint_amd import host as H
    nil = H.Header(chain_id="x", height=1, time=(0, 0))
    assert fake_real.header_hashes([nil]) == [None]


def test_go_formatting_cpp(fake_real):
    import ctypes
    Lc = fake_real.L
    Lc.commitcheck_go_format.argtypes = [ctypes.c_int, ctypes.c_int64, ctypes.c_int32, ctypes.c_char_p,
                                         ctypes.c_size_t]
    buf = ctypes.create_string_buffer(128)
    for t in [0, 1405 * L.NS, 1603270053 * L.NS + 160327005, 1500, -62135596800 * L.NS]:
        Lc.commitcheck_go_format(0, t // L.NS, t % L.NS, buf, 128)
        assert buf.value.decode() == L.go_time(t)
    for d in [0, 1, 1100, 2_200_000, 10**9, 3_500_000_000, 60 * 10**9, 3600 * 10**9, 1400 * 10**9, -1500 * 10**6,
              90061 * 10**9 + 5]:
        Lc.commitcheck_go_format(1, d, 0, buf, 128)
        assert buf.value.decode("utf-8") == L.go_duration(d)
    for s in ['a"b\\c', "tab\there", "plain-chain_1"]:
        b = ctypes.create_string_buffer(s.encode(), 128)
        Lc.commitcheck_go_format(2, 0, 0, b, 128)
        assert b.value.decode() == L.go_quote(s)


def _mutations(rng, case_json, inp_json):
    """One random mutation of (trusted, trusted next vals, untrusted, vals,
    now, trusting period, drift, trust, mode) as JSON-level dicts."""
    import copy
    t = copy.deepcopy(case_json["initial"]["signed_header"])
    tv = copy.deepcopy(case_json["initial"]["next_validator_set"])
    u = copy.deepcopy(inp_json["signed_header"])
    uv = copy.deepcopy(inp_json["validator_set"])
    now = list(inp_json["now"])
    period = case_json["initial"]["trusting_period_ns"]
    drift, trust, mode = M.MAX_CLOCK_DRIFT_NS, (1, 3), 0
    h, c = u["header"], u["commit"]
    k = rng.randrange(30)
    if k == 0: h["version_block"] = 10
    elif k == 1: h["chain_id"] = rng.choice(["other", "", "x" * 51, 'q"uote'])
    elif k == 2: h["height"] += rng.choice([-5, -1, 1, 7])
    elif k == 3: c["height"] += 1
    elif k == 4: h["time"][0] += rng.choice([-10**6, -1, 1, 10**6])
    elif k == 5:
        f = rng.choice(["last_commit_hash", "data_hash", "validators_hash", "next_validators_hash", "consensus_hash",
                        "last_results_hash", "evidence_hash"])
        h[f] = rng.choice(["", "ab" * 31, "cd" * 33, "ee" * 32])
    elif k == 6: h["proposer_address"] = rng.choice(["", "11" * 19, "22" * 21])
    elif k == 7: h["last_block_id"]["hash"] = "ab" * 31
    elif k == 8: h["last_block_id"]["psh_hash"] = "cd" * 5
    elif k == 9: c["round"] = -1
    elif k == 10: c["block_id"] = {"hash": "", "psh_total": 0, "psh_hash": ""}
    elif k == 11: c["signatures"] = []
    elif k == 12: c["signatures"][rng.randrange(len(c["signatures"]))]["flag"] = rng.choice([0, 4, 7])
    elif k == 13:
        s = c["signatures"][rng.randrange(len(c["signatures"]))]
        s["flag"] = 1
        if rng.random() < 0.5: s["signature"] = ""; s["time"] = [-62135596800, 0]
    elif k == 14: c["signatures"][rng.randrange(len(c["signatures"]))]["signature"] = ""
    elif k == 15: c["signatures"][rng.randrange(len(c["signatures"]))]["signature"] += "00"
    elif k == 16:
        full = [s for s in c["signatures"] if len(s["signature"]) == 128]
        if full:
            s = rng.choice(full)
            b = bytearray.fromhex(s["signature"]); b[rng.randrange(64)] ^= 1 << rng.randrange(8)
            s["signature"] = b.hex()
    elif k == 17: c["signatures"][rng.randrange(len(c["signatures"]))]["address"] = "33" * 19
    elif k == 18:
        if uv: uv.pop(rng.randrange(len(uv)))
    elif k == 19:
        if uv: uv[rng.randrange(len(uv))]["voting_power"] += 1
    elif k == 20: now[0] += rng.choice([-10**7, -5, 5, 10**9])
    elif k == 21: period = rng.choice([1, 10**9, 10**18])
    elif k == 22: drift = rng.choice([0, 1, 5 * 10**9, 3_600_000_000_123])
    elif k == 23: trust = rng.choice([(1, 4), (2, 3), (1, 1), (1, 0), (9, 10)])
    elif k == 24: mode = rng.choice([1, 2])
    elif k == 25: t["header"]["height"] = 0
    elif k == 26: t["header"]["time"] = [-62135596800, 0]
    elif k == 27: t["header"]["chain_id"] = ""
    elif k == 28: t["header"]["next_validators_hash"] = ""; mode = 1
    elif k == 29:  # sign bytes of another vote: the flag Nil keeps the signature but changes the message
        c["signatures"][rng.randrange(len(c["signatures"]))]["flag"] = 3
    return t, tv, u, uv, now, period, drift, trust, mode


def test_host_layer_mutations_match_oracle(fake_real):
    """Differential check over every error branch light/verifier.go and
    types/{block,light,validation}.go can take: 300 random mutations of the
    fixture inputs, C++ host layer vs the oracle, class and text."""
    import json
    import random
    from tendermint_amd import host as H
    rng = random.Random(1234)
    with open(M.GOLDEN) as f:
        raw = json.load(f)["cases"]
    seen = set()
    for it in range(300):
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
        want = (L.OK, None) if r is None else (r.kind, r.text)
        job = H.LightJob(M.host_signed_header(t), M.host_valset(tv), M.host_signed_header(u), M.host_valset(uv),
                         period, tuple(now), drift, trust, mode)
        got = fake_real.light_verify_many([job])[0]
        assert got == want, (it, got, want)
        seen.add(" ".join(want[1].split()[:5]) if want[1] else "ok")
    assert len(seen) >= 15, seen


@pytest.mark.parametrize("slice_jobs", ["0", "7"])
def test_host_layer_many_equals_single(fake_real, slice_jobs, monkeypatch):
    """A window of jobs in one tmv_light_verify_many call (shared headers and
    sets, one signature batch) returns what each job returns alone -- in one
    pass and in pipelined slices of 7 jobs on two threads (TMV_HOST_SLICE)."""
    monkeypatch.setenv("TMV_HOST_SLICE", slice_jobs)
    from tendermint_amd import host as H
    jobs = []
    for c in HOST_CASES:
        for inp in c["inputs"]:
            jobs.append(H.LightJob(c["trusted"], c["trusted_next_vals"], inp["signed_header"], inp["vals"],
                                   c["trusting_period_ns"], inp["now"], M.MAX_CLOCK_DRIFT_NS, M.TRUST_LEVEL))
    many = fake_real.light_verify_many(jobs * 2)
    single = [fake_real.light_verify_many([j])[0] for j in jobs]
    assert many == single * 2
